// PM-RoPE + KV-cache store, and GQA attention (decode / prefill / encoder / cross).
//
// RoPE follows [tf] T5GemmaRotaryEmbedding + apply_rotary_pos_emb with FLOAT
// progress positions (hf_export/modeling_t5gemma_voice.py:516-531, 669-681,
// 817-832): angle = inv_freq[i] * pos in fp32, cos/sin rounded to bf16, then
// out = bf16(bf16(x*cos) + bf16(rotate_half(x)*sin)) -- three bf16 tensor ops.
//
// Attention: one block per (query, kv head, key split); the G = Hq/Hkv query
// heads of a GQA group share every K/V row read (GQA reuse). K/V cache rows are
// read with 16-byte lanes, LPK = D/8 lanes per key (32 at D = 256: two keys per
// wave instruction, a contiguous 1 KiB). Numerics mirror torch's CPU SDPA flash
// kernel (fp32 scores, fp32 exp and sum, exp values rounded to bf16 before P.V,
// O / sum rounded once); ``eager`` mirrors eager_attention_forward (bf16 scores,
// tanh softcap, bf16-rounded normalised probabilities).
#include "common.h"
#include "exact_math.h"
#include "t5g_kernels.h"

namespace t5g {

typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

T5G_TS_UNIT(attn)

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rope_store_kernel(RopeArgs a) {
    // grid: (token, pair-block); thread = one (head, i) rotation pair (i, i + D/2)
    const int m = blockIdx.x;
    const int D = a.D, H2 = D / 2;
    const int nh = a.nq + a.nk + a.nv;
    const int idx = blockIdx.y * blockDim.x + threadIdx.x;
    if (idx >= nh * H2) return;
    const int h = idx / H2, i = idx % H2;
    const int row = a.tok_row ? a.tok_row[m] : m;
    const bool isq = h < a.nq, isk = !isq && h < a.nq + a.nk;
    const int slot = isq ? 0 : (a.tok_t ? a.tok_t[m] : a.kv_len[row] - 1);   // issued first
    float x1, x2;
    if (a.Xpart) {
        float p1[8], p2[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) {   // clamped, unconditional (see attn_decode_kernel)
            const float* ps = a.Xpart + ((long)min(s, a.nsplit - 1) * a.M + m) * a.ldx + a.col0 + h * D;
            p1[s] = ps[i];
            p2[s] = ps[i + H2];
        }
        x1 = p1[0];
        x2 = p2[0];
#pragma unroll
        for (int s = 1; s < 8; ++s)
            if (s < a.nsplit) {
                x1 += p1[s];
                x2 += p2[s];
            }
        x1 = rbf(x1);
        x2 = rbf(x2);
    } else {
        const bf16_t* xh = a.X + (long)m * a.ldx + a.col0 + h * D;
        x1 = bf2f(xh[i]);
        x2 = bf2f(xh[i + H2]);
    }
    float o1 = x1, o2 = x2;
    if ((isq && a.rope_q) || (isk && a.rope_k)) {
        float c, sn;
        if (a.rope_tab) {
            c = a.rope_tab[(long)row * D + i];
            sn = a.rope_tab[(long)row * D + H2 + i];
        } else {
            const float ang = a.inv_freq[i] * a.pos[m];
            c = a.exact_trig ? t5g_exact::rope_trig(ang, 0, a.trig_exc, a.n_trig_exc) : rbf(cosf(ang));
            sn = a.exact_trig ? t5g_exact::rope_trig(ang, 1, a.trig_exc, a.n_trig_exc) : rbf(sinf(ang));
        }
        o1 = rbf(rbf(x1 * c) + rbf(-x2 * sn));
        o2 = rbf(rbf(x2 * c) + rbf(x1 * sn));
    }
    bf16_t* dst;
    if (isq) {
        dst = a.Qout + (long)m * a.ldq + h * D;
    } else {
        dst = (isk ? a.Kc + (h - a.nq) * a.c_hstride : a.Vc + (h - a.nq - a.nk) * a.c_hstride) +
              row * a.c_bstride + (long)slot * D;
    }
    dst[i] = f2bf(o1);
    dst[i + H2] = f2bf(o2);
}

int rope_store(const RopeArgs& a, hipStream_t st) {
    if (a.M <= 0) return 0;
    if (a.nq && a.Qout == a.X && a.ldq != a.ldx) return -1;
    if (!a.X && !a.Xpart) return -1;
    if (a.Xpart && (a.nsplit < 1 || a.nsplit > 8)) return -1;
    const int pairs = (a.nq + a.nk + a.nv) * (a.D / 2);
    // in-place q rope is safe: each (h, i) pair is read and written by one thread
    hipLaunchKernelGGL(rope_store_kernel, dim3((unsigned)a.M, (unsigned)((pairs + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---------------------------------------------------------------------------
// Many-query attention (encoder self attention, decoder prefill self / cross attention,
// eager decode): one block per (query, kv head) over all of the row's keys, the G query
// heads of the GQA group sharing every K/V row read. ``sdpa`` numerics follow aten's CPU
// flash attention (common.h sdpa_*): kv blocks of 512 keys with a running max, the fast
// exp on each block's 16-multiple prefix, lane-ordered sums, bf16 P before P.V, output
// scaled by 1/l; a causal row t sees its q-block's key range (sdpa_qsplit). ``eager``
// mirrors eager_attention_forward (bf16 scores, tanh softcap, bf16 normalised probs).

template <int D, int G, bool EAGER>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
    constexpr int LPK = D / 8;        // lanes per key row
    constexpr int KPW = 64 / LPK;     // keys per wave instruction
    constexpr int KPB = KPW * 4;      // keys per block iteration
    static_assert(SDPA_KV_BLOCK % KPB == 0, "kv blocks must hold whole key groups");
    extern __shared__ __attribute__((aligned(16))) float sm[];  // [G][chunk] scores, then probs
    __shared__ float red[32];
    __shared__ f32x4 ored[4][G][64][2];
    __shared__ float blk_et[G][SDPA_MAX_BLOCKS];
    __shared__ float stat_l[G];

    const int qi = blockIdx.x, kvh = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kg = lane / LPK, dl = lane % LPK;
    const int row = a.q_row ? a.q_row[qi] : qi;
    const int len = a.kv_len[row];
    const int t = a.q_pos ? a.q_pos[qi] : len - 1;
    int lo = 0, hi = len;
    if (a.causal) {
        hi = min(t + 1, len);
        if (a.window > 0) lo = max(0, t - a.window + 1);
    } else if (a.window > 0) {
        lo = max(0, t - a.window);
        hi = min(len, t + a.window + 1);
    }
    const int n = hi - lo;
    if (n <= 0) return;
    // keys in aten's blocks for this row: a causal row sees its q-block's range
    int nk = hi;
    if (a.causal && a.window == 0) {
        const int qs = sdpa_qsplit(len);
        nk = min(t - t % qs + qs, len);
    }
    float q[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        u32x4 w = *(const u32x4*)(a.Q + (long)qi * a.ldq + (kvh * G + g) * D + 8 * dl);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            q[g][2 * j] = bf_lo(w[j]);
            q[g][2 * j + 1] = bf_hi(w[j]);
        }
    }
    const bf16_t* Kb = a.K + row * a.kv_bstride + kvh * a.kv_hstride;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride;

    // ---- scores
    for (int j0 = lo; j0 < hi; j0 += KPB) {
        const int j = j0 + wave * KPW + kg;
        float s[G];
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] = 0.f;
        if (j < hi) {
            u32x4 w = *(const u32x4*)(Kb + (long)j * D + 8 * dl);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                float k0 = bf_lo(w[jj]), k1 = bf_hi(w[jj]);
#pragma unroll
                for (int g = 0; g < G; ++g) s[g] += q[g][2 * jj] * k0 + q[g][2 * jj + 1] * k1;
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            s[g] = xsum<LPK>(s[g]);
        }
        if (dl == 0 && j < hi) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float v;
                if constexpr (EAGER) {
                    v = rbf(rbf(s[g]) * a.scale);
                    if (a.softcap > 0.f) v = rbf(rbf(tanhf(rbf(v / a.softcap))) * a.softcap);
                } else {
                    v = __fmul_rn(s[g], a.scale);
                }
                sm[g * a.chunk + (j - lo)] = v;
            }
        }
    }
    __syncthreads();
    // ---- softmax
    if constexpr (EAGER) {
        // softmax(fp32) over the row, normalised probabilities rounded to bf16
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float lm = -INFINITY;
            for (int i = threadIdx.x; i < n; i += 256) lm = fmaxf(lm, sm[g * a.chunk + i]);
            const float mx = block_max(lm, red);
            float ls = 0.f;
            for (int i = threadIdx.x; i < n; i += 256) ls += expf(sm[g * a.chunk + i] - mx);
            const float inv = 1.0f / block_sum(ls, red);
            __syncthreads();
            for (int i = threadIdx.x; i < n; i += 256) sm[g * a.chunk + i] = rbf(expf(sm[g * a.chunk + i] - mx) * inv);
        }
    } else if (wave < G) {
        // one wave per query head, block by block (running max, lane-ordered sums)
        const int g = wave;
        float* sg = sm + g * a.chunk;
        float m = -INFINITY, l = 0.f;
        int b = 0;
        for (int bs = lo; bs < nk; bs += SDPA_KV_BLOCK, ++b) {
            const int blen = min(SDPA_KV_BLOCK, nk - bs);
            const int bhi = min(bs + blen, hi);   // keys past hi are masked (p = 0)
            float lm = -INFINITY;
            for (int i = bs + lane; i < bhi; i += 64) lm = fmaxf(lm, sg[i - lo]);
            const float mn = fmaxf(m, wave_max(lm));
            auto pf = [&](int pos) -> float {
                return bs + pos < bhi ? sdpa_p(__fsub_rn(sg[bs + pos - lo], mn), pos, blen) : 0.f;
            };
            const float ts = sdpa_block_sum(blen, lane, pf);
            const float et = sdpa_block_rescale(m, mn);
            l = fmaf(et, l, ts);
            // this wave's lanes all finished reading the block's scores before any writes
            float pw[SDPA_KV_BLOCK / 64];
#pragma unroll
            for (int k = 0; k < SDPA_KV_BLOCK / 64; ++k) pw[k] = pf(lane + 64 * k);
#pragma unroll
            for (int k = 0; k < SDPA_KV_BLOCK / 64; ++k)
                if (bs + lane + 64 * k < bhi) sg[bs + lane + 64 * k - lo] = rbf(pw[k]);
            if (lane == 0) blk_et[g][b] = et;
            m = mn;
        }
        if (lane == 0) stat_l[g] = l;
    }
    __syncthreads();
    // ---- P.V: lane owns dims [8*dl, 8*dl+8) of key group kg
    float o[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[g][jj] = 0.f;
    for (int j0 = lo; j0 < hi; j0 += KPB) {
        if (!EAGER && j0 > lo && (j0 - lo) % SDPA_KV_BLOCK == 0) {
            // a new kv block: dst *= expf(m_old - m_new) (aten rescales before adding P.V)
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const float et = blk_et[g][(j0 - lo) / SDPA_KV_BLOCK];
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) o[g][jj] *= et;
            }
        }
        const int j = j0 + wave * KPW + kg;
        if (j < hi) {
            u32x4 w = *(const u32x4*)(Vb + (long)j * D + 8 * dl);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float p = sm[g * a.chunk + (j - lo)];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    o[g][2 * jj] += p * bf_lo(w[jj]);
                    o[g][2 * jj + 1] += p * bf_hi(w[jj]);
                }
            }
        }
    }
    // reduce over key groups within the wave (lanes differing in bits >= log2(LPK))
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
#pragma unroll
            for (int off = LPK; off < 64; off <<= 1) o[g][jj] += __shfl_xor(o[g][jj], off, 64);
        }
    if (kg == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            ored[wave][g][dl][0] = (f32x4){o[g][0], o[g][1], o[g][2], o[g][3]};
            ored[wave][g][dl][1] = (f32x4){o[g][4], o[g][5], o[g][6], o[g][7]};
        }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < G * LPK; idx += 256) {
        const int g = idx / LPK, d8 = idx % LPK;
        f32x4 lo4 = ored[0][g][d8][0] + ored[1][g][d8][0] + ored[2][g][d8][0] + ored[3][g][d8][0];
        f32x4 hi4 = ored[0][g][d8][1] + ored[1][g][d8][1] + ored[2][g][d8][1] + ored[3][g][d8][1];
        float v[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        const float inv = EAGER ? 1.0f : __fdiv_rn(1.0f, stat_l[g]);
        u32x4 w;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) w[jj] = pack2(__fmul_rn(v[2 * jj], inv), __fmul_rn(v[2 * jj + 1], inv));
        *(u32x4*)(a.O + (long)qi * a.ldo + (kvh * G + g) * D + 8 * d8) = w;
    }
}

// ---------------------------------------------------------------------------
// Decode attention (one query row per (row, kv head), sdpa numerics): the row's keys
// [lo, hi) are cut into 64-key chunks from lo, one workgroup each, so aten's 512-key
// blocks are whole chunk groups.
//  * attn_decode_kernel: q straight from the projection's fp32 split-K slabs (summed,
//    rounded, PM-RoPE'd in-kernel), the step's own k/v appended to the cache by the
//    chunk holding t, scores of the chunk. A row of <= 64 keys is finished here (softmax,
//    P.V, output). Longer rows publish scores + chunk maxima for:
//  * attn_pvc_kernel: per (row, kv head, 32-dimension slice) the exact p of every key
//    against its block's running max, l with aten's lane-ordered block sums, bf16 P.V
//    over the slice, rescaled across blocks, scaled by 1/l.
constexpr int QSMAX = 4;   // q / appended-k/v projection slabs read by the decode kernel
constexpr int DCH = 64;    // keys per decode chunk

// Flash-form tail of a chunk workgroup (see attn_decode_kernel): sm holds the chunk's
// scaled scores, vr its V rows (appended value included). Partials go out as sc1
// (write-through) buffer stores; every storing wave drains; one lane takes the (row, kv
// head)'s ticket; the workgroup whose add returns nch - 1 reads them back with sc1 loads
// (the sampler's / fused block's hand-off form, CDNA guide G16 row 1) and resets the ticket.
template <int D, int G>
__device__ __forceinline__ void attn_flash_finish(const AttnArgs& a, float (&sm)[G][DCH], const u32x4 (&vr)[DCH / (4 * (64 / (D / 8)))],
                                                  int qi, int kvh, int sp, int nch, int n, int wave, int lane, int kg,
                                                  int dl) {
    constexpr int LPK = D / 8;
    constexpr int KPW = 64 / LPK;
    constexpr int KPB = KPW * 4;
    constexpr int NIT = DCH / KPB;
    constexpr int FB = 16;  // chunk partials per combine batch (one batch up to 1 024 keys)
    __shared__ f32x4 ored[4][G][LPK][2];
    __shared__ float cstat[G][2];
    __shared__ float wts[G][DEC_MAX_CHUNKS];
    __shared__ float lsum[G];
    __shared__ int last;
    const int tid = (int)threadIdx.x;
    const long rec = ((long)qi * a.Hkv + kvh) * a.nsplit;   // chunk records of this (row, kv head)
    if (wave < G) {
        const int g = wave;
        const float s = lane < n ? sm[g][lane] : -INFINITY;
        const float mx = wave_max(s);
        const float p = lane < n ? __expf(s - mx) : 0.f;
        sm[g][lane] = rbf(p);
        const float l = xsum<64>(p);
        if (lane == 0) {
            cstat[g][0] = mx;
            cstat[g][1] = l;
        }
    }
    __syncthreads();
    float o[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[g][jj] = 0.f;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int jl = i * KPB + wave * KPW + kg;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float p = sm[g][jl];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                o[g][2 * jj] += p * bf_lo(vr[i][jj]);
                o[g][2 * jj + 1] += p * bf_hi(vr[i][jj]);
            }
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
#pragma unroll
            for (int off = LPK; off < 64; off <<= 1) o[g][jj] += __shfl_xor(o[g][jj], off, 64);
    if (kg == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            ored[wave][g][dl][0] = (f32x4){o[g][0], o[g][1], o[g][2], o[g][3]};
            ored[wave][g][dl][1] = (f32x4){o[g][4], o[g][5], o[g][6], o[g][7]};
        }
    }
    __syncthreads();
    const long nrec = (long)a.Mq * a.Hkv * a.nsplit;
    const __amdgpu_buffer_rsrc_t prs = frag_rsrc(a.fpart, (uint32_t)(nrec * G * D * 4));
    const __amdgpu_buffer_rsrc_t srs = frag_rsrc(a.fstat, (uint32_t)(nrec * G * 2 * 4));
    for (int idx = tid; idx < G * LPK; idx += 256) {
        const int g = idx / LPK, d8 = idx % LPK;
        const f32x4 lo4 = ored[0][g][d8][0] + ored[1][g][d8][0] + ored[2][g][d8][0] + ored[3][g][d8][0];
        const f32x4 hi4 = ored[0][g][d8][1] + ored[1][g][d8][1] + ored[2][g][d8][1] + ored[3][g][d8][1];
        const int off = (int)((((rec + sp) * G + g) * D + 8 * d8) * 4);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo4), prs, off, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi4), prs, off + 16, 0, 16);
    }
    if (tid < G) {
        const u32x2_t st = {__float_as_uint(cstat[tid][0]), __float_as_uint(cstat[tid][1])};
        __builtin_amdgcn_raw_buffer_store_b64(st, srs, (int)((((rec + sp) * G + tid) * 2) * 4), 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    T5G_TS(3);
    if (tid == 0)
        last = __hip_atomic_fetch_add(a.fticket + (long)qi * a.Hkv + kvh, 1u, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nch - 1);
    __syncthreads();
    T5G_TS(4);
    if (!last) return;
    // ---- the combine (last chunk to arrive). Waves 0..G-1: the chunk weights
    // exp(m_c - M) and the sum; waves G..: the output octets, their first batch of
    // partials requested before the weights are known.
    if (tid == 0) __hip_atomic_store(a.fticket + (long)qi * a.Hkv + kvh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    constexpr int NOUT = G * D / 4;                   // f32x4 outputs
    static_assert(NOUT <= 256 - 64 * G, "flash combine geometry");
    const int ot = tid - 64 * G;                       // output thread index
    const bool outer = ot >= 0 && ot < NOUT;
    const int og = outer ? ot / (D / 4) : 0, o4 = outer ? ot % (D / 4) : 0;
    auto pload = [&](f32x4 (&pv)[FB], int c0) {
#pragma unroll
        for (int k = 0; k < FB; ++k) {
            int off = (c0 + k < nch && outer) ? (int)((((rec + c0 + k) * G + og) * D + 4 * o4) * 4) : (int)0x7ffffff0;
            asm volatile("" : "+v"(off));
            pv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, off, 0, 16));
        }
    };
    f32x4 pv[FB];
    pload(pv, 0);
    if (wave < G) {
        // lane owns chunks lane + 64 i (rows of up to DEC_MAX_CHUNKS chunks)
        constexpr int CPL = DEC_MAX_CHUNKS / 64;
        const int g = wave;
        float m[CPL], l[CPL];
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
            const int c = lane + 64 * i;
            int off = c < nch ? (int)((((rec + c) * G + g) * 2) * 4) : (int)0x7ffffff0;
            asm volatile("" : "+v"(off));
            const u32x2_t st = __builtin_amdgcn_raw_buffer_load_b64(srs, off, 0, 16);
            m[i] = c < nch ? __uint_as_float(st[0]) : -INFINITY;
            l[i] = c < nch ? __uint_as_float(st[1]) : 0.f;
        }
        float mm = m[0];
#pragma unroll
        for (int i = 1; i < CPL; ++i) mm = fmaxf(mm, m[i]);
        const float M = wave_max(mm);
        float wl = 0.f;
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
            const float w = lane + 64 * i < nch ? __expf(m[i] - M) : 0.f;
            wts[g][lane + 64 * i] = w;
            wl += w * l[i];
        }
        const float L = xsum<64>(wl);
        if (lane == 0) lsum[g] = L;
    }
    __syncthreads();
    T5G_TS(6);
    if (!outer) return;
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nch; c0 += FB) {
        if (c0 > 0) pload(pv, c0);
#pragma unroll
        for (int k = 0; k < FB; ++k) {
            const float w = c0 + k < nch ? wts[og][c0 + k] : 0.f;
            acc += w * pv[k];
        }
    }
    const float inv = 1.0f / lsum[og];
    const u32x2_t ow = {pack2(acc[0] * inv, acc[1] * inv), pack2(acc[2] * inv, acc[3] * inv)};
    *(u32x2_t*)(a.O + (long)qi * a.ldo + (kvh * G + og) * D + 4 * o4) = ow;
    T5G_TS_BY(5, 64 * G);
}

//  * FLASH (fast path, a.flash): rows of > 64 keys finish in the same launch -- each
//    chunk's workgroup requests its V with K, computes its online-softmax partial (chunk
//    max m_c, l_c = sum exp(s - m_c), unnormalised bf16(p).V) and hands it off through
//    write-through stores + an arrival ticket; the last chunk of the (row, kv head) to
//    arrive combines: O = sum_c exp(m_c - M) o_c / sum_c exp(m_c - M) l_c (M = max m_c).
//    Not aten's 512-key block order: fast mode only (parity mode runs xattn.hip).
template <int D, int G, bool VFIRST, bool FLASH = false>
__global__ __launch_bounds__(256, 2) void attn_decode_kernel(AttnArgs a) {
    constexpr int LPK = D / 8;
    constexpr int KPW = 64 / LPK;
    constexpr int KPB = KPW * 4;
    constexpr int NIT = DCH / KPB;
    __shared__ float sm[G][DCH];
    __shared__ float pl[G][DCH + 16];
    __shared__ float stat_l[G];
    __shared__ f32x4 ored[4][G][LPK][2];
    __shared__ float qs[G][D];
    __shared__ float kvnew[2][D];   // appended key (pre-RoPE) / value of position t

    const int qi = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kg = lane / LPK, dl = lane % LPK;
    T5G_TS(0);
    const int row = a.q_row ? a.q_row[qi] : qi;
    // row length / query position first: the oldest outstanding load is the first one a
    // wave can wait for, so these must not queue behind the K/V stream
    const int len = a.kv_len[row];
    const int t = a.q_pos ? a.q_pos[qi] : len - 1;
    int lo = 0, hi = len;
    if (a.causal) {
        hi = min(t + 1, len);
        if (a.window > 0) lo = max(0, t - a.window + 1);
    } else if (a.window > 0) {
        lo = max(0, t - a.window);
        hi = min(len, t + a.window + 1);
    }
    const int span = max(hi - lo, 0);
    const bool single = span <= DCH;     // the whole row is chunk 0: finished in this kernel
    const int c0 = lo + sp * DCH;
    const int c1 = min(hi, c0 + DCH);
    const int n = c1 - c0;
    // chunks past the row (the grid covers the cache capacity) leave before any request:
    // they publish nothing, and the block holding t always has keys
    if (n <= 0) return;
    // the block whose keys include t appends the step's own key/value (a.append)
    const bool has_t = a.append && a.Qpart && t >= c0 && t < c1;
    // head_split > 1 (single-chunk rows, no append: cross attention): blockIdx.y is a q
    // head run alone (G = 1) against kv head blockIdx.y / head_split
    const int kvc = kvh / a.head_split;
    const bf16_t* Kb = a.K + row * a.kv_bstride + kvc * a.kv_hstride;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvc * a.kv_hstride;
    // Issue order = wait order (vmcnt is in-order): first what the q path needs (the
    // projection's split-K slabs, the PM-RoPE table), then the K (and, for a single-chunk
    // row, V) stream, so q can be summed, staged and rotated while they are in flight.
    // All loads are unconditional (clamped addresses): a load under a branch makes the
    // compiler wait for everything in flight at the join.
    f32x4 u[QSMAX];
    int role = -1, c4 = 0, g_own = 0;
    if (a.Qpart) {
        const int tq = (int)threadIdx.x;
        int col = kvh * G * D;   // idle threads: quad 0 of q
        if (tq < G * D / 4) {
            role = 0;
            g_own = tq / (D / 4);
            c4 = tq % (D / 4);
            col = (kvh * G + g_own) * D + 4 * c4;
        } else if (has_t && tq < (G + 2) * D / 4) {
            const int idx = tq - G * D / 4;
            role = 1 + idx / (D / 4);   // 1: key, 2: value
            c4 = idx % (D / 4);
            col = (role == 1 ? a.k_col0 : a.v_col0) + kvc * D + 4 * c4;
        }
#pragma unroll
        for (int s = 0; s < QSMAX; ++s)
            u[s] = *(const f32x4*)(a.Qpart + ((long)min(s, a.q_nsplit - 1) * a.Mq + qi) * a.ldqp + col);
    }
    float c8[8], s8[8];
    if (a.rope_tab) {
        const float* tr = a.rope_tab + (long)row * D + (8 * dl) % (D / 2);
        const f32x4 ca = *(const f32x4*)tr, cb = *(const f32x4*)(tr + 4);
        const f32x4 sa = *(const f32x4*)(tr + D / 2), sb = *(const f32x4*)(tr + D / 2 + 4);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            c8[jj] = ca[jj];
            c8[4 + jj] = cb[jj];
            s8[jj] = sa[jj];
            s8[4 + jj] = sb[jj];
        }
    }
    // buffer loads: keys past c1 (and V of multi-chunk rows) fall outside the descriptor
    // (zeros, no traffic) -- no branch
    const __amdgpu_buffer_rsrc_t krs = frag_rsrc(Kb, (uint32_t)a.kv_cap * D * 2u);
    const __amdgpu_buffer_rsrc_t vrs = frag_rsrc(Vb, (uint32_t)a.kv_cap * D * 2u);
    // V is read only by single-chunk rows. VFIRST (launches whose rows are all one chunk:
    // cross attention) requests it with K; otherwise it is requested after the scores, so
    // NIT V registers are not held through the K stream: <= 128 VGPRs, four workgroups per
    // CU, 1 024 chunk workgroups in one round (32 rows x 4 kv heads x 8 chunks)
    // (all K requests ahead of all V requests measured the same: the data phase is the
    // memory system's loaded latency for every chunk's requests at once, not the order)
    u32x4 kr[NIT], vr[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int j = c0 + i * KPB + wave * KPW + kg;
        const int off = j < c1 ? (j * D + 8 * dl) * 2 : (int)0x7ffffff0;
        kr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
        if constexpr (VFIRST)
            vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  vrs, (single || FLASH) ? off : (int)0x7ffffff0, 0, 0));
    }
    float q[G][8];
    if (a.Qpart) {
        f32x4 acc = u[0];
#pragma unroll
        for (int s = 1; s < QSMAX; ++s)
            if (s < a.q_nsplit) acc += u[s];
        if (role == 0) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) qs[g_own][4 * c4 + jj] = rbf(acc[jj]);
        } else if (role > 0) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) kvnew[role - 1][4 * c4 + jj] = rbf(acc[jj]);
        }
        if (!a.rope_tab) {
            const float ps = a.pos[row];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const float ang = a.inv_freq[(8 * dl + jj) % (D / 2)] * ps;
                c8[jj] = rbf(cosf(ang));
                s8[jj] = rbf(sinf(ang));
            }
        }
        __syncthreads();
        T5G_TS(1);
        // lower half: x*c + (-x2)*s ; upper half: x*c + x1*s (one branch-free formula)
        const float sg = dl < LPK / 2 ? -1.0f : 1.0f;
        const int pbase = (8 * dl + D / 2) % D;
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const float x = qs[g][8 * dl + jj];
                const float pr = qs[g][pbase + jj];
                q[g][jj] = rbf(rbf(x * c8[jj]) + rbf((sg * pr) * s8[jj]));
            }
    } else {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            u32x4 w = *(const u32x4*)(a.Q + (long)qi * a.ldq + (kvh * G + g) * D + 8 * dl);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                q[g][2 * j] = bf_lo(w[j]);
                q[g][2 * j + 1] = bf_hi(w[j]);
            }
        }
    }
    if (n <= 0) return;
    u32x4 vt = (u32x4){0u, 0u, 0u, 0u};   // the appended value, for the lane holding key t
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int j = c0 + i * KPB + wave * KPW + kg;
        if (j >= c1) {
            kr[i] = (u32x4){0u, 0u, 0u, 0u};
            if constexpr (VFIRST) vr[i] = (u32x4){0u, 0u, 0u, 0u};
        }
        if (has_t && j == t) {
            // key t: PM-RoPE of the new key (rope_store_kernel's arithmetic), then append
            const float sg = dl < LPK / 2 ? -1.0f : 1.0f;
            const int pbase = (8 * dl + D / 2) % D;
            u32x4 kw, vw;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                float ko[2], vo[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int dd = 8 * dl + 2 * jj + e;
                    const float c = c8[2 * jj + e], sn = s8[2 * jj + e];
                    const float x = kvnew[0][dd], pr = kvnew[0][pbase + 2 * jj + e];
                    ko[e] = rbf(rbf(x * c) + rbf((sg * pr) * sn));
                    vo[e] = kvnew[1][dd];
                }
                kw[jj] = pack2(ko[0], ko[1]);
                vw[jj] = pack2(vo[0], vo[1]);
            }
            kr[i] = kw;
            vt = vw;
            if constexpr (VFIRST) vr[i] = vw;
            *(u32x4*)(const_cast<bf16_t*>(Kb) + (long)t * D + 8 * dl) = kw;
            *(u32x4*)(const_cast<bf16_t*>(Vb) + (long)t * D + 8 * dl) = vw;
        }
    }
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        float s[G];
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] = 0.f;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const float k0 = bf_lo(kr[i][jj]), k1 = bf_hi(kr[i][jj]);
#pragma unroll
            for (int g = 0; g < G; ++g) s[g] += q[g][2 * jj] * k0 + q[g][2 * jj + 1] * k1;
        }
#pragma unroll
        for (int g = 0; g < G; ++g)
            s[g] = xsum<LPK>(s[g]);
        const int jl = i * KPB + wave * KPW + kg;
        if (dl == 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) sm[g][jl] = fast_score(s[g], a.scale, a.softcap);
        }
    }
    __syncthreads();
    T5G_TS(2);
    if constexpr (FLASH) {
        if (!single) {
            attn_flash_finish<D, G>(a, sm, vr, qi, kvh, sp, (span + DCH - 1) / DCH, n, wave, lane, kg, dl);
            return;
        }
    }
    if (!single) {
        // publish the chunk's scores and maxima (read by the next two launches)
        if (wave < G) {
            const int g = wave;
            const float s = lane < n ? sm[g][lane] : -INFINITY;
            if (lane < n) a.sbuf[((long)qi * a.Hkv * G + kvh * G + g) * a.kv_cap + c0 + lane] = s;
            const float mx = wave_max(s);
            if (lane == 0) a.mbuf[(((long)qi * a.Hkv + kvh) * a.nsplit + sp) * G + g] = mx;
        }
        T5G_TS(5);
        return;
    }
    // single-chunk row: one aten kv block of `span` keys; every lane computes its key's p
    // once (the tail's double exp included), the block sum then only chains adds. Its V
    // (the appended value from registers, not from the store above) is requested first.
    if constexpr (!VFIRST) {
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int j = c0 + i * KPB + wave * KPW + kg;
            const int off = (j < c1 && !(has_t && j == t)) ? (j * D + 8 * dl) * 2 : (int)0x7ffffff0;
            vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0));
            if (has_t && j == t) vr[i] = vt;
        }
    }
    if (wave < G) {
        const int g = wave;
        const float s = lane < n ? sm[g][lane] : -INFINITY;
        const float mx = wave_max(s);
        const float p = lane < n ? sdpa_p(__fsub_rn(s, mx), lane, span) : 0.f;
        pl[g][lane] = p;
        if (lane < 16) pl[g][DCH + lane] = 0.f;
        sm[g][lane] = rbf(p);
        __builtin_amdgcn_wave_barrier();
        const float l = sdpa_block_sum_lds<DCH>(pl[g], span, lane);
        if (lane == 0) stat_l[g] = l;
    }
    __syncthreads();
    float o[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[g][jj] = 0.f;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int jl = i * KPB + wave * KPW + kg;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float p = sm[g][jl];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                o[g][2 * jj] += p * bf_lo(vr[i][jj]);
                o[g][2 * jj + 1] += p * bf_hi(vr[i][jj]);
            }
        }
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
#pragma unroll
            for (int off = LPK; off < 64; off <<= 1) o[g][jj] += __shfl_xor(o[g][jj], off, 64);
    if (kg == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            ored[wave][g][dl][0] = (f32x4){o[g][0], o[g][1], o[g][2], o[g][3]};
            ored[wave][g][dl][1] = (f32x4){o[g][4], o[g][5], o[g][6], o[g][7]};
        }
    }
    __syncthreads();
    T5G_TS(4);
    for (int idx = threadIdx.x; idx < G * LPK; idx += 256) {
        const int g = idx / LPK, d8 = idx % LPK;
        const f32x4 lo4 = ored[0][g][d8][0] + ored[1][g][d8][0] + ored[2][g][d8][0] + ored[3][g][d8][0];
        const f32x4 hi4 = ored[0][g][d8][1] + ored[1][g][d8][1] + ored[2][g][d8][1] + ored[3][g][d8][1];
        const float inv = __fdiv_rn(1.0f, stat_l[g]);
        u32x4 w;
        w[0] = pack2(__fmul_rn(lo4[0], inv), __fmul_rn(lo4[1], inv));
        w[1] = pack2(__fmul_rn(lo4[2], inv), __fmul_rn(lo4[3], inv));
        w[2] = pack2(__fmul_rn(hi4[0], inv), __fmul_rn(hi4[1], inv));
        w[3] = pack2(__fmul_rn(hi4[2], inv), __fmul_rn(hi4[3], inv));
        *(u32x4*)(a.O + (long)qi * a.ldo + (kvh * G + g) * D + 8 * d8) = w;
    }
    T5G_TS(5);
}

// row geometry shared by the pv / combine kernels (same rules as attn_decode_kernel)
struct DecRow {
    int lo, hi, span;
};
__device__ __forceinline__ DecRow dec_row(const AttnArgs& a, int qi) {
    const int row = a.q_row ? a.q_row[qi] : qi;
    const int len = a.kv_len[row];
    const int t = a.q_pos ? a.q_pos[qi] : len - 1;
    int lo = 0, hi = len;
    if (a.causal) {
        hi = min(t + 1, len);
        if (a.window > 0) lo = max(0, t - a.window + 1);
    } else if (a.window > 0) {
        lo = max(0, t - a.window);
        hi = min(len, t + a.window + 1);
    }
    return {lo, hi, max(hi - lo, 0)};
}

// P.V and combine of the rows of > 64 keys in ONE launch (attn_pvc_kernel). Workgroup
// (row, kv head, z) owns PVC_DZ of the D output dimensions of the G heads, for every key
// of the row, so nothing is handed between workgroups: it recomputes the exact p of each
// aten 512-key block from the published scores and chunk maxima (cheap: <= 2 x 4096
// exps), takes l from aten's lane-ordered block sums of them, and streams only its
// DZ-wide slice of V (DZ = 32: 64 B per key at D = 256, all 8 slices of a row on one XCD
// under round-robin placement, so a 128-B line is fetched once; DZ = 64 when 32-wide
// slices would need more than one workgroup per CU, e.g. 16 or 32 rows).
// The fp32 sums keep the order of the former per-chunk P.V + combine pair, so results are
// bit-identical to it: per 64-key chunk, KPB key slots (slot = wave * KPW + kg of the
// chunk kernel's lane map) each accumulate NIT keys j = c0 + i * KPB + slot in i order;
// the KPW slots of a wave fold as a pairwise (xor-butterfly) tree, the 4 waves in order;
// the chunks of a block are summed in order from 0; dst = dst * exp(m_old - m) + block.
template <int D, int G, int PVC_DZ>   // PVC_DZ: output dimensions per workgroup
__global__ __launch_bounds__(256) void attn_pvc_kernel(AttnArgs a) {
    constexpr int LPK = D / 8;
    constexpr int KPW = 64 / LPK;
    constexpr int KPB = KPW * 4;                // key slots per chunk
    constexpr int NIT = DCH / KPB;              // keys per slot chain
    constexpr int NOCT = PVC_DZ / 8;            // 16-byte dimension octets per workgroup
    constexpr int TPC = KPB * NOCT;             // threads per chunk
    constexpr int CPR = 256 / TPC;              // chunks per sub-round
    constexpr int CPB = SDPA_KV_BLOCK / DCH;    // chunks per aten kv block
    constexpr int RPB = CPB / CPR;              // sub-rounds per kv block
    constexpr int PPT = SDPA_KV_BLOCK / 256;    // block positions per thread when staging p
    static_assert(256 % TPC == 0 && CPB % CPR == 0 && D % PVC_DZ == 0, "pvc geometry");
    __shared__ float pex[G][SDPA_KV_BLOCK + 16];   // exact p of the current block (l)
    __shared__ float pbf[G][SDPA_KV_BLOCK];        // bf16-rounded p (P.V)
    __shared__ float mrun[G][SDPA_MAX_BLOCKS];     // running max through block b
    __shared__ float et_s[G], stat_l[G];
    // slot chain sums of the sub-round, one padded row per slot: a wave's slots then start
    // on different banks (unpadded, the 16 slots of a wave's lanes met on 4 banks: 16-way)
    constexpr int OLW = G * PVC_DZ + 4;
    __shared__ __attribute__((aligned(16))) float ol[CPR][KPB][OLW];
    // second block of the one-pass path (rows of <= 1024 keys)
    __shared__ float pex1[G][SDPA_KV_BLOCK + 16];
    __shared__ float pbf1[G][SDPA_KV_BLOCK];
    __shared__ __attribute__((aligned(16))) float ol1[CPR][KPB][OLW];
    __shared__ float tsum[G][2];
    const int qi = blockIdx.x, kvh = blockIdx.y, z = blockIdx.z;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    T5G_TS(0);
    const int row = a.q_row ? a.q_row[qi] : qi;
    const DecRow r = dec_row(a, qi);
    if (r.span <= DCH) return;                  // finished by attn_decode_kernel
    const int nch = (r.span + DCH - 1) / DCH;
    const int nblk = (r.span + SDPA_KV_BLOCK - 1) / SDPA_KV_BLOCK;
    const int nsr = nblk * RPB;
    const int cr = tid / TPC, slot = (tid % TPC) / NOCT, od = tid % NOCT;
    // a sub-round's V slice (unconditional: keys past the row read as zeros through the
    // buffer range check)
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride;
    const __amdgpu_buffer_rsrc_t vrs = frag_rsrc(Vb, (uint32_t)a.kv_cap * D * 2u);
    auto vload = [&](u32x4 (&v)[NIT], int sr) {
        const int c = (sr / RPB) * CPB + (sr % RPB) * CPR + cr;
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int j = r.lo + c * DCH + i * KPB + slot;
            int off = (sr < nsr && j < r.hi) ? (j * D + PVC_DZ * z + 8 * od) * 2 : (int)0x7ffffff0;
            // an opaque offset: otherwise the uniform sr < nsr test becomes a branch between
            // two forms of the load, and its join waits for every load in flight
            asm volatile("" : "+v"(off));
            v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0));
        }
    };
    // the scores and chunk maxima first (small, L2-resident: the scores launch wrote them),
    // then the V slices: the running maxima, the exact p and the block sums are computed
    // while V is in flight (vmcnt is in order). Every load unconditional (clamped index).
    const float* sb = a.sbuf + ((long)qi * a.Hkv * G + kvh * G) * a.kv_cap + r.lo;
    auto sload = [&](float (&sc)[G][PPT], int b) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int k = 0; k < PPT; ++k) {
                const int pos = b * SDPA_KV_BLOCK + tid + 256 * k;
                sc[g][k] = sb[(long)g * a.kv_cap + (pos < r.span ? pos : 0)];
            }
    };
    float scn[G][PPT], sc1[G][PPT];
    sload(scn, 0);
    if constexpr (RPB == 1) sload(sc1, 1);
    constexpr int CPL = DEC_MAX_CHUNKS / 64;    // chunk maxima per lane (chunk lane + 64 i)
    float cmv[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i)
        cmv[i] = a.mbuf[(((long)qi * a.Hkv + kvh) * a.nsplit + min(lane + 64 * i, a.nsplit - 1)) * G + min(wave, G - 1)];
    u32x4 vn[NIT], v1[NIT];
    vload(vn, 0);
    if constexpr (RPB == 1) vload(v1, 1);   // the second block's slice (zeros if none)
    if (wave < G) {   // running maxima through each block, from the chunk maxima
        const int g = wave;
        for (int b = 0; b < nblk; ++b) {
            const int lim = min(nch, (b + 1) * CPB);
            float cm = -INFINITY;
#pragma unroll
            for (int i = 0; i < CPL; ++i)
                if (lane + 64 * i < lim) cm = fmaxf(cm, cmv[i]);
            const float mb = wave_max(cm);
            if (lane == 0) mrun[g][b] = mb;
        }
        if (lane < 16) {
            pex[g][SDPA_KV_BLOCK + lane] = 0.f;
            pex1[g][SDPA_KV_BLOCK + lane] = 0.f;
        }
    }
    __syncthreads();
    T5G_TS(2);
    const bool folder = tid < G * PVC_DZ;
    const int fg = tid / PVC_DZ, fdd = tid % PVC_DZ;
    if constexpr (RPB == 1) {
        if (nblk <= 2) {
            // rows of <= 1024 keys: both blocks in one pass -- every p staged at once, the
            // (head, block) sums on separate waves, the chains of both blocks before one
            // fold. The same operations and order as the block loop below (bit-identical),
            // two barriers instead of five.
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
                if (bb < nblk) {
                    const int blen = min(SDPA_KV_BLOCK, r.span - bb * SDPA_KV_BLOCK);
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        const float mb = mrun[g][bb];
#pragma unroll
                        for (int k = 0; k < PPT; ++k) {
                            const int pos = tid + 256 * k;
                            const float scv = bb ? sc1[g][k] : scn[g][k];
                            const float p = pos < blen ? sdpa_p(__fsub_rn(scv, mb), pos, blen) : 0.f;
                            (bb ? pex1 : pex)[g][pos] = p;
                            (bb ? pbf1 : pbf)[g][pos] = rbf(p);
                        }
                    }
                }
            }
            __syncthreads();
            T5G_TS(3);
            if (wave < G * nblk) {
                const int g = wave % G, bb = wave / G;
                const int blen = min(SDPA_KV_BLOCK, r.span - bb * SDPA_KV_BLOCK);
                const float ts = sdpa_block_sum_lds<SDPA_KV_BLOCK>(bb ? pex1[g] : pex[g], blen, lane);
                if (lane == 0) tsum[g][bb] = ts;
            }
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
                if (bb < nblk) {
                    const int jb = cr * DCH;
                    float o[G][8];
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int jj = 0; jj < 8; ++jj) o[g][jj] = 0.f;
#pragma unroll
                    for (int i = 0; i < NIT; ++i) {
                        const int jl = jb + i * KPB + slot;
                        const u32x4 vv = bb ? v1[i] : vn[i];
#pragma unroll
                        for (int g = 0; g < G; ++g) {
                            const float p = (bb ? pbf1 : pbf)[g][jl];
#pragma unroll
                            for (int jj = 0; jj < 4; ++jj) {
                                o[g][2 * jj] += p * bf_lo(vv[jj]);
                                o[g][2 * jj + 1] += p * bf_hi(vv[jj]);
                            }
                        }
                    }
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        float* dst = &(bb ? ol1 : ol)[cr][slot][g * PVC_DZ + 8 * od];
                        *(f32x4*)dst = (f32x4){o[g][0], o[g][1], o[g][2], o[g][3]};
                        *(f32x4*)(dst + 4) = (f32x4){o[g][4], o[g][5], o[g][6], o[g][7]};
                    }
                }
            }
            __syncthreads();
            T5G_TS(4);
            if (!folder) return;
            float lsum = 0.f, mo = -INFINITY, dd = 0.f;
            for (int bb = 0; bb < nblk; ++bb) {
                const float mb = mrun[fg][bb];
                const float et = sdpa_block_rescale(mo, mb);
                lsum = fmaf(et, lsum, tsum[fg][bb]);
                mo = mb;
                float bk = 0.f;
#pragma unroll
                for (int c = 0; c < CPR; ++c) {
                    float w4[4];
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        float t[KPW];
#pragma unroll
                        for (int k = 0; k < KPW; ++k) t[k] = (bb ? ol1 : ol)[c][w * KPW + k][fg * PVC_DZ + fdd];
#pragma unroll
                        for (int st = 1; st < KPW; st <<= 1)
#pragma unroll
                            for (int k = 0; k < KPW; k += 2 * st) t[k] = t[k] + t[k + st];
                        w4[w] = t[0];
                    }
                    const float pc = ((w4[0] + w4[1]) + w4[2]) + w4[3];
                    if (bb * CPB + c < nch) bk += pc;
                }
                dd = dd * et + bk;
            }
            const float inv = __fdiv_rn(1.0f, lsum);
            a.O[(long)qi * a.ldo + (kvh * G + fg) * D + PVC_DZ * z + fdd] = f2bf(__fmul_rn(dd, inv));
            T5G_TS(1);
            return;
        }
    }
    float l = 0.f, m_old = -INFINITY;            // wave g < G: head g's running sum
    float dst = 0.f, blk = 0.f;                  // fold thread (g, dd)
    auto stage = [&](const float (&sc)[G][PPT], int b) {   // exact p of block b -> LDS
        const int blen = min(SDPA_KV_BLOCK, r.span - b * SDPA_KV_BLOCK);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float mb = mrun[g][b];
#pragma unroll
            for (int k = 0; k < PPT; ++k) {
                const int pos = tid + 256 * k;
                const float p = pos < blen ? sdpa_p(__fsub_rn(sc[g][k], mb), pos, blen) : 0.f;
                pex[g][pos] = p;
                pbf[g][pos] = rbf(p);
            }
        }
        __syncthreads();
        if (wave < G) {
            const int g = wave;
            const float ts = sdpa_block_sum_lds<SDPA_KV_BLOCK>(pex[g], blen, lane);
            const float mb = mrun[g][b];
            const float et = sdpa_block_rescale(m_old, mb);
            l = fmaf(et, l, ts);
            m_old = mb;
            if (lane == 0) et_s[g] = et;
        }
    };
    auto subround = [&](const u32x4 (&v)[NIT], int sr) {
        const int b = sr / RPB, rr = sr % RPB;
        const int jb = (rr * CPR + cr) * DCH;   // chunk start within the block
        float o[G][8];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) o[g][jj] = 0.f;
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int jl = jb + i * KPB + slot;
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const float p = pbf[g][jl];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    o[g][2 * jj] += p * bf_lo(v[i][jj]);
                    o[g][2 * jj + 1] += p * bf_hi(v[i][jj]);
                }
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float* dst = &ol[cr][slot][g * PVC_DZ + 8 * od];
            *(f32x4*)dst = (f32x4){o[g][0], o[g][1], o[g][2], o[g][3]};
            *(f32x4*)(dst + 4) = (f32x4){o[g][4], o[g][5], o[g][6], o[g][7]};
        }
        __syncthreads();
        if (folder) {
            if (rr == 0) blk = 0.f;
#pragma unroll
            for (int c = 0; c < CPR; ++c) {
                float w4[4];
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    float t[KPW];
#pragma unroll
                    for (int k = 0; k < KPW; ++k) t[k] = ol[c][w * KPW + k][fg * PVC_DZ + fdd];
#pragma unroll
                    for (int st = 1; st < KPW; st <<= 1)
#pragma unroll
                        for (int k = 0; k < KPW; k += 2 * st) t[k] = t[k] + t[k + st];
                    w4[w] = t[0];
                }
                const float pc = ((w4[0] + w4[1]) + w4[2]) + w4[3];
                if (b * CPB + rr * CPR + c < nch) blk += pc;
            }
            if (rr == RPB - 1) dst = dst * et_s[fg] + blk;
        }
        __syncthreads();   // ol / pbf / et_s are rewritten by the next sub-round
    };
    // one sub-round per iteration; the next sub-round's V slice (and at a block start
    // the next block's scores) are requested before this one is computed
    for (int sr = 0; sr < nsr; ++sr) {
        if (sr % RPB == 0) {
            const int b = sr / RPB;
            float sc[G][PPT];
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < PPT; ++k) sc[g][k] = scn[g][k];
            sload(scn, b + 1 < nblk ? b + 1 : b);
            stage(sc, b);
        }
        u32x4 v[NIT];
#pragma unroll
        for (int i = 0; i < NIT; ++i) v[i] = vn[i];
        vload(vn, sr + 1);
        subround(v, sr);
    }
    if (wave < G && lane == 0) stat_l[wave] = l;
    __syncthreads();
    T5G_TS(1);
    if (!folder) return;
    const float inv = __fdiv_rn(1.0f, stat_l[fg]);
    a.O[(long)qi * a.ldo + (kvh * G + fg) * D + PVC_DZ * z + fdd] = f2bf(__fmul_rn(dst, inv));
}

template <int D, int G>
static int launch_decode(const AttnArgs& a_in, hipStream_t st) {
    AttnArgs a = a_in;
    a.head_split = 1;
    if constexpr (G == 2) {
        // one chunk and nothing appended (cross attention): one workgroup per q head
        // instead of per kv group -- half the serial work per workgroup, twice the CUs;
        // each head's sums are the same as in the G = 2 kernel (bit-identical)
        if (a.nsplit == 1 && !a.append) {
            a.head_split = 2;
            a.Hkv *= 2;
            a.G = 1;
            hipLaunchKernelGGL((attn_decode_kernel<D, 1, true>), dim3((unsigned)a.Mq, (unsigned)a.Hkv, 1u), dim3(256),
                               0, st, a);
            return hipGetLastError() == hipSuccess ? 0 : -2;
        }
    }
    dim3 grid((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)a.nsplit);
    if (a.flash && a.nsplit > 1) {
        hipLaunchKernelGGL((attn_decode_kernel<D, G, true, true>), grid, dim3(256), 0, st, a);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    if (a.nsplit == 1) hipLaunchKernelGGL((attn_decode_kernel<D, G, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((attn_decode_kernel<D, G, false>), grid, dim3(256), 0, st, a);
    if (a.nsplit > 1) {
        // one round of workgroups: 32-wide slices (one workgroup per CU: 256 VGPRs) while
        // they fit, else 64-wide (two per CU)
        if (D >= 64 && (long)a.Mq * a.Hkv * (D / 32) > 256)
            hipLaunchKernelGGL((attn_pvc_kernel<D, G, 64>), dim3((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)(D / 64)),
                               dim3(256), 0, st, a);
        else
            hipLaunchKernelGGL((attn_pvc_kernel<D, G, 32>), dim3((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)(D / 32)),
                               dim3(256), 0, st, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int attention_decode(const AttnArgs& a, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (a.eager || a.kv_cap <= 0 || a.kv_cap > SDPA_KV_BLOCK * SDPA_MAX_BLOCKS) return -1;
    // 64-key chunks from the row start; the grid covers nsplit of them (the call's longest
    // row, <= the cache capacity: rows longer than nsplit * 64 keys are refused on the host)
    if (a.nsplit < 1 || a.nsplit > (a.kv_cap + DCH - 1) / DCH) return -1;
    if (a.nsplit > 1 && (!a.sbuf || !a.mbuf || a.nsplit > DEC_MAX_CHUNKS)) return -1;
    if (a.flash && a.nsplit > 1 && (!a.fpart || !a.fstat || !a.fticket || a.G * a.D / 4 > 256 - 64 * a.G ||
                                    (long)a.Mq * a.Hkv * a.nsplit * a.G * a.D * 4 > 0x7fff0000L))
        return -1;
    if (a.append && (!a.Qpart || !a.rope_tab || (a.G + 2) * a.D / 4 > 256)) return -1;
    if (a.Qpart && (a.q_nsplit < 1 || a.q_nsplit > QSMAX)) return -1;
    if (a.D == 256 && a.G == 2) return launch_decode<256, 2>(a, st);
    if (a.D == 64 && a.G == 2) return launch_decode<64, 2>(a, st);
    if (a.D == 128 && a.G == 2) return launch_decode<128, 2>(a, st);
    if (a.D == 256 && a.G == 1) return launch_decode<256, 1>(a, st);
    return -3;
}

template <int D, int G>
static int launch_attn(const AttnArgs& a, hipStream_t st) {
    dim3 grid((unsigned)a.Mq, (unsigned)a.Hkv, 1u);
    size_t shm = (size_t)G * a.chunk * sizeof(float);
    if (shm > 64 * 1024) {   // rows of > 8 192 keys (G = 2): opt in to 96 KiB, once per device
        static bool attr[T5G_MAX_DEVICES][2] = {};
        const int dev = t5g_cur_device();
        if (dev < 0) return -2;
        if (!attr[dev][a.eager ? 1 : 0]) {
            (void)hipFuncSetAttribute(a.eager ? (const void*)attn_kernel<D, G, true> : (const void*)attn_kernel<D, G, false>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
            attr[dev][a.eager ? 1 : 0] = true;
        }
    }
    if (a.eager)
        hipLaunchKernelGGL((attn_kernel<D, G, true>), grid, dim3(256), shm, st, a);
    else
        hipLaunchKernelGGL((attn_kernel<D, G, false>), grid, dim3(256), shm, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int attention(const AttnArgs& a, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (a.nsplit != 1 || a.chunk < 1 || a.chunk > SDPA_KV_BLOCK * SDPA_MAX_BLOCKS) return -1;
    if ((size_t)a.G * a.chunk * sizeof(float) > 96 * 1024) return -1;
    if (a.D == 256 && a.G == 2) return launch_attn<256, 2>(a, st);
    if (a.D == 64 && a.G == 2) return launch_attn<64, 2>(a, st);
    if (a.D == 128 && a.G == 2) return launch_attn<128, 2>(a, st);
    if (a.D == 256 && a.G == 1) return launch_attn<256, 1>(a, st);
    return -3;
}

}  // namespace t5g

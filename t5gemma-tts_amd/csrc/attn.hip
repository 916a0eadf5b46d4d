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
#include "t5g_kernels.h"

namespace t5g {

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
            c = rbf(cosf(ang));
            sn = rbf(sinf(ang));
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

__global__ void rope_table_kernel(const float* pos, const float* inv_freq, int D, float* tab) {
    const int r = blockIdx.x, H2 = D / 2;
    for (int i = threadIdx.x; i < H2; i += blockDim.x) {
        const float ang = inv_freq[i] * pos[r];
        tab[(long)r * D + i] = rbf(cosf(ang));
        tab[(long)r * D + H2 + i] = rbf(sinf(ang));
    }
}

int rope_table(const float* pos, const float* inv_freq, int rows, int D, float* tab, hipStream_t st) {
    if (rows <= 0) return 0;
    hipLaunchKernelGGL(rope_table_kernel, dim3((unsigned)rows), dim3(128), 0, st, pos, inv_freq, D, tab);
    return hipGetLastError() == hipSuccess ? 0 : -2;
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
constexpr int SDPA_KV_BLOCK = 512;
constexpr int SDPA_MAX_BLOCKS = 8;   // kv_cap <= 4096

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
#pragma unroll
            for (int o = LPK / 2; o > 0; o >>= 1) s[g] += __shfl_xor(s[g], o, 64);
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
//  * attn_pv_kernel: the chunk's p against its block's running max (known only once
//    every chunk of the block has its scores), bf16 P, partial P.V;
//  * attn_combine_kernel: l with aten's lane-ordered block sums, the partial P.V summed
//    per block, rescaled across blocks, scaled by 1/l.
constexpr int QSMAX = 4;   // q / appended-k/v projection slabs read by the decode kernel
constexpr int DCH = 64;    // keys per decode chunk

template <int D, int G>
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
    // the block whose keys include t appends the step's own key/value (a.append)
    const bool has_t = a.append && a.Qpart && t >= c0 && t < c1;
    const bf16_t* Kb = a.K + row * a.kv_bstride + kvh * a.kv_hstride;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride;
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
            col = (role == 1 ? a.k_col0 : a.v_col0) + kvh * D + 4 * c4;
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
    u32x4 kr[NIT], vr[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int j = c0 + i * KPB + wave * KPW + kg;
        const int off = j < c1 ? (j * D + 8 * dl) * 2 : (int)0x7ffffff0;
        kr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
        vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, single ? off : (int)0x7ffffff0,
                                                                              0, 0));
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
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int j = c0 + i * KPB + wave * KPW + kg;
        if (j >= c1) {
            kr[i] = (u32x4){0u, 0u, 0u, 0u};
            vr[i] = (u32x4){0u, 0u, 0u, 0u};
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
            if (single) vr[i] = vw;
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
#pragma unroll
            for (int o = LPK / 2; o > 0; o >>= 1) s[g] += __shfl_xor(s[g], o, 64);
        const int jl = i * KPB + wave * KPW + kg;
        if (dl == 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) sm[g][jl] = __fmul_rn(s[g], a.scale);
        }
    }
    __syncthreads();
    T5G_TS(2);
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
    // once (the tail's double exp included), the block sum then only chains adds
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

template <int D, int G>
__global__ __launch_bounds__(256, 2) void attn_pv_kernel(AttnArgs a) {
    constexpr int LPK = D / 8;
    constexpr int KPW = 64 / LPK;
    constexpr int KPB = KPW * 4;
    constexpr int NIT = DCH / KPB;
    constexpr int CPB = SDPA_KV_BLOCK / DCH;   // chunks per aten kv block
    __shared__ float sp_p[G][DCH];
    __shared__ float mrun[G];
    __shared__ f32x4 ored[4][G][LPK][2];
    const int qi = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int kg = lane / LPK, dl = lane % LPK;
    const int row = a.q_row ? a.q_row[qi] : qi;
    const DecRow r = dec_row(a, qi);
    if (r.span <= DCH) return;                  // finished by attn_decode_kernel
    const int c0 = r.lo + sp * DCH;
    if (c0 >= r.hi) return;
    const int c1 = min(r.hi, c0 + DCH);
    const int n = c1 - c0;
    // V rows of the chunk first (in flight while the maxima and scores are read)
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride;
    const __amdgpu_buffer_rsrc_t vrs = frag_rsrc(Vb, (uint32_t)a.kv_cap * D * 2u);
    u32x4 vr[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int j = c0 + i * KPB + wave * KPW + kg;
        const int off = j < c1 ? (j * D + 8 * dl) * 2 : (int)0x7ffffff0;
        vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0));
    }
    const int bi = sp / CPB;                                  // aten kv block of this chunk
    const int nch = (r.span + DCH - 1) / DCH;
    const int blen = min(SDPA_KV_BLOCK, r.span - bi * SDPA_KV_BLOCK);
    if (wave < G) {
        const int g = wave;
        // running max through the end of this chunk's block
        const int cend = min(nch, (bi + 1) * CPB);
        const float m = lane < cend ? a.mbuf[(((long)qi * a.Hkv + kvh) * a.nsplit + lane) * G + g] : -INFINITY;
        const float mx = wave_max(m);
        if (lane == 0) mrun[g] = mx;
        float* srow = a.sbuf + ((long)qi * a.Hkv * G + kvh * G + g) * a.kv_cap + c0;
        const float s = lane < n ? srow[lane] : 0.f;
        const int pos = c0 + lane - r.lo - bi * SDPA_KV_BLOCK;
        const float p = lane < n ? sdpa_p(__fsub_rn(s, mx), pos, blen) : 0.f;
        sp_p[g][lane] = rbf(p);
        if (lane < n) srow[lane] = p;   // the exact p replaces the score: read by the combine
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
            const float p = sp_p[g][jl];
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
    float* pbase = a.part + (((long)qi * a.Hkv + kvh) * a.nsplit + sp) * (G * (D + 2));
    for (int idx = threadIdx.x; idx < G * LPK; idx += 256) {
        const int g = idx / LPK, d8 = idx % LPK;
        const f32x4 lo4 = ored[0][g][d8][0] + ored[1][g][d8][0] + ored[2][g][d8][0] + ored[3][g][d8][0];
        const f32x4 hi4 = ored[0][g][d8][1] + ored[1][g][d8][1] + ored[2][g][d8][1] + ored[3][g][d8][1];
        float* pg = pbase + g * (D + 2);
        if (d8 == 0) pg[0] = mrun[g];
        *(f32x4*)(pg + 2 + 8 * d8) = lo4;
        *(f32x4*)(pg + 6 + 8 * d8) = hi4;
    }
}

// Each (row, kv head) is combined by CZ blocks of 64*G threads, one slice of the (g, d4)
// quads each (a single block per (row, kv head) was per-CU-bandwidth bound).
template <int D, int G>
constexpr int combine_cz() { return (G * D / 4 + 31) / 32; }

template <int D, int G>
__global__ __launch_bounds__(64 * G) void attn_combine_kernel(AttnArgs a) {
    constexpr int CPB = SDPA_KV_BLOCK / DCH;
    __shared__ float blk_et[G][SDPA_MAX_BLOCKS];
    __shared__ float stat_l[G];
    __shared__ float pl[G][SDPA_KV_BLOCK + 16];
    const int qi = blockIdx.x, kvh = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    T5G_TS(3);
    const DecRow r = dec_row(a, qi);
    if (r.span <= DCH) return;
    const int nch = (r.span + DCH - 1) / DCH;
    const int nblk = (r.span + SDPA_KV_BLOCK - 1) / SDPA_KV_BLOCK;
    // this thread's output quad, and the partial P.V sums of the first two kv blocks
    // requested now (unconditional clamped loads), so they land while l is computed
    constexpr int QPB = (G * D / 4 + combine_cz<D, G>() - 1) / combine_cz<D, G>();
    const int quad = (int)blockIdx.z * QPB + (int)threadIdx.x;
    const bool mq = (int)threadIdx.x < QPB && quad < G * D / 4;
    const int gq = mq ? quad / (D / 4) : 0, d4 = mq ? quad % (D / 4) : 0;
    const float* base = a.part + ((long)qi * a.Hkv + kvh) * a.nsplit * (G * (D + 2)) + gq * (D + 2) + 2 + 4 * d4;
    constexpr int NPRE = 2;
    f32x4 pre[NPRE];
#pragma unroll
    for (int b = 0; b < NPRE; ++b) {
        pre[b] = (f32x4){0.f, 0.f, 0.f, 0.f};
        const int ce = min(nch, (b + 1) * CPB);
#pragma unroll
        for (int k = 0; k < CPB; ++k) {
            const int c = b * CPB + k;
            const f32x4 v = *(const f32x4*)(base + (long)(c < ce ? c : 0) * G * (D + 2));
            pre[b] += (c < ce) ? v : (f32x4){0.f, 0.f, 0.f, 0.f};
        }
    }
    {   // wave g: l of head g with aten's lane-ordered block sums over the exact p values
        // attn_pv_kernel left in sbuf, staged block by block in LDS; the serial adds run
        // out of LDS
        const int g = wave;
        const float* mb = a.mbuf + ((long)qi * a.Hkv + kvh) * a.nsplit * G + g;
        const float* pb = a.sbuf + ((long)qi * a.Hkv * G + kvh * G + g) * a.kv_cap + r.lo;
        const float cmax = lane < nch ? mb[lane * G] : -INFINITY;   // chunk `lane`'s max
        // block b's p in registers (8 per lane, coalesced); the next block's loads are
        // issued before this block's serial adds
        float pw[SDPA_KV_BLOCK / 64];
#pragma unroll
        for (int k = 0; k < SDPA_KV_BLOCK / 64; ++k) {
            const int pos = 64 * k + lane;
            pw[k] = pos < r.span ? pb[pos] : 0.f;
        }
        if (lane < 16) pl[g][SDPA_KV_BLOCK + lane] = 0.f;
        float m = -INFINITY, l = 0.f;
        for (int b = 0; b < nblk; ++b) {
            __builtin_amdgcn_wave_barrier();   // the previous block's LDS reads are done
#pragma unroll
            for (int k = 0; k < SDPA_KV_BLOCK / 64; ++k) pl[g][64 * k + lane] = pw[k];
#pragma unroll
            for (int k = 0; k < SDPA_KV_BLOCK / 64; ++k) {
                const int pos = (b + 1) * SDPA_KV_BLOCK + 64 * k + lane;
                pw[k] = pos < r.span ? pb[pos] : 0.f;
            }
            __builtin_amdgcn_wave_barrier();
            const float mn = fmaxf(m, wave_max(lane / CPB == b ? cmax : -INFINITY));
            const int blen = min(SDPA_KV_BLOCK, r.span - b * SDPA_KV_BLOCK);
            const float ts = sdpa_block_sum_lds<SDPA_KV_BLOCK>(pl[g], blen, lane);
            const float et = sdpa_block_rescale(m, mn);
            l = fmaf(et, l, ts);
            if (lane == 0) blk_et[g][b] = et;
            m = mn;
        }
        if (lane == 0) stat_l[g] = l;
    }
    __syncthreads();
    if (!mq) return;
    const int g = gq;
    f32x4 dst = {0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < nblk; ++b) {
        f32x4 blk = {0.f, 0.f, 0.f, 0.f};
        if (b < NPRE) {
            blk = b == 0 ? pre[0] : pre[1];
        } else {
            const int ce = min(nch, (b + 1) * CPB);
#pragma unroll
            for (int k = 0; k < CPB; ++k) {   // predicated, not a loop-carried wait per chunk
                const int c = b * CPB + k;
                if (c < ce) blk += *(const f32x4*)(base + (long)c * G * (D + 2));
            }
        }
        dst = dst * blk_et[g][b] + blk;
    }
    const float inv = __fdiv_rn(1.0f, stat_l[g]);
    uint2 o;
    o.x = pack2(__fmul_rn(dst[0], inv), __fmul_rn(dst[1], inv));
    o.y = pack2(__fmul_rn(dst[2], inv), __fmul_rn(dst[3], inv));
    *(uint2*)(a.O + (long)qi * a.ldo + (kvh * G + g) * D + 4 * d4) = o;
    T5G_TS(6);
}

template <int D, int G>
static int launch_decode(const AttnArgs& a, hipStream_t st) {
    dim3 grid((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)a.nsplit);
    hipLaunchKernelGGL((attn_decode_kernel<D, G>), grid, dim3(256), 0, st, a);
    if (a.nsplit > 1) {
        hipLaunchKernelGGL((attn_pv_kernel<D, G>), grid, dim3(256), 0, st, a);
        hipLaunchKernelGGL((attn_combine_kernel<D, G>), dim3((unsigned)a.Mq, (unsigned)a.Hkv, combine_cz<D, G>()),
                           dim3(64 * G), 0, st, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int attention_decode(const AttnArgs& a, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (a.eager || !a.part || a.kv_cap <= 0 || a.kv_cap > SDPA_KV_BLOCK * SDPA_MAX_BLOCKS) return -1;
    if (a.nsplit != (a.kv_cap + DCH - 1) / DCH) return -1;   // 64-key chunks from the row start
    if (a.nsplit > 1 && (!a.sbuf || !a.mbuf || a.nsplit > 64)) return -1;
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

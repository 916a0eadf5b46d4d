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

__global__ void rope_table_kernel(const float* pos, const float* inv_freq, int D, float* tab, unsigned* epoch) {
    const int r = blockIdx.x, H2 = D / 2;
    // the decode step's first kernel also advances the step epoch that the PRO_LEAD row
    // hand-offs of this step publish and poll (gemv.hip): no per-step flag reset
    if (epoch && r == 0 && threadIdx.x == 0) *epoch = *epoch + 1u == 0u ? 1u : *epoch + 1u;
    for (int i = threadIdx.x; i < H2; i += blockDim.x) {
        const float ang = inv_freq[i] * pos[r];
        tab[(long)r * D + i] = rbf(cosf(ang));
        tab[(long)r * D + H2 + i] = rbf(sinf(ang));
    }
}

int rope_table(const float* pos, const float* inv_freq, int rows, int D, float* tab, hipStream_t st,
               unsigned* epoch) {
    if (rows <= 0) return 0;
    hipLaunchKernelGGL(rope_table_kernel, dim3((unsigned)rows), dim3(128), 0, st, pos, inv_freq, D, tab, epoch);
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
template <int D, int G, bool EAGER>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
    constexpr int LPK = D / 8;        // lanes per key row
    constexpr int KPW = 64 / LPK;     // keys per wave instruction
    constexpr int KPB = KPW * 4;      // keys per block iteration
    extern __shared__ __attribute__((aligned(16))) float sm[];  // [G][chunk] scores, then probs
    __shared__ float red[32];
    __shared__ f32x4 ored[4][G][64][2];

    const int qi = blockIdx.x, kvh = blockIdx.y, sp = blockIdx.z;
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
    const int c0 = lo + sp * a.chunk;
    const int c1 = min(hi, c0 + a.chunk);
    const int n = c1 - c0;

    float* part = a.part ? a.part + (((long)qi * a.Hkv + kvh) * a.nsplit + sp) * (G * (D + 2)) : nullptr;
    if (n <= 0) {
        if (a.nsplit > 1 && threadIdx.x < G) {
            part[threadIdx.x * (D + 2)] = -INFINITY;
            part[threadIdx.x * (D + 2) + 1] = 0.f;
        }
        return;
    }
    // q fragment: 8 dims per lane per head
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
    for (int j0 = c0; j0 < c1; j0 += KPB) {
        const int j = j0 + wave * KPW + kg;
        float s[G];
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] = 0.f;
        if (j < c1) {
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
        if (dl == 0 && j < c1) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float v;
                if constexpr (EAGER) {
                    v = rbf(rbf(s[g]) * a.scale);
                    if (a.softcap > 0.f) v = rbf(rbf(tanhf(rbf(v / a.softcap))) * a.softcap);
                } else {
                    v = s[g] * a.scale;
                }
                sm[g * a.chunk + (j - c0)] = v;
            }
        }
    }
    __syncthreads();
    // ---- softmax statistics
    float mx[G], sum[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float lm = -INFINITY;
        for (int i = threadIdx.x; i < n; i += 256) lm = fmaxf(lm, sm[g * a.chunk + i]);
        mx[g] = block_max(lm, red);
        float ls = 0.f;
        for (int i = threadIdx.x; i < n; i += 256) ls += expf(sm[g * a.chunk + i] - mx[g]);
        sum[g] = block_sum(ls, red);
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const float inv = 1.0f / sum[g];
        for (int i = threadIdx.x; i < n; i += 256) {
            float e = expf(sm[g * a.chunk + i] - mx[g]);
            sm[g * a.chunk + i] = EAGER ? rbf(e * inv) : rbf(e);
        }
    }
    __syncthreads();
    // ---- P.V: lane owns dims [8*dl, 8*dl+8) of key group kg
    float o[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o[g][jj] = 0.f;
    for (int j0 = c0; j0 < c1; j0 += KPB) {
        const int j = j0 + wave * KPW + kg;
        if (j < c1) {
            u32x4 w = *(const u32x4*)(Vb + (long)j * D + 8 * dl);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float p = sm[g * a.chunk + (j - c0)];
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
    // final: thread t handles (g, dl) pairs
    for (int idx = threadIdx.x; idx < G * LPK; idx += 256) {
        const int g = idx / LPK, d8 = idx % LPK;
        f32x4 lo4 = ored[0][g][d8][0] + ored[1][g][d8][0] + ored[2][g][d8][0] + ored[3][g][d8][0];
        f32x4 hi4 = ored[0][g][d8][1] + ored[1][g][d8][1] + ored[2][g][d8][1] + ored[3][g][d8][1];
        float v[8] = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
        if (a.nsplit > 1) {
            float* pg = part + g * (D + 2);
            if (d8 == 0) {
                pg[0] = mx[g];
                pg[1] = sum[g];
            }
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) pg[2 + 8 * d8 + jj] = v[jj];
        } else {
            const float inv = EAGER ? 1.0f : 1.0f / sum[g];
            u32x4 w;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) w[jj] = pack2(v[2 * jj] * inv, v[2 * jj + 1] * inv);
            *(u32x4*)(a.O + (long)qi * a.ldo + (kvh * G + g) * D + 8 * d8) = w;
        }
    }
}

// Decode-shaped attention (one query row per (row, kv head)): 64 keys per block,
// every K and V row of the block is requested before the first use (16 B per lane,
// NIT loads of each in flight), softmax statistics by one wave per head.
// Fusions: (1) q may come straight from the q-projection's fp32 split-K slabs; the
// block sums them, rounds to bf16 and applies the float-position PM-RoPE with a
// lane shuffle (rotate_half partner = lane ^ LPK/2), bit-identical to
// rope_store_kernel; (2) the key-split partials are merged in the same launch by
// the last-arriving block of each (row, kv head) (agent-scope release/acquire
// ticket, CDNA guide G16), so no combine launch.
template <int D, int G>
__device__ __forceinline__ void merge_splits(const AttnArgs& a, const float* base, int qi, int kvh, float* wz,
                                             float* Linv, int q0 = 0, int nq = G * D / 4) {
    constexpr int ZMAX = 16;  // splits held in registers; more are streamed
    const int S = a.nsplit;
    // Slabs are read with sc1 loads (L1 bypass): in the in-launch merge they were
    // written moments ago by other workgroups with sc1 (write-through) stores, the
    // CDNA guide G16 row-1 hand-off (no acquire fence needed).
    const __amdgpu_buffer_rsrc_t rs = frag_rsrc(base, (uint32_t)S * G * (D + 2) * 4u);
    auto ld4 = [&](int off) __attribute__((always_inline)) {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off * 4, 0, 16));
    };
    auto ld1 = [&](int off) __attribute__((always_inline)) {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off * 4, 0, 16));
    };
    // thread idx owns (g, d4) quad q0 + idx of this block's nq quads (all G*D/4 of them in
    // the in-launch merge; a slice of them per combine block)
    const int idx = threadIdx.x;
    const bool own = idx < nq;
    const int quad = q0 + (own ? idx : 0);
    const int g = quad / (D / 4), d4 = quad % (D / 4);
    f32x4 pv[ZMAX];
#pragma unroll
    for (int z = 0; z < ZMAX; ++z)
        if (own && z < S) pv[z] = ld4(z * G * (D + 2) + g * (D + 2) + 2 + 4 * d4);
    if (threadIdx.x < 64 * G) {
        const int gg = threadIdx.x / 64, z = threadIdx.x % 64;
        const float m = z < S ? ld1(z * G * (D + 2) + gg * (D + 2)) : -INFINITY;
        const float l = z < S ? ld1(z * G * (D + 2) + gg * (D + 2) + 1) : 0.f;
        const float M = wave_max(m);
        const float w = (m == -INFINITY) ? 0.f : expf(m - M);
        const float L = wave_sum(w * l);
        wz[gg * 64 + z] = w;
        if (z == 0) Linv[gg] = 1.0f / L;
    }
    __syncthreads();
    if (!own) return;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int z = 0; z < ZMAX; ++z)
        if (z < S) {
            const float w = wz[g * 64 + z];
            if (w != 0.f) acc += w * pv[z];
        }
    for (int z = ZMAX; z < S; ++z) {
        const float w = wz[g * 64 + z];
        if (w != 0.f) acc += w * ld4(z * G * (D + 2) + g * (D + 2) + 2 + 4 * d4);
    }
    const float inv = Linv[g];
    uint2 o;
    o.x = pack2(acc[0] * inv, acc[1] * inv);
    o.y = pack2(acc[2] * inv, acc[3] * inv);
    *(uint2*)(a.O + (long)qi * a.ldo + (kvh * G + g) * D + 4 * d4) = o;
}

constexpr int QSMAX = 4;   // q / appended-k/v projection slabs read by the decode kernel

template <int D, int G>
__global__ __launch_bounds__(256, 2) void attn_decode_kernel(AttnArgs a) {
    constexpr int CH = 64;
    constexpr int LPK = D / 8;
    constexpr int KPW = 64 / LPK;
    constexpr int KPB = KPW * 4;
    constexpr int NIT = CH / KPB;
    __shared__ float sm[G][CH];
    __shared__ float stat[G][2];
    __shared__ f32x4 ored[4][G][LPK][2];
    __shared__ float wz[G * 64];
    __shared__ float Linv[G];
    __shared__ int last_flag;
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
    // The row's keys [lo, hi) are split into nsplit equal chunks (<= CH keys each, since
    // nsplit * CH >= kv_cap): every block streams the same share whatever the row length,
    // and no block loads keys past it (the old fixed 64-key chunks streamed whole chunks
    // for blocks past the length: 31 MB instead of 17 MB per layer at L = 527). A row of
    // <= CH keys stays one chunk (one softmax pass, no merge: closest to the reference's
    // single-pass sdpa on short rows).
    const int span = max(hi - lo, 0);
    const int chunk = span <= CH ? span : (span + a.nsplit - 1) / a.nsplit;
    const int c0 = lo + sp * chunk;
    const int c1 = min(hi, c0 + chunk);
    const int n = c1 - c0;
    // the block whose keys include t appends the step's own key/value (a.append)
    const bool has_t = a.append && a.Qpart && t >= c0 && t < c1;
    const bf16_t* Kb = a.K + row * a.kv_bstride + kvh * a.kv_hstride;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride;
    // Issue order = wait order (vmcnt is in-order): first what the q path needs (the
    // projection's split-K slabs, the PM-RoPE table), then the K/V stream, so q can be
    // summed, staged and rotated while K/V are still in flight. All loads are
    // unconditional (clamped addresses): a load under a branch makes the compiler
    // wait for everything in flight at the join.
    // Thread roles in the slab stage: quads [0, G*D/4) are q, the next 2*D/4 the
    // appended k and v (block holding key t only); the rest re-read quad 0.
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
    // this lane's 8 cos / 8 sin of the row's PM-RoPE table (dims 8*dl .. 8*dl+7 never wrap
    // D/2): four 16-B loads
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
    // K/V of the block's keys, requested right behind the q slabs: buffer loads, keys
    // past c1 fall outside the descriptor (zeros, no traffic) -- no branch, so the
    // compiler keeps one in-order wait per use
    const __amdgpu_buffer_rsrc_t krs = frag_rsrc(Kb, (uint32_t)a.kv_cap * D * 2u);
    const __amdgpu_buffer_rsrc_t vrs = frag_rsrc(Vb, (uint32_t)a.kv_cap * D * 2u);
    u32x4 kr[NIT], vr[NIT];
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
        const int j = c0 + i * KPB + wave * KPW + kg;
        const int off = j < c1 ? (j * D + 8 * dl) * 2 : (int)0x7ffffff0;
        kr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
        vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0));
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
    const long pstride = (long)G * (D + 2);
    float* pbase = a.part + ((long)qi * a.Hkv + kvh) * a.nsplit * pstride;
    const __amdgpu_buffer_rsrc_t prs = frag_rsrc(pbase, (uint32_t)(a.nsplit * pstride * 4));
    if (n > 0) {
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
                vr[i] = vw;
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
                for (int g = 0; g < G; ++g) sm[g][jl] = s[g] * a.scale;
            }
        }
        __syncthreads();
        T5G_TS(2);
        if (wave < G) {
            const int g = wave;
            const float s = lane < n ? sm[g][lane] : -INFINITY;
            const float mx = wave_max(s);
            const float e = lane < n ? expf(s - mx) : 0.f;
            const float l = wave_sum(e);
            sm[g][lane] = rbf(e);
            if (lane == 0) {
                stat[g][0] = mx;
                stat[g][1] = l;
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
        T5G_TS(4);
        for (int idx = threadIdx.x; idx < G * LPK; idx += 256) {
            const int g = idx / LPK, d8 = idx % LPK;
            const f32x4 lo4 = ored[0][g][d8][0] + ored[1][g][d8][0] + ored[2][g][d8][0] + ored[3][g][d8][0];
            const f32x4 hi4 = ored[0][g][d8][1] + ored[1][g][d8][1] + ored[2][g][d8][1] + ored[3][g][d8][1];
            if (a.nsplit > 1) {
                // sc1 (write-through) slab stores: the merging block may sit on another XCD
                const int pg = sp * (int)pstride + g * (D + 2);
                if (d8 == 0) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(stat[g][0]), prs, pg * 4, 0, 16);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(stat[g][1]), prs, (pg + 1) * 4, 0, 16);
                }
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo4), prs, (pg + 2 + 8 * d8) * 4, 0, 16);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi4), prs, (pg + 6 + 8 * d8) * 4, 0, 16);
            } else {
                const float inv = 1.0f / stat[g][1];
                u32x4 w;
                w[0] = pack2(lo4[0] * inv, lo4[1] * inv);
                w[1] = pack2(lo4[2] * inv, lo4[3] * inv);
                w[2] = pack2(hi4[0] * inv, hi4[1] * inv);
                w[3] = pack2(hi4[2] * inv, hi4[3] * inv);
                *(u32x4*)(a.O + (long)qi * a.ldo + (kvh * G + g) * D + 8 * d8) = w;
            }
        }
    } else if (a.nsplit > 1 && threadIdx.x < G) {
        const int pg = sp * (int)pstride + threadIdx.x * (D + 2);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(-INFINITY), prs, pg * 4, 0, 16);
        __builtin_amdgcn_raw_buffer_store_b32(0u, prs, (pg + 1) * 4, 0, 16);
    }
    T5G_TS(5);
    if (a.nsplit == 1 || !a.counters) return;
    // ---- in-launch merge (CDNA guide G16, valid form row 1): every storing wave drains
    // its sc1 slab stores, then one lane adds to the (row, kv head) ticket; the block
    // whose add returns nsplit-1 merges, reading the slabs with sc1 loads. No fences.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int* ctr = a.counters + qi * a.Hkv + kvh;
        const int ticket = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = ticket == a.nsplit - 1;
        if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
        last_flag = last;
    }
    __syncthreads();
    if (!last_flag) return;
    T5G_TS(3);
    merge_splits<D, G>(a, pbase, qi, kvh, wz, Linv);
    T5G_TS(6);
}

// merge of the key-split partials (used when no ticket counters are supplied):
// O = sum_z e^(m_z - M) o_z / sum_z e^(m_z - M) l_z
// Each (row, kv head) is merged by CZ blocks of 64*G threads, one slice of 32 (g, d4) quads
// each: a block reads 1/CZ of the slabs, so the merge is spread over 4x the CUs (a single
// block per (row, kv head) was per-CU-bandwidth bound: 31 KB of slabs at 15 splits).
template <int D, int G>
constexpr int combine_cz() { return (G * D / 4 + 31) / 32; }

template <int D, int G>
__global__ __launch_bounds__(64 * G) void attn_combine_kernel(AttnArgs a) {
    __shared__ float wz[G * 64];
    __shared__ float Linv[G];
    const int qi = blockIdx.x, kvh = blockIdx.y;
    T5G_TS(3);
    const float* base = a.part + ((long)qi * a.Hkv + kvh) * a.nsplit * (G * (D + 2));
    constexpr int QPB = (G * D / 4 + combine_cz<D, G>() - 1) / combine_cz<D, G>();
    const int q0 = (int)blockIdx.z * QPB;
    merge_splits<D, G>(a, base, qi, kvh, wz, Linv, q0, min(QPB, G * D / 4 - q0));
    T5G_TS(6);
}

template <int D, int G>
static int launch_decode(const AttnArgs& a, hipStream_t st) {
    dim3 grid((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)a.nsplit);
    hipLaunchKernelGGL((attn_decode_kernel<D, G>), grid, dim3(256), 0, st, a);
    if (a.nsplit > 1 && !a.counters)
        hipLaunchKernelGGL((attn_combine_kernel<D, G>), dim3((unsigned)a.Mq, (unsigned)a.Hkv, combine_cz<D, G>()),
                           dim3(64 * G), 0,
                           st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int attention_decode(const AttnArgs& a, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (a.nsplit < 1 || a.nsplit > 64 || !a.part || a.eager) return -1;
    if ((long)a.nsplit * 64 < a.kv_cap || a.kv_cap <= 0) return -1;   // chunks of <= 64 keys
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
    dim3 grid((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)a.nsplit);
    size_t shm = (size_t)G * a.chunk * sizeof(float);
    if (a.eager)
        hipLaunchKernelGGL((attn_kernel<D, G, true>), grid, dim3(256), shm, st, a);
    else
        hipLaunchKernelGGL((attn_kernel<D, G, false>), grid, dim3(256), shm, st, a);
    if (a.nsplit > 1)
        hipLaunchKernelGGL((attn_combine_kernel<D, G>), dim3((unsigned)a.Mq, (unsigned)a.Hkv, combine_cz<D, G>()),
                           dim3(64 * G), 0,
                           st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int attention(const AttnArgs& a, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (a.nsplit < 1 || a.chunk < 1) return -1;
    if (a.eager && a.nsplit != 1) return -1;       // eager normalises over the full row
    if (a.nsplit > 1 && !a.part) return -1;
    if ((size_t)a.G * a.chunk * sizeof(float) > 96 * 1024) return -1;
    if (a.D == 256 && a.G == 2) return launch_attn<256, 2>(a, st);
    if (a.D == 64 && a.G == 2) return launch_attn<64, 2>(a, st);
    if (a.D == 128 && a.G == 2) return launch_attn<128, 2>(a, st);
    if (a.D == 256 && a.G == 1) return launch_attn<256, 1>(a, st);
    return -3;
}

}  // namespace t5g

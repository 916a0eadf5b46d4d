// Eager attention in the reference host's CPU order (parity mode for checkpoints with
// attn_implementation="eager", the reference default: hf_export/configuration_t5gemma_voice.py:59,
// config.py:87). [tf] eager_attention_forward (modeling_t5gemma.py:199-230):
//   w = bf16(q.k^T) ; w = bf16(w * scale) ; w = bf16(tanh(bf16(w / softcap)) * softcap) ;
//   w += finfo.min where masked ; p = bf16(softmax_fp32(w)) ; o = bf16(p.V)
// as oracle.cpu_order.eager_attention restates it (pinned bitwise on the reference's own
// 26+26-layer eager run, tests/test_cpu_order_cpu.py):
//   * the matmuls in the accumulation model oneDNN selects for the reference's call shape
//     (batch 1, 8 query heads, head_dim 256; tools/cpu_order/eager_table_2b2b.jsonl):
//     q.k^T 4 interleaved accumulators when Tq * Tk == 2, else per 32-element chunk an
//     even and an odd fmaf chain, chunk = E + O, chunks folded in order; P.V one pair chain
//     (odd product first) when Tq * Tk < 64 and (Tq == 1 or Tk even), else the E/O chunks
//     over the keys -- no K split;
//   * the softmax of aten's AVX-512 float path: Sleef expf_u10 of every (w - max), one
//     16-lane accumulator (lane j % 16, a zero-filled partial tail) reduced by the halves
//     tree, x * (1 / sum);
//   * tanh from the reference host's bf16 table (data/tanh_bf16.bin).
// Two launches: eager_scores_kernel (workgroup per (query, kv head, 64 keys): four threads
// per key, each two 32-element chunk sums, one thread folds the eight in order) writes the
// post-softcap scores; eager_pv_kernel (workgroup per (query, kv head, 32 output dims))
// recomputes the row's softmax from them and runs P.V for its slice.
#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

constexpr int EA_D = 256;      // head_dim of the measured call shape
constexpr int EA_CH = 64;      // keys per scores workgroup
constexpr int EA_DZ = 32;      // output dims per P.V workgroup
constexpr int EA_MAXK = SDPA_KV_BLOCK * SDPA_MAX_BLOCKS;   // keys per call: the engine's cache capacity

struct EaRow {
    int row, Tq, Tk, lo, abs_t;
    bool has_mask, causal_mask;
};

// the call's keys and mask, exact.hip's conventions (DynamicSlidingWindowLayer trims a
// long-enough sliding cache to its last `window` keys at decode; prefill builds the mask)
__device__ __forceinline__ EaRow ea_row(const ExactAttnArgs& a, int qi) {
    EaRow r;
    r.row = a.q_row ? a.q_row[qi] : qi;
    const int Tk_all = a.kv_len[r.row];
    r.Tq = a.q_len ? a.q_len[r.row] : 1;
    const int tq = a.q_pos ? a.q_pos[qi] : r.Tq - 1;
    r.abs_t = tq + (Tk_all - r.Tq);
    r.has_mask = a.window > 0 && Tk_all >= a.window;
    r.lo = (r.has_mask && r.Tq == 1 && a.causal) ? Tk_all - a.window : 0;
    r.Tk = Tk_all - r.lo;
    r.causal_mask = a.causal && !r.has_mask && r.Tq > 1;
    return r;
}

__device__ __forceinline__ bool ea_visible(const ExactAttnArgs& a, const EaRow& r, int key) {
    const int kabs = key + r.lo;
    if (r.has_mask) {
        if (r.Tq == 1 && a.causal) return true;
        if (a.causal) return kabs <= r.abs_t && kabs > r.abs_t - a.window;
        return abs(r.abs_t - kabs) <= a.window;
    }
    return !r.causal_mask || kabs <= r.abs_t;
}

// RoPE of one rotation pair as rope_store_kernel computes it (the three bf16 tensor ops of
// apply_rotary_pos_emb; xattn.hip xd_rope)
__device__ __forceinline__ void ea_rope(float x1, float x2, float c, float sn, float& o1, float& o2) {
    o1 = rbf(rbf(x1 * c) + rbf(-x2 * sn));
    o2 = rbf(rbf(x2 * c) + rbf(x1 * sn));
}

// stage the G query rows of kv head kvh into qs; with a.rope_tab they arrive un-rotated and
// are rotated here (decode: the step's per-row cos / sin table)
template <int G>
__device__ __forceinline__ void ea_stage_q(const ExactAttnArgs& a, const EaRow& r, int qi, int kvh, float (&qs)[G][256]) {
    constexpr int H2 = 128;
    const int tid = threadIdx.x;
    if (a.rope_tab) {
        const float* tab = a.rope_tab + (long)r.row * 256;
        for (int i = tid; i < G * H2; i += 256) {
            const int g = i / H2, d = i % H2;
            const bf16_t* qh = a.Q + (long)qi * a.ldq + (kvh * G + g) * 256;
            float o1, o2;
            ea_rope(bf2f(qh[d]), bf2f(qh[d + H2]), tab[d], tab[H2 + d], o1, o2);
            qs[g][d] = o1;
            qs[g][d + H2] = o2;
        }
    } else {
        for (int i = tid; i < G * 256; i += 256) {
            const int g = i / 256, d = i % 256;
            qs[g][d] = bf2f(a.Q[(long)qi * a.ldq + (kvh * G + g) * 256 + d]);
        }
    }
}

// Sleef_expf16_u10 (sleefsimdsp.c xexpf; aten Vectorized<float>::exp) for d <= 0
__device__ __forceinline__ float ea_sleef_expf(float d) {
    if (d < -104.f) return 0.f;
    const float q = rintf(__fmul_rn(d, 1.442695040888963407359924681001892137426645954152985934135449406931f));
    float s = fmaf(q, -0.693145751953125f, d);
    s = fmaf(q, -1.428606765330187045e-06f, s);
    float u = 0.000198527617612853646278381f;
    u = fmaf(u, s, 0.00139304355252534151077271f);
    u = fmaf(u, s, 0.00833336077630519866943359f);
    u = fmaf(u, s, 0.0416664853692054748535156f);
    u = fmaf(u, s, 0.166666671633720397949219f);
    u = fmaf(u, s, 0.5f);
    u = __fadd_rn(1.0f, fmaf(__fmul_rn(s, s), u, s));
    const int qi = (int)q, e1 = qi >> 1;
    u = __fmul_rn(u, __int_as_float((e1 + 127) << 23));
    return __fmul_rn(u, __int_as_float((qi - e1 + 127) << 23));
}

// the two 32-element chunk sums (E + O chains over dims) of thread qa's quarter of key kl's
// row, for the G heads, into cs[g][kl][2 qa], [2 qa + 1]
template <int G>
__device__ __forceinline__ void ea_chunk_sums(const float (&qs)[G][EA_D], const u32x4 (&kv)[8],
                                              float (&cs)[G][EA_CH][9], int kl, int qa) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int cc = 0; cc < 2; ++cc) {
            const int c = 2 * qa + cc;
            // chunk c = dims 32 c .. 32 c + 31 = kv[4 cc .. 4 cc + 3]; pair i of word w holds
            // dims 32 c + 8 w + 2 i (lo) and + 1 (hi)
            float e = 0.f, o = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t kw = kv[4 * cc + w][i];
                    const int dd = 32 * c + 8 * w + 2 * i;
                    if (w == 0 && i == 0) {
                        e = __fmul_rn(qs[g][dd], bf_lo(kw));
                        o = __fmul_rn(qs[g][dd + 1], bf_hi(kw));
                    } else {
                        e = fmaf(qs[g][dd], bf_lo(kw), e);
                        o = fmaf(qs[g][dd + 1], bf_hi(kw), o);
                    }
                }
            cs[g][kl][c] = __fadd_rn(e, o);
        }
    }
}

// key `key`'s post-softcap score for one head from its 8 chunk sums (or, when the call is
// Tq * Tk == 2, the 4-accumulator order over the 256 dims)
__device__ __forceinline__ float ea_score(const ExactAttnArgs& a, const EaRow& r, const float* q, const bf16_t* kb,
                                          int key, const float* csk) {
    float s;
    if (r.Tq * r.Tk == 2) {
        const bf16_t* kk = kb + (long)key * EA_D;
        float ac[4] = {0.f, 0.f, 0.f, 0.f};
        for (int d = 0; d < EA_D; ++d) ac[d & 3] = fmaf(q[d], bf2f(kk[d]), ac[d & 3]);
        s = __fadd_rn(__fadd_rn(__fadd_rn(ac[0], ac[1]), ac[2]), ac[3]);
    } else {
        s = csk[0];
#pragma unroll
        for (int c = 1; c < 8; ++c) s = __fadd_rn(s, csk[c]);
    }
    float w = rbf(s);
    w = rbf(__fmul_rn(w, a.scale));
    if (a.softcap > 0.f) {
        w = rbf(__fdiv_rn(w, a.softcap));
        w = bf2f(a.tanh_lut[__float_as_uint(w) >> 16]);
        w = rbf(__fmul_rn(w, a.softcap));
    }
    return w;
}

template <int G>
__global__ __launch_bounds__(256) void eager_scores_kernel(ExactAttnArgs a, float* sbuf, int cap) {
    __shared__ float qs[G][EA_D];
    __shared__ float cs[G][EA_CH][9];   // chunk sums [head][key][chunk] (padded)
    const int qi = blockIdx.x, kvh = blockIdx.y, ch = blockIdx.z, tid = threadIdx.x;
    const int kl = tid >> 2, qa = tid & 3;
    const EaRow r = ea_row(a, qi);
    const int c0 = ch * EA_CH;
    if (c0 >= r.Tk) return;
    const int key = c0 + kl;
    const bool valid = key < r.Tk;
    const bf16_t* kb = a.K + r.row * a.kv_bstride + kvh * a.kv_hstride + (long)r.lo * EA_D;
    // this thread's 64 dims of its key (chunks 2 qa, 2 qa + 1)
    u32x4 kv[8];
    const bf16_t* kr = kb + (long)(valid ? key : c0) * EA_D + 64 * qa;
#pragma unroll
    for (int i = 0; i < 8; ++i) kv[i] = *(const u32x4*)(kr + 8 * i);
    ea_stage_q<G>(a, r, qi, kvh, qs);
    // decode self attention (kv_new, with rope_tab): the workgroup holding the row's new key
    // (the call's last key) rotates it, appends K and V to the cache and uses the rotated key
    // directly -- xattn.hip's fused form, so no separate RoPE launch
    __shared__ uint32_t knew[EA_D / 2];
    const bool has_new = a.kv_new && a.rope_tab && r.Tk - 1 >= c0 && r.Tk - 1 < c0 + EA_CH;
    if (has_new) {
        constexpr int H2 = EA_D / 2;
        const float* tab = a.rope_tab + (long)r.row * EA_D;
        const long slot = r.lo + r.Tk - 1;
        const bf16_t* kn = a.kv_new + (long)qi * a.ld_new + a.k_col0 + kvh * EA_D;
        const bf16_t* vn = a.kv_new + (long)qi * a.ld_new + a.v_col0 + kvh * EA_D;
        bf16_t* kc = (bf16_t*)a.K + r.row * a.kv_bstride + kvh * a.kv_hstride + slot * EA_D;
        bf16_t* vc = (bf16_t*)a.V + r.row * a.kv_bstride + kvh * a.kv_hstride + slot * EA_D;
        for (int d = tid; d < H2; d += 256) {
            float o1, o2;
            ea_rope(bf2f(kn[d]), bf2f(kn[d + H2]), tab[d], tab[H2 + d], o1, o2);
            kc[d] = f2bf(o1);
            kc[d + H2] = f2bf(o2);
            ((bf16_t*)knew)[d] = f2bf(o1);
            ((bf16_t*)knew)[d + H2] = f2bf(o2);
        }
        for (int d = tid; d < EA_D; d += 256) vc[d] = vn[d];
    }
    __syncthreads();
    if (has_new && key == r.Tk - 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) kv[i] = *(const u32x4*)&knew[32 * qa + 4 * i];
    }
    ea_chunk_sums<G>(qs, kv, cs, kl, qa);
    __syncthreads();
    if (qa != 0 || !valid) return;
    const bool vis = ea_visible(a, r, key);
#pragma unroll
    for (int g = 0; g < G; ++g)
        sbuf[((long)qi * a.Hq + kvh * G + g) * cap + key] = vis ? ea_score(a, r, qs[g], kb, key, cs[g][kl]) : -INFINITY;
}

// softmax + P.V of one (query, kv head, 32-dim slice) from the G post-softcap score rows
// in LDS pb [G][Tk] (-inf: masked); writes the slice of the G heads' outputs
template <int G>
__device__ __forceinline__ void ea_softmax_pv(const ExactAttnArgs& a, const EaRow& r, float* pb, int qi, int kvh,
                                              int z) {
    constexpr int NDP = EA_DZ / 2;            // dimension pairs of the slice (16)
    constexpr int NCL = 256 / NDP;            // chunk lanes (16)
    __shared__ float cs[NCL][G][EA_DZ + 1];   // chunk sums of one round [chunk lane][head][dim]
    __shared__ uint32_t vs[64][NDP];          // pair chain (< 64 keys): the slice's V rows
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int Tk = r.Tk;
    // ---- softmax of each head's row (wave g): max, Sleef exp, 16-lane sum, x (1 / sum)
    if (wave < G) {
        float* p = pb + wave * Tk;
        float m = -INFINITY;
        for (int j = lane; j < Tk; j += 64) m = fmaxf(m, p[j]);
        m = wave_max(m);
        for (int j = lane; j < Tk; j += 64) {
            const float w = p[j];
            p[j] = w == -INFINITY ? 0.f : ea_sleef_expf(__fsub_rn(w, m));
        }
        __builtin_amdgcn_wave_barrier();
        float sum;
        if (Tk < 16) {
            sum = p[0];
            for (int j = 1; j < Tk; ++j) sum = __fadd_rn(sum, p[j]);
        } else {
            const int n16 = Tk - Tk % 16;
            float acc = 0.f;
            if (lane < 16) {
                acc = p[lane];
                int j = 16 + lane;
                // 8 values per LDS round trip, added in order
                for (; j + 7 * 16 < n16; j += 8 * 16) {
                    float t[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) t[u] = p[j + 16 * u];
#pragma unroll
                    for (int u = 0; u < 8; ++u) acc = __fadd_rn(acc, t[u]);
                }
                for (; j < n16; j += 16) acc = __fadd_rn(acc, p[j]);
                if (lane < Tk - n16) acc = __fadd_rn(acc, p[n16 + lane]);
            }
            acc = __fadd_rn(acc, xlane<8>(acc));
            acc = __fadd_rn(acc, xlane<4>(acc));
            acc = __fadd_rn(acc, xlane<2>(acc));
            acc = __fadd_rn(acc, xlane<1>(acc));
            sum = __shfl(acc, 0, 64);
        }
        const float inv = __fdiv_rn(1.0f, sum);
        __builtin_amdgcn_wave_barrier();
        for (int j = lane; j < Tk; j += 64) p[j] = rbf(__fmul_rn(p[j], inv));
    }
    __syncthreads();
    // ---- P.V: thread (dimension pair dp, chunk lane cl) for both heads (they share V)
    const int dp = tid % NDP, cl = tid / NDP;
    const int d0 = z * EA_DZ + 2 * dp;
    const bf16_t* vb = a.V + r.row * a.kv_bstride + kvh * a.kv_hstride + (long)r.lo * EA_D + d0;
    const bool pair = r.Tq * Tk < 64 && (r.Tq == 1 || Tk % 2 == 0);
    float tot[G][2];
    if (pair) {
        // the slice's V rows (< 64 keys x 16 bf16 pairs) into LDS in one pass, then one
        // chain per dimension pair reads them
        {
            const bf16_t* vs0 = a.V + r.row * a.kv_bstride + kvh * a.kv_hstride + (long)r.lo * EA_D + z * EA_DZ;
            for (int i = tid; i < Tk * NDP; i += 256) {
                const int k = i / NDP, q2 = i % NDP;
                vs[k][q2] = *(const uint32_t*)(vs0 + (long)k * EA_D + 2 * q2);
            }
        }
        __syncthreads();
        if (cl == 0) {
            float acc[G][2] = {};
            for (int k = 0; k < Tk; k += 2) {
                if (k + 1 < Tk) {
                    const uint32_t w = vs[k + 1][dp];
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        acc[g][0] = fmaf(pb[g * Tk + k + 1], bf_lo(w), acc[g][0]);
                        acc[g][1] = fmaf(pb[g * Tk + k + 1], bf_hi(w), acc[g][1]);
                    }
                }
                const uint32_t w = vs[k][dp];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    acc[g][0] = fmaf(pb[g * Tk + k], bf_lo(w), acc[g][0]);
                    acc[g][1] = fmaf(pb[g * Tk + k], bf_hi(w), acc[g][1]);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                tot[g][0] = acc[g][0];
                tot[g][1] = acc[g][1];
            }
        }
    } else {
        const int nch = (Tk + 31) / 32;
        for (int r0 = 0; r0 < nch; r0 += NCL) {
            const int c = r0 + cl;
            if (c < nch) {
                const int k0 = 32 * c, n = min(32, Tk - k0);
                uint32_t vw[32];
#pragma unroll
                for (int t = 0; t < 32; ++t) vw[t] = *(const uint32_t*)(vb + (long)(k0 + min(t, n - 1)) * EA_D);
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const float* pg = pb + g * Tk + k0;
                    float e0 = __fmul_rn(pg[0], bf_lo(vw[0])), e1 = __fmul_rn(pg[0], bf_hi(vw[0]));
                    float o0 = 0.f, o1 = 0.f;
                    if (n > 1) {
                        o0 = __fmul_rn(pg[1], bf_lo(vw[1]));
                        o1 = __fmul_rn(pg[1], bf_hi(vw[1]));
                    }
#pragma unroll
                    for (int t = 2; t < 32; ++t) {
                        if (t < n) {
                            const float pt = pg[t];
                            if (t & 1) {
                                o0 = fmaf(pt, bf_lo(vw[t]), o0);
                                o1 = fmaf(pt, bf_hi(vw[t]), o1);
                            } else {
                                e0 = fmaf(pt, bf_lo(vw[t]), e0);
                                e1 = fmaf(pt, bf_hi(vw[t]), e1);
                            }
                        }
                    }
                    cs[cl][g][2 * dp] = __fadd_rn(e0, o0);
                    cs[cl][g][2 * dp + 1] = __fadd_rn(e1, o1);
                }
            }
            __syncthreads();
            if (cl == 0) {
                for (int u = 0; u < NCL && r0 + u < nch; ++u)
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int h = 0; h < 2; ++h)
                            tot[g][h] = (r0 + u == 0) ? cs[u][g][2 * dp + h] : __fadd_rn(tot[g][h], cs[u][g][2 * dp + h]);
            }
            __syncthreads();
        }
    }
    if (cl == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int col = (kvh * G + g) * EA_D + d0 + h;
                const bf16_t ob = f2bf(tot[g][h]);
                a.O[(long)qi * a.ldo + col] = ob;
                if (a.O16) a.O16[x16_off(qi, col, a.ldo / 32)] = ob;
            }
    }
}

template <int G>
__global__ __launch_bounds__(256) void eager_pv_kernel(ExactAttnArgs a, const float* sbuf, int cap) {
    extern __shared__ __attribute__((aligned(16))) float ea_smem[];
    float* pb = ea_smem;                      // [G][Tk]: scores, then e, then bf16-rounded p
    const int qi = blockIdx.x, kvh = blockIdx.y, z = blockIdx.z, tid = threadIdx.x;
    const EaRow r = ea_row(a, qi);
    const int Tk = r.Tk;
    if (Tk <= 0) return;
    // the G score rows into LDS in one coalesced pass
    for (int i = tid; i < G * Tk; i += 256) {
        const int g = i / Tk, j = i - g * Tk;
        pb[i] = sbuf[((long)qi * a.Hq + kvh * G + g) * cap + j];
    }
    __syncthreads();
    ea_softmax_pv<G>(a, r, pb, qi, kvh, z);
}

// Decode rows of <= 64 keys (the cross attention over the text): scores, softmax and P.V in
// ONE launch -- workgroup (row, kv head, 32-dim slice) computes the row's scores itself (the
// scores kernel's code; the slices of a row share an XCD, so K comes from its L2) into LDS.
template <int G>
__global__ __launch_bounds__(256) void eager_single_kernel(ExactAttnArgs a) {
    __shared__ float qs[G][EA_D];
    __shared__ float cs[G][EA_CH][9];
    __shared__ float pb[G * EA_CH];
    const int qi = blockIdx.x, kvh = blockIdx.y, z = blockIdx.z, tid = threadIdx.x;
    const int kl = tid >> 2, qa = tid & 3;
    const EaRow r = ea_row(a, qi);
    if (r.Tk <= 0) return;
    const bool valid = kl < r.Tk;
    const bf16_t* kb = a.K + r.row * a.kv_bstride + kvh * a.kv_hstride + (long)r.lo * EA_D;
    u32x4 kv[8];
    const bf16_t* kr = kb + (long)(valid ? kl : 0) * EA_D + 64 * qa;
#pragma unroll
    for (int i = 0; i < 8; ++i) kv[i] = *(const u32x4*)(kr + 8 * i);
    ea_stage_q<G>(a, r, qi, kvh, qs);
    __syncthreads();
    ea_chunk_sums<G>(qs, kv, cs, kl, qa);
    __syncthreads();
    if (qa == 0 && valid) {
        const bool vis = ea_visible(a, r, kl);
#pragma unroll
        for (int g = 0; g < G; ++g) pb[g * r.Tk + kl] = vis ? ea_score(a, r, qs[g], kb, kl, cs[g][kl]) : -INFINITY;
    }
    __syncthreads();
    ea_softmax_pv<G>(a, r, pb, qi, kvh, z);
}

int eager_attention(const ExactAttnArgs& a, float* sbuf, int cap, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (!a.Q || !a.K || !a.V || !a.kv_len || !a.O || !sbuf || !a.tanh_lut) return -1;
    // the measured call shape (tools/cpu_order/eager_table_2b2b.jsonl): 8 query heads of 256
    if (a.D != EA_D || a.Hq != 8 || a.Hq % a.Hkv || cap <= 0 || cap > EA_MAXK) return -3;
    const int G = a.Hq / a.Hkv;
    // span_max (host bound on every row's keys, 0: cap) sizes the scores grid and the P.V
    // launch's LDS rows (G x keys fp32: 96 KiB at 12 288 keys)
    const int span_max = a.span_max > 0 ? min(a.span_max, cap) : cap;
    const dim3 gs((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)((span_max + EA_CH - 1) / EA_CH));
    const dim3 gp((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)(EA_D / EA_DZ));
    const size_t shm = (size_t)G * span_max * sizeof(float);
    if ((a.rope_tab || a.kv_new) && (a.q_pos || a.q_len)) return -1;   // the fused RoPE / append: decode only
    if (a.kv_new && !a.rope_tab) return -1;
    if (!a.q_pos && !a.q_len && span_max <= EA_CH && !a.kv_new) {   // decode rows of <= 64 keys: one launch
        if (G == 2) hipLaunchKernelGGL(eager_single_kernel<2>, gp, dim3(256), 0, st, a);
        else if (G == 1) hipLaunchKernelGGL(eager_single_kernel<1>, gp, dim3(256), 0, st, a);
        else return -3;
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    if (G == 2) {
        const int dev = t5g_cur_device();
        if (dev < 0) return -2;
        static bool attr[T5G_MAX_DEVICES] = {};   // function attributes are per device
        if (!attr[dev]) {
            (void)hipFuncSetAttribute((const void*)eager_pv_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)(2 * EA_MAXK * sizeof(float)));
            attr[dev] = true;
        }
        hipLaunchKernelGGL(eager_scores_kernel<2>, gs, dim3(256), 0, st, a, sbuf, cap);
        hipLaunchKernelGGL(eager_pv_kernel<2>, gp, dim3(256), shm, st, a, sbuf, cap);
    } else if (G == 1) {
        hipLaunchKernelGGL(eager_scores_kernel<1>, gs, dim3(256), 0, st, a, sbuf, cap);
        hipLaunchKernelGGL(eager_pv_kernel<1>, gp, dim3(256), shm, st, a, sbuf, cap);
    } else {
        return -3;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

// Exact-order decode attention (parity mode, one query per row): two launches instead of
// exact.hip's one workgroup per (row, q head, 32-dim slice) that recomputed every score
// eight times.
//
// The reference's decode step calls F.scaled_dot_product_attention with one query
// ([tf] T5GemmaSelfAttention :264-304, PMCrossAttention :167-253); aten's CPU flash
// attention then runs oneDNN's gemv for q.k and P.V:
//   q.k: 16 lane accumulators, lane l taking the pair (2l, 2l+1) of every 32-element chunk,
//        odd product first, then l + l^8, adjacent pairs, adjacent pairs, the last pair;
//   softmax per 512-key block against the running max (common.h sdpa_*);
//   P.V: groups of 8 keys, each a fresh pair-ordered chain (odd key first), added in
//        group order onto the (rescaled) output.
// * xattn_scores_kernel: one wave per (row, kv head, 64-key chunk); a lane per key computes
//   the scores of the G query heads in the gemv order (the 16 accumulators in registers,
//   the q rows broadcast from LDS), writes them and the chunk maxima.
// * xattn_pv_kernel: per (row, kv head, 32-dim slice): running maxima from the chunk
//   maxima, exact p of each block, aten's block sums, the 8-key group chains of its slice
//   in parallel (16 group lanes x 16 dimension pairs), then the group sums folded in order
//   by one thread per (head, dimension); output x 1/l, also written in the X16 layout of
//   the o-projection (xmm.hip).
#include "common.h"
#include "exact_dev.h"
#include "t5g_kernels.h"

namespace t5g {

constexpr int XD_CH = 64;    // keys per scores workgroup
constexpr int XD_DZ = 32;    // output dims per P.V workgroup

// keys [lo, hi) of a decode query (the sdpa call's keys: a sliding-window layer whose
// cache is at least `window` long sees its last `window` keys, DynamicSlidingWindowLayer)
__device__ __forceinline__ void xd_range(const ExactAttnArgs& a, int row, int& lo, int& hi) {
    hi = a.kv_len[row];
    lo = (a.window > 0 && a.causal && hi >= a.window) ? hi - a.window : 0;
}

// FUSE: the queries arrive un-rotated and are rotated while staged (rope_tab), and, with
// kv_new, the workgroup holding the row's new key (slot kv_len - 1) rotates it, appends it
// and its value to the cache and uses the rotated key directly (no separate RoPE launch).
// Four threads per key (t = 4 key + qa): thread qa keeps the gemv's lane accumulators
// l2 = 4 qa .. 4 qa + 3 (its 16-byte slice of every 32-element chunk of the key's row) and
// chains them over the chunks; the hadd tree (l2 + l2 ^ 8, adjacent pairs, pairs, last
// pair) then takes two exchanges inside the quad -- the oneDNN gemv's adds in its order.
template <int G, int XD_D, bool FUSE>
__global__ __launch_bounds__(256) void xattn_scores_kernel(ExactAttnArgs a, float* sbuf, float* mbuf, int cap,
                                                           int nsplit) {
    constexpr int H2 = XD_D / 2, NCB = XD_D / 32;
    __shared__ float qs[G][XD_D];
    __shared__ uint32_t knew[FUSE ? XD_D / 2 : 1];   // the rotated new key as bf16 pairs
    __shared__ float wmax[4][G];
    const int qi = blockIdx.x, kvh = blockIdx.y, ch = blockIdx.z, tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6, kl = tid >> 2, qa = tid & 3;
    const int row = a.q_row ? a.q_row[qi] : qi;
    int lo, hi;
    xd_range(a, row, lo, hi);
    const int c0 = lo + ch * XD_CH;
    if (c0 >= hi) return;
    const int key = c0 + kl;
    const bool valid = key < hi;
    const bf16_t* kr = a.K + row * a.kv_bstride + kvh * a.kv_hstride + (long)(valid ? key : c0) * XD_D + 8 * qa;
    u32x4 kv[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) kv[cb] = *(const u32x4*)(kr + 32 * cb);
    // the G query rows of this kv head (GQA: heads kvh * G + g), broadcast from LDS
    if constexpr (FUSE) {
        const float* tab = a.rope_tab + (long)row * XD_D;
        for (int i = tid; i < G * H2; i += 256) {
            const int g = i / H2, d = i % H2;
            const bf16_t* qh = a.Q + (long)qi * a.ldq + (kvh * G + g) * XD_D;
            float o1, o2;
            xd_rope(bf2f(qh[d]), bf2f(qh[d + H2]), tab[d], tab[H2 + d], o1, o2);
            qs[g][d] = o1;
            qs[g][d + H2] = o2;
        }
        // the workgroup holding the new key: rotate it, append K and V
        const bool has_new = a.kv_new && hi - 1 >= c0 && hi - 1 < c0 + XD_CH;
        if (has_new) {
            const long slot = hi - 1;
            const bf16_t* kn = a.kv_new + (long)qi * a.ld_new + a.k_col0 + kvh * XD_D;
            const bf16_t* vn = a.kv_new + (long)qi * a.ld_new + a.v_col0 + kvh * XD_D;
            bf16_t* kc = (bf16_t*)a.K + row * a.kv_bstride + kvh * a.kv_hstride + slot * XD_D;
            bf16_t* vc = (bf16_t*)a.V + row * a.kv_bstride + kvh * a.kv_hstride + slot * XD_D;
            for (int d = tid; d < H2; d += 256) {
                float o1, o2;
                xd_rope(bf2f(kn[d]), bf2f(kn[d + H2]), tab[d], tab[H2 + d], o1, o2);
                kc[d] = f2bf(o1);
                kc[d + H2] = f2bf(o2);
                ((bf16_t*)knew)[d] = f2bf(o1);
                ((bf16_t*)knew)[d + H2] = f2bf(o2);
            }
            for (int d = tid; d < XD_D; d += 256) vc[d] = vn[d];
        }
        __syncthreads();
        if (has_new && key == hi - 1) {
#pragma unroll
            for (int cb = 0; cb < NCB; ++cb) kv[cb] = *(const u32x4*)&knew[cb * 16 + 4 * qa];
        }
    } else {
        for (int i = tid; i < G * XD_D / 2; i += 256) {
            const int g = i / (XD_D / 2), p = i % (XD_D / 2);
            const uint32_t w = *(const uint32_t*)(a.Q + (long)qi * a.ldq + (kvh * G + g) * XD_D + 2 * p);
            qs[g][2 * p] = bf_lo(w);
            qs[g][2 * p + 1] = bf_hi(w);
        }
        __syncthreads();
    }
    float sc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};   // lane accumulators l2 = 4 qa + i
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
            const float* qc = &qs[g][cb * 32 + 8 * qa];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t kw = kv[cb][i];
                acc[i] = fmaf(qc[2 * i + 1], bf_hi(kw), acc[i]);
                acc[i] = fmaf(qc[2 * i], bf_lo(kw), acc[i]);
            }
        }
        // v8[l2] = acc[l2] + acc[l2 + 8] (partner quad lane qa ^ 2), on lanes qa = 0, 1
        float v8[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v8[i] = __fadd_rn(acc[i], xlane<2>(acc[i]));
        // v4: lane 0 holds v8[0..3] -> v4[0], v4[1]; lane 1 holds v8[4..7] -> v4[2], v4[3]
        const float va = __fadd_rn(__fadd_rn(v8[0], v8[1]), __fadd_rn(v8[2], v8[3]));
        // (v4[0] + v4[1]) + (v4[2] + v4[3]) on lane qa = 0
        sc[g] = __fmul_rn(__fadd_rn(va, xlane<1>(va)), a.scale);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const bool own = valid && qa == 0;
        const float s = own ? sc[g] : -INFINITY;
        if (own) sbuf[((long)qi * a.Hq + kvh * G + g) * cap + (key - lo)] = s;
        const float mx = wave_max(s);
        if (lane == 0) wmax[wave][g] = mx;
    }
    __syncthreads();
    if (tid < G)
        mbuf[(((long)qi * a.Hkv + kvh) * nsplit + ch) * G + tid] =
            fmaxf(fmaxf(wmax[0][tid], wmax[1][tid]), fmaxf(wmax[2][tid], wmax[3][tid]));
}

// Round 6 schedule (the same operations in the same order as round 5's, bitwise): every
// global read the workgroup needs for the first two 512-key blocks -- the chunk maxima, the
// V rows of its 32-dimension slice, its scores -- is issued at once, right after the row
// length, so one memory round trip precedes the arithmetic instead of three in sequence
// (chunk maxima -> V -> scores, the scores waiting behind V in issue order). V comes in as
// 16-byte words: lane (group gl = tid / 4 of the block, 8-dimension slice tid % 4) holds
// the 8 keys of its group, 4x fewer load instructions than 4-byte words. Blocks past the
// second load at the top of their own iteration.
template <int G, int XD_D>
__global__ __launch_bounds__(256) void xattn_pv_kernel(ExactAttnArgs a, const float* sbuf, const float* mbuf,
                                                       int cap, int nsplit) {
    constexpr int BLK = SDPA_KV_BLOCK;           // 512
    constexpr int NGRP = BLK / 8;                // 8-key groups per block (64: one per lane quad)
    constexpr int PPT = BLK / 256;               // block positions per thread (2)
    static_assert(NGRP * 4 == 256 && XD_DZ == 32, "lane map: 64 groups x 4 eight-dimension slices");
    __shared__ float pex[G][BLK + 16];           // exact p (block sums)
    __shared__ float pbf[G][BLK];                // bf16-rounded p (P.V)
    __shared__ float tmp[NGRP][G][XD_DZ];        // group chain sums of the block
    __shared__ float mrun[G][SDPA_MAX_BLOCKS];
    __shared__ float et_s[G], l_s[G];
    const int qi = blockIdx.x, kvh = blockIdx.y, z = blockIdx.z, tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int row = a.q_row ? a.q_row[qi] : qi;
    int lo, hi;
    xd_range(a, row, lo, hi);
    const int span = max(hi - lo, 0);
    if (span == 0) return;
    const int nch = (span + XD_CH - 1) / XD_CH;
    const int nblk = (span + BLK - 1) / BLK;
    const float* sb = sbuf + ((long)qi * a.Hq + kvh * G) * cap;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride + (long)lo * XD_D + z * XD_DZ;
    const int d8 = tid & 3, gl = tid >> 2;       // P.V role: 8-key group gl, dims 8 d8 .. 8 d8 + 7
    const float* mb_row = mbuf + ((long)qi * a.Hkv + kvh) * nsplit * G;
    // ---- every read up front (unconditional: clamped addresses, so the waits stay exact)
    const int gm = wave < G ? wave : G - 1;
    float cmx[(SDPA_MAX_BLOCKS * (BLK / XD_CH) + 63) / 64];
    constexpr int NCM = (SDPA_MAX_BLOCKS * (BLK / XD_CH) + 63) / 64;
#pragma unroll
    for (int i = 0; i < NCM; ++i) cmx[i] = mb_row[min(lane + 64 * i, nch - 1) * G + gm];
    auto vload = [&](u32x4 (&v)[8], int b) {
        const int bs = b * BLK, blen = min(BLK, span - bs);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *(const u32x4*)(Vb + (long)(bs + min(gl * 8 + j, blen - 1)) * XD_D + 8 * d8);
    };
    auto sload = [&](float (&sv)[G][PPT], int b) {
        const int bs = b * BLK, blen = min(BLK, span - bs);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int i = 0; i < PPT; ++i) sv[g][i] = sb[(long)g * cap + bs + min(tid + 256 * i, blen - 1)];
    };
    u32x4 v0[8], v1[8];
    float s0[G][PPT], s1[G][PPT];
    const int b1 = min(1, nblk - 1);
    vload(v0, 0);
    sload(s0, 0);
    vload(v1, b1);
    sload(s1, b1);
    if (wave < G) {   // running max through each block, from the chunk maxima
        const int g = wave;
        float run = -INFINITY;
        for (int b = 0; b < nblk; ++b) {
            float cm = -INFINITY;
#pragma unroll
            for (int i = 0; i < NCM; ++i) {
                const int c = lane + 64 * i;
                if (c >= b * (BLK / XD_CH) && c < min(nch, (b + 1) * (BLK / XD_CH))) cm = fmaxf(cm, cmx[i]);
            }
            run = fmaxf(run, wave_max(cm));
            if (lane == 0) mrun[g][b] = run;
        }
        if (lane < 16) pex[g][BLK + lane] = 0.f;
    }
    float l = 0.f, m_old = -INFINITY;            // wave g < G: head g's running sum
    float dst = 0.f;                             // folder (g, dim) = tid < G * XD_DZ
    const int fg = tid / XD_DZ, fd = tid % XD_DZ;
    __syncthreads();
    for (int b = 0; b < nblk; ++b) {
        const int bs = b * BLK, blen = min(BLK, span - bs);
        u32x4 vb[8];
        float sv[G][PPT];
        if (b == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) vb[j] = v0[j];
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int i = 0; i < PPT; ++i) sv[g][i] = s0[g][i];
        } else if (b == 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) vb[j] = v1[j];
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int i = 0; i < PPT; ++i) sv[g][i] = s1[g][i];
        } else {
            vload(vb, b);
            sload(sv, b);
        }
        // exact p of the block's keys
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float mb = mrun[g][b];
#pragma unroll
            for (int i = 0; i < PPT; ++i) {
                const int pos = tid + 256 * i;
                const float p = pos < blen ? sdpa_p(__fsub_rn(sv[g][i], mb), pos, blen) : 0.f;
                pex[g][pos] = p;
                pbf[g][pos] = rbf(p);
            }
        }
        __syncthreads();
        if (wave < G) {
            const int g = wave;
            const float ts = sdpa_block_sum_lds<BLK>(pex[g], blen, lane);
            const float mb = mrun[g][b];
            const float et = sdpa_block_rescale(m_old, mb);
            l = fmaf(et, l, ts);
            m_old = mb;
            if (lane == 0) et_s[g] = et;
        }
        // the 8-key group chain of group gl over dims 8 d8 .. 8 d8 + 7: pairs, odd key
        // first (keys past the block count 0 and add nothing: the chain stops there)
        const int ngrp = (blen + 7) / 8;
        if (gl < ngrp) {
            const int k0 = gl * 8, cn = min(8, blen - k0);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                float t[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) t[i] = 0.f;
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    if (j < cn) {
                        if (j + 1 < cn) {
                            const float p1 = pbf[g][k0 + j + 1];
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                t[2 * q] = fmaf(p1, bf_lo(vb[j + 1][q]), t[2 * q]);
                                t[2 * q + 1] = fmaf(p1, bf_hi(vb[j + 1][q]), t[2 * q + 1]);
                            }
                        }
                        const float p0 = pbf[g][k0 + j];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            t[2 * q] = fmaf(p0, bf_lo(vb[j][q]), t[2 * q]);
                            t[2 * q + 1] = fmaf(p0, bf_hi(vb[j][q]), t[2 * q + 1]);
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) tmp[gl][g][8 * d8 + i] = t[i];
            }
        }
        __syncthreads();
        if (tid < G * XD_DZ) {
            float acc = bs == 0 ? 0.f : __fmul_rn(dst, et_s[fg]);
            // 16 group sums read per batch (one LDS round trip), then added in order
            for (int g0 = 0; g0 < ngrp; g0 += 16) {
                float t[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) t[u] = tmp[min(g0 + u, NGRP - 1)][fg][fd];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (g0 + u < ngrp) acc = __fadd_rn(acc, t[u]);
            }
            dst = acc;
        }
        __syncthreads();   // pex / pbf / tmp / et_s are rewritten by the next block
    }
    if (wave < G && lane == 0) l_s[wave] = l;
    __syncthreads();
    if (tid < G * XD_DZ) {
        const int col = (kvh * G + fg) * XD_D + z * XD_DZ + fd;
        const bf16_t o = f2bf(__fmul_rn(dst, __fdiv_rn(1.0f, l_s[fg])));
        a.O[(long)qi * a.ldo + col] = o;
        if (a.O16) a.O16[x16_off(qi, col, a.ldo / 32)] = o;
    }
}

// Rows of one 64-key chunk (cap <= 64: the PM cross attention over the text keys) in ONE
// launch: workgroup (row, kv head, 32-dimension slice) recomputes the row's <= 64 scores
// itself -- the scores kernel's code, four threads per key; the slices of a row share an
// XCD (blockIdx.x = row fastest), so the K rows come from its L2 -- then runs the P.V
// kernel's one-block path on them from LDS. The same operations in the same order as the
// two launches (the chunk max is the block's running max; a 64-entry block-sum buffer adds
// the same terms as the 512-entry one, the rest being +0), so the output is bit-identical.
template <int G, int XD_D, bool FUSE>
__global__ __launch_bounds__(256) void xattn_single_kernel(ExactAttnArgs a) {
    constexpr int NCB = XD_D / 32, H2 = XD_D / 2;
    constexpr int DP = XD_DZ / 2;                // dimension pairs per workgroup (16)
    constexpr int NG8 = XD_CH / 8;               // 8-key groups of the chunk
    __shared__ float qs[G][XD_D];
    __shared__ float wmax[4][G];
    __shared__ float ss[G][XD_CH];
    __shared__ float pex[G][XD_CH + 16];
    __shared__ float pbf[G][XD_CH];
    __shared__ float tmp[NG8][G][XD_DZ];
    __shared__ float l_s[G];
    const int qi = blockIdx.x, kvh = blockIdx.y, z = blockIdx.z, tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6, kl = tid >> 2, qa = tid & 3;
    const int row = a.q_row ? a.q_row[qi] : qi;
    int lo, hi;
    xd_range(a, row, lo, hi);
    const int span = hi - lo;
    if (span <= 0) return;
    const int key = lo + kl;
    const bool valid = key < hi;
    const bf16_t* kr = a.K + row * a.kv_bstride + kvh * a.kv_hstride + (long)(valid ? key : lo) * XD_D + 8 * qa;
    u32x4 kv[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) kv[cb] = *(const u32x4*)(kr + 32 * cb);
    // the V words of this lane's 8-key group (lanes of groups past the chunk: none)
    const int dp = tid % DP, gl = tid / DP;
    const bool vlane = gl < NG8;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride + (long)lo * XD_D + z * XD_DZ;
    uint32_t vw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        vw[j] = *(const uint32_t*)(Vb + (long)min(vlane ? gl * 8 + j : 0, span - 1) * XD_D + 2 * dp);
    if constexpr (FUSE) {
        const float* tab = a.rope_tab + (long)row * XD_D;
        for (int i = tid; i < G * H2; i += 256) {
            const int g = i / H2, d = i % H2;
            const bf16_t* qh = a.Q + (long)qi * a.ldq + (kvh * G + g) * XD_D;
            float o1, o2;
            xd_rope(bf2f(qh[d]), bf2f(qh[d + H2]), tab[d], tab[H2 + d], o1, o2);
            qs[g][d] = o1;
            qs[g][d + H2] = o2;
        }
    } else {
        for (int i = tid; i < G * XD_D / 2; i += 256) {
            const int g = i / (XD_D / 2), p = i % (XD_D / 2);
            const uint32_t w = *(const uint32_t*)(a.Q + (long)qi * a.ldq + (kvh * G + g) * XD_D + 2 * p);
            qs[g][2 * p] = bf_lo(w);
            qs[g][2 * p + 1] = bf_hi(w);
        }
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
            const float* qc = &qs[g][cb * 32 + 8 * qa];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t kw = kv[cb][i];
                acc[i] = fmaf(qc[2 * i + 1], bf_hi(kw), acc[i]);
                acc[i] = fmaf(qc[2 * i], bf_lo(kw), acc[i]);
            }
        }
        float v8[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v8[i] = __fadd_rn(acc[i], xlane<2>(acc[i]));
        const float va = __fadd_rn(__fadd_rn(v8[0], v8[1]), __fadd_rn(v8[2], v8[3]));
        const float sc = __fmul_rn(__fadd_rn(va, xlane<1>(va)), a.scale);
        const bool own = valid && qa == 0;
        const float sv = own ? sc : -INFINITY;
        if (own) ss[g][kl] = sv;
        const float mx = wave_max(sv);
        if (lane == 0) wmax[wave][g] = mx;
    }
    __syncthreads();
    // exact p of the block (= the chunk) against its max
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const float mb = fmaxf(fmaxf(wmax[0][g], wmax[1][g]), fmaxf(wmax[2][g], wmax[3][g]));
        if (tid < XD_CH) {
            const float p = tid < span ? sdpa_p(__fsub_rn(ss[g][tid], mb), tid, span) : 0.f;
            pex[g][tid] = p;
            pbf[g][tid] = rbf(p);
        } else if (tid < XD_CH + 16) {
            pex[g][tid] = 0.f;
        }
    }
    __syncthreads();
    if (wave < G) {
        const int g = wave;
        const float mb = fmaxf(fmaxf(wmax[0][g], wmax[1][g]), fmaxf(wmax[2][g], wmax[3][g]));
        const float ts = sdpa_block_sum_lds<XD_CH>(pex[g], span, lane);
        const float l = fmaf(sdpa_block_rescale(-INFINITY, mb), 0.f, ts);
        if (lane == 0) l_s[g] = l;
    }
    const int ngrp = (span + 7) / 8;
    if (vlane && gl < ngrp) {
        const int k0 = gl * 8, cn = min(8, span - k0);
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float t0 = 0.f, t1 = 0.f;
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                if (j < cn) {
                    if (j + 1 < cn) {
                        const float p1 = pbf[g][k0 + j + 1];
                        t0 = fmaf(p1, bf_lo(vw[j + 1]), t0);
                        t1 = fmaf(p1, bf_hi(vw[j + 1]), t1);
                    }
                    const float p0 = pbf[g][k0 + j];
                    t0 = fmaf(p0, bf_lo(vw[j]), t0);
                    t1 = fmaf(p0, bf_hi(vw[j]), t1);
                }
            }
            tmp[gl][g][2 * dp] = t0;
            tmp[gl][g][2 * dp + 1] = t1;
        }
    }
    __syncthreads();
    if (tid < G * XD_DZ) {
        const int fg = tid / XD_DZ, fd = tid % XD_DZ;
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < NG8; ++u)
            if (u < ngrp) acc = __fadd_rn(acc, tmp[u][fg][fd]);
        const int col = (kvh * G + fg) * XD_D + z * XD_DZ + fd;
        const bf16_t o = f2bf(__fmul_rn(acc, __fdiv_rn(1.0f, l_s[fg])));
        a.O[(long)qi * a.ldo + col] = o;
        if (a.O16) a.O16[x16_off(qi, col, a.ldo / 32)] = o;
    }
}

// decode attention (one query per row, gemv numerics) on the scores scratch sbuf
// [Mq][Hq][cap] and chunk maxima mbuf [Mq][Hkv][nsplit][G]
template <int G, int D>
static void launch_xd(const ExactAttnArgs& a, float* sbuf, float* mbuf, int cap, int nsplit, hipStream_t st) {
    const dim3 gs((unsigned)a.Mq, (unsigned)a.Hkv, (unsigned)nsplit), gp((unsigned)a.Mq, (unsigned)a.Hkv, D / XD_DZ);
    const int span_max = a.span_max > 0 ? min(a.span_max, cap) : cap;
    if (span_max <= XD_CH && !a.kv_new) {   // one chunk per row, nothing appended: one launch
        if (a.rope_tab) hipLaunchKernelGGL((xattn_single_kernel<G, D, true>), gp, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((xattn_single_kernel<G, D, false>), gp, dim3(256), 0, st, a);
        return;
    }
    if (a.rope_tab) hipLaunchKernelGGL((xattn_scores_kernel<G, D, true>), gs, dim3(256), 0, st, a, sbuf, mbuf, cap, nsplit);
    else hipLaunchKernelGGL((xattn_scores_kernel<G, D, false>), gs, dim3(256), 0, st, a, sbuf, mbuf, cap, nsplit);
    hipLaunchKernelGGL((xattn_pv_kernel<G, D>), gp, dim3(256), 0, st, a, sbuf, mbuf, cap, nsplit);
}

// the softmax's std::exp(float) restatement (common.h sdpa_expf) over an array: the test hook
// that pins it against the reference host's glibc expf (tests/test_gpu_exact.py)
__global__ void sdpa_expf_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        y[i] = sdpa_expf(x[i]);
}
int sdpa_expf_array(const float* x, float* y, long n, hipStream_t st) {
    if (n <= 0) return 0;
    if (!x || !y) return -1;
    const long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(sdpa_expf_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, st, x, y, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

bool exact_attention_decode_supported(int G, int D) {
    return (G == 2 && (D == 256 || D == 128 || D == 64)) || (G == 1 && (D == 256 || D == 64));
}

int exact_attention_decode(const ExactAttnArgs& a, float* sbuf, float* mbuf, int cap, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (!a.Q || !a.K || !a.V || !a.kv_len || !a.O || !sbuf || !mbuf || a.Hq % a.Hkv) return -1;
    if (a.q_pos || a.q_len) return -1;   // one query per row, at its last key
    if (a.kv_new && !a.rope_tab) return -1;
    const int G = a.Hq / a.Hkv;
    // the grid covers the call's key bound (span_max: host hint on every row's keys, the
    // sampler force-stops rows there; 0: the cache capacity)
    const int span_b = a.span_max > 0 ? min(a.span_max, cap) : cap;
    const int nsplit = (span_b + XD_CH - 1) / XD_CH;
    if ((cap + SDPA_KV_BLOCK - 1) / SDPA_KV_BLOCK > SDPA_MAX_BLOCKS) return -1;
    if (G == 2 && a.D == 256) launch_xd<2, 256>(a, sbuf, mbuf, cap, nsplit, st);
    else if (G == 2 && a.D == 128) launch_xd<2, 128>(a, sbuf, mbuf, cap, nsplit, st);
    else if (G == 2 && a.D == 64) launch_xd<2, 64>(a, sbuf, mbuf, cap, nsplit, st);
    else if (G == 1 && a.D == 256) launch_xd<1, 256>(a, sbuf, mbuf, cap, nsplit, st);
    else if (G == 1 && a.D == 64) launch_xd<1, 64>(a, sbuf, mbuf, cap, nsplit, st);
    else return -3;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

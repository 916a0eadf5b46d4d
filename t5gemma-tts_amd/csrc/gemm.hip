// Weight-streaming bf16 GEMM on v_mfma_f32_16x16x32_bf16 for the T5Gemma-TTS engine.
//
// Y[M][N] = X[M][K] . W[N][K]^T  (nn.Linear layout), fp32 accumulation, one
// rounding to bf16 in the epilogue (the reference's CPU bf16 F.linear rounds once).
//
// Packed weight layout "P16" (built once at load time by t5g_pack_p16):
//   fragment (g, kb) = 16 rows x 32 k = 1 KiB, stored in the exact lane order of the
//   MFMA A operand: lane l holds W[g*16 + (l&15)][kb*32 + 8*(l>>4) + 0..7].
//   Fragments are g-major, so one row group's K stream is contiguous and a wave
//   reads each fragment with ONE fully coalesced 1 KiB global_load_dwordx4.
//   NG (row groups) is padded to a multiple of 4 with zero rows.
//
// Activations are the MFMA B operand (lane l: X[m = l&15][k = 8*(l>>4) + 0..7]),
// so the batch rides in the 16 MFMA columns: at decode (M <= 16) one MFMA per
// 1 KiB of weights -- VALU stays idle, the kernel is a pure HBM stream.
//
// Block = 4 waves. WPG waves share one row group and split its K range
// (WPG = 4: decode, 1 row group / block; WPG = 1: prefill, 4 row groups / block
// reading the same X fragments through L1). blockIdx.y splits K across blocks
// (fp32 partial slabs reduced by the consumer kernel, in fixed order).
#include <stdlib.h>

#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

T5G_TS_UNIT(gemm)

__global__ void pack_p16_kernel(const bf16_t* __restrict__ src, int N, int K, long ld,
                                bf16_t* __restrict__ dst, int KB, long nfrag) {
    long frag = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (frag >= nfrag) return;
    int lane = threadIdx.x & 63;
    long g = frag / KB;
    int kb = (int)(frag % KB);
    long row = g * 16 + (lane & 15);
    int k0 = kb * 32 + 8 * (lane >> 4);
    u32x4 v = {0u, 0u, 0u, 0u};
    if (row < N && k0 < K) v = *(const u32x4*)(src + row * ld + k0);
    *(u32x4*)(dst + (frag * 64 + lane) * 8) = v;
}

template <int MT>
__device__ __forceinline__ void load_x(const bf16_t* __restrict__ X, int ldx, int M, int m0, int kb,
                                       int lane, bf16x8_s (&xf)[MT]) {
    // unconditional (clamped row) loads + select: a load under a branch makes the
    // compiler wait for every load in flight at the join
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = m0 + mt * 16 + (lane & 15);
        const bf16x8_s v = *(const bf16x8_s*)(X + (long)min(m, M - 1) * ldx + kb * 32 + 8 * (lane >> 4));
        xf[mt] = m < M ? v : (bf16x8_s){0, 0, 0, 0, 0, 0, 0, 0};
    }
}

// KS = K-interleave factor of the accumulation: k-step kb belongs to slice
// (kb - kb_lo) % KS, each slice is accumulated in k order, and the slices are
// summed in slice order at the end. The result is therefore bit-identical
// whether a slice runs on its own wave (WPG == KS, decode) or all slices of a row
// group run on one wave (WPG == 1, prefill) -- a row's logits do not depend on
// which other rows share the batch.
template <int MT, int WPG, int KS, int EPI, bool XLDS>
__global__ __launch_bounds__(256) void gemm_p16_kernel(GemmArgs a) {
    static_assert(WPG == KS || WPG == 1, "slice mapping");
    constexpr int RG = 4 / WPG;  // row groups per block
    constexpr int SPW = KS / WPG;  // slices per wave
    constexpr int UN = (WPG == 1) ? KS : 8;  // k-steps in flight per wave per iteration
    constexpr int XCH = 18;  // X-staging chunks per thread (XLDS: rows * K_slice / 8 <= 256 * XCH)
    __shared__ f32x4 red[4][MT][64];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    T5G_TS(0);
    const int g = blockIdx.x * RG + wave / WPG;
    const int ks = wave % WPG;
    const int m0 = blockIdx.z * 16 * MT;
    const int per = (a.KB + a.splits - 1) / a.splits;
    const int kb_lo = blockIdx.y * per;
    const int kb_hi = min(a.KB, kb_lo + per);

    f32x4 acc[SPW][MT];
#pragma unroll
    for (int s = 0; s < SPW; ++s)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[s][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};

    const bf16x8_s* wp = (const bf16x8_s*)a.W + ((long)g * a.KB) * 64 + lane;
    if (kb_hi <= kb_lo) {
        // empty K slice (splits not dividing K): contributes zeros
    } else if constexpr (WPG == KS && MT == 1 && XLDS) {
        // Decode (M <= 16): the block's X rows for its K range are staged once in LDS, so
        // the vector-memory path carries only the weight stream (one 1 KiB fragment per
        // MFMA). Weight fragments are register double-buffered: group g+1 (UN steps) is in
        // flight while group g is multiplied; the first group is issued before the X
        // staging barrier.
        extern __shared__ bf16_t xs[];
        const int rows = min(16, a.M - m0);
        const int kspan = kb_hi - kb_lo;
        const int ldsx = kspan * 32 + 8;   // +16 B row pad spreads the 16 row reads over banks
        constexpr int STEP = UN * KS;
        int kb = kb_lo + ks;
        // fragments kb >= kb_hi fall outside the descriptor: zero, no traffic
        const __amdgpu_buffer_rsrc_t wr = frag_rsrc(a.W + (long)g * a.KB * 512, (uint32_t)kb_hi * 1024u);
        bf16x8_s wcur[UN];
        {
            // all X chunks of the thread are requested at once (buffer loads: slots past
            // the block's rows fall outside the descriptor -> 0, no traffic), then the first
            // weight group: vmcnt retires in issue order, so the LDS writes below wait for
            // the X rows only, not behind the weight group (HBM) they were queued after
            // before (5 us of the gate/up block spent here, tools/micro_timeline.cpp)
            const int total = rows * kspan * 4;
            const __amdgpu_buffer_rsrc_t xrs = frag_rsrc(a.X + (long)m0 * a.ldx, (uint32_t)rows * a.ldx * 2u);
            bf16x8_s xv[XCH];
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                const int idx = threadIdx.x + 256 * i;
                const int r = idx / (kspan * 4), c = idx - r * (kspan * 4);
                const int off = idx < total ? (r * a.ldx + kb_lo * 32 + 8 * c) * 2 : 0x7ffffff0;
                xv[i] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
            }
#pragma unroll
            for (int u = 0; u < UN; ++u) wcur[u] = frag_load(wr, kb + u * KS, lane);
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                const int idx = threadIdx.x + 256 * i;
                const int r = idx / (kspan * 4), c = idx - r * (kspan * 4);
                if (idx < total) *(bf16x8_s*)(xs + r * ldsx + 8 * c) = xv[i];
            }
        }
        __syncthreads();
        T5G_TS(1);
        const int xr = lane & 15;
        const bf16_t* xrow = xs + min(xr, rows - 1) * ldsx + 8 * (lane >> 4) - kb_lo * 32;
        for (; kb < kb_hi; kb += STEP) {
            bf16x8_s wnext[UN];
            const int kn = kb + STEP;
#pragma unroll
            for (int u = 0; u < UN; ++u) wnext[u] = frag_load(wr, kn + u * KS, lane);
#pragma unroll
            for (int u = 0; u < UN; ++u)
                if (kb + u * KS < kb_hi) {   // uniform: the same for every lane of the wave
                    const bf16x8_s xv = *(const bf16x8_s*)(xrow + (kb + u * KS) * 32);
                    const bf16x8_s xf = xr < rows ? xv : (bf16x8_s){0, 0, 0, 0, 0, 0, 0, 0};
                    acc[0][0] = mfma16(wcur[u], xf, acc[0][0]);
                }
#pragma unroll
            for (int u = 0; u < UN; ++u) wcur[u] = wnext[u];
        }
    } else if constexpr (WPG == KS) {
        // one slice per wave: kb = kb_lo + ks, +KS, ...; every group of UD k-steps is
        // issued at once (predicated), so a short slice costs a single memory round trip
        constexpr int UD = (MT == 1) ? 16 : (MT == 2 ? 12 : 8);
        for (int kb = kb_lo + ks; kb < kb_hi; kb += UD * KS) {
            bf16x8_s wf[UD];
            bf16x8_s xf[UD][MT];
#pragma unroll
            for (int u = 0; u < UD; ++u) {
                // predicated: a short slice issues only its own fragments (all loads are
                // waited for together before the MFMAs anyway)
                const bool ok = kb + u * KS < kb_hi;
                wf[u] = ok ? __builtin_nontemporal_load(wp + (long)(kb + u * KS) * 64)
                           : (bf16x8_s){0, 0, 0, 0, 0, 0, 0, 0};
                if (ok) {
                    load_x<MT>(a.X, a.ldx, a.M, m0, kb + u * KS, lane, xf[u]);
                } else {
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) xf[u][mt] = (bf16x8_s){0, 0, 0, 0, 0, 0, 0, 0};
                }
            }
#pragma unroll
            for (int u = 0; u < UD; ++u)
                if (kb + u * KS < kb_hi)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) acc[0][mt] = mfma16(wf[u], xf[u][mt], acc[0][mt]);
        }
    } else {
        // all KS slices on this wave: step u of a group of KS k-steps is slice u
        for (int kb0 = kb_lo; kb0 < kb_hi; kb0 += KS) {
            bf16x8_s wf[KS];
            bf16x8_s xf[KS][MT];
#pragma unroll
            for (int u = 0; u < KS; ++u)
                if (kb0 + u < kb_hi) wf[u] = __builtin_nontemporal_load(wp + (long)(kb0 + u) * 64);
#pragma unroll
            for (int u = 0; u < KS; ++u)
                if (kb0 + u < kb_hi) load_x<MT>(a.X, a.ldx, a.M, m0, kb0 + u, lane, xf[u]);
#pragma unroll
            for (int u = 0; u < KS; ++u)
                if (kb0 + u < kb_hi)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) acc[u][mt] = mfma16(wf[u], xf[u][mt], acc[u][mt]);
        }
#pragma unroll
        for (int s = 1; s < SPW; ++s)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[0][mt] += acc[s][mt];
    }

#pragma unroll
    T5G_TS(2);
    for (int mt = 0; mt < MT; ++mt) red[wave][mt][lane] = acc[0][mt];
    __syncthreads();

    // GeGLU: a row group is 8 gate rows then the same 8 features' up rows (so one group
    // is one output group and the decode grid has 2F/16 blocks): lanes 0-31 hold the
    // gate sums, lanes 32-63 the up sums of the same (feature, batch row)
    constexpr int OG = RG;  // output groups per block
    constexpr bool GLU = EPI == EPI_GEGLU;
    if (wave >= OG || (GLU && lane >= 32)) return;
    const int og = wave;
    const int n_out = GLU ? a.N / 2 : a.N;
    const int gout = blockIdx.x * OG + og;
    const int n0 = gout * (GLU ? 8 : 16) + 4 * (lane >> 4);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = m0 + mt * 16 + (lane & 15);
        if (m >= a.M) continue;
        float v[4];
        if constexpr (GLU) {
            f32x4 gs = {0.f, 0.f, 0.f, 0.f}, us = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < WPG; ++s) {
                gs += red[og * WPG + s][mt][lane];
                us += red[og * WPG + s][mt][lane + 32];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float gg = rbf(gs[r]);
                float act = rbf(gelu_tanh(gg));
                float uu = rbf(us[r]);
                v[r] = act * uu;
            }
        } else {
            f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < WPG; ++s) s4 += red[og * WPG + s][mt][lane];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = s4[r];
        }
        if constexpr (EPI == EPI_F32) {
            float* y = (float*)a.Y + ((long)blockIdx.y * a.M + m) * a.ldy;
            if (n0 + 3 < n_out) {
                *(f32x4*)(y + n0) = (f32x4){v[0], v[1], v[2], v[3]};
            } else {
                for (int r = 0; r < 4; ++r)
                    if (n0 + r < n_out) y[n0 + r] = v[r];
            }
        } else {
            bf16_t o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float x = v[r];
                const int n = n0 + r;
                if constexpr (EPI == EPI_BIAS_BF16 || EPI == EPI_BIAS_GELU) {
                    if (n < n_out) x = x + bf2f(a.bias[n]);
                }
                if constexpr (EPI == EPI_BIAS_GELU) x = gelu_erf(rbf(x));
                o[r] = f2bf(x);
            }
            bf16_t* y = (bf16_t*)a.Y + (long)m * a.ldy;
            if (n0 + 3 < n_out && ((a.ldy & 3) == 0)) {
                uint2 w;
                w.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
                w.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
                *(uint2*)(y + n0) = w;
            } else {
                for (int r = 0; r < 4; ++r)
                    if (n0 + r < n_out) y[n0 + r] = o[r];
            }
        }
    }
    T5G_TS(3);
}

// ---------------------------------------------------------------------------
int pack_p16(const bf16_t* src, int N, int K, long ld, bf16_t* dst, int NGpad, hipStream_t st) {
    if (K % 32 != 0 || NGpad * 16 < N || NGpad % 4 != 0) return -1;
    const int KB = K / 32;
    long nfrag = (long)NGpad * KB;
    hipLaunchKernelGGL(pack_p16_kernel, dim3((unsigned)((nfrag + 3) / 4)), dim3(256), 0, st, src, N, K,
                       ld, dst, KB, nfrag);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// shortest per-wave k-stream that stages X in LDS (r01 probe: the staging barrier costs
// ~1 us, repaid from 16 fragments per wave)
constexpr int XLDS_MIN = 16;

template <int MT, int WPG, int KS, int EPI>
static void launch_t(const GemmArgs& a, int mblocks, hipStream_t st) {
    constexpr int RG = 4 / WPG;
    dim3 grid((unsigned)(a.NG / RG), (unsigned)a.splits, (unsigned)mblocks);
    const int per = (a.KB + a.splits - 1) / a.splits;
    // decode with a long K stream per wave: stage the X rows in LDS once per block (the
    // staging barrier costs ~1 us, repaid only when each wave streams >= 16 fragments)
    if (WPG == KS && MT == 1 && per / KS >= XLDS_MIN && min(16, a.M) * per * 4 <= 256 * 18) {
        const size_t shm = (size_t)min(16, a.M) * (per * 32 + 8) * sizeof(bf16_t);
        hipLaunchKernelGGL((gemm_p16_kernel<MT, WPG, KS, EPI, true>), grid, dim3(256), shm, st, a);
    } else {
        hipLaunchKernelGGL((gemm_p16_kernel<MT, WPG, KS, EPI, false>), grid, dim3(256), 0, st, a);
    }
}


// decode (WPG = KS) and prefill (WPG = 1) instantiate the same slice order
template <int MT, bool PREFILL>
static int launch_epi(const GemmArgs& a, int epi, int mblocks, hipStream_t st) {
    constexpr int W4 = PREFILL ? 1 : 4;
    constexpr int W2 = PREFILL ? 1 : 2;
    switch (epi) {
        case EPI_BF16: launch_t<MT, W4, 4, EPI_BF16>(a, mblocks, st); break;
        case EPI_BIAS_BF16: launch_t<MT, W4, 4, EPI_BIAS_BF16>(a, mblocks, st); break;
        case EPI_BIAS_GELU: launch_t<MT, W4, 4, EPI_BIAS_GELU>(a, mblocks, st); break;
        // GeGLU: 2 row groups x 2-way K interleave per decode block (r01 probe: 1 group x 4
        // waves, twice the blocks, was not faster)
        case EPI_GEGLU: launch_t<MT, W2, 2, EPI_GEGLU>(a, mblocks, st); break;
        case EPI_F32: launch_t<MT, W4, 4, EPI_F32>(a, mblocks, st); break;
        default: return -4;
    }
    return 0;
}

// ---------------------------------------------------------------------------
// Prefill / encoder GEMM (many tokens: the encoder's B*T_x rows, the decoder prefill's
// B*(T_p+1) rows). Block = 4 waves in a 2 x 2 arrangement over a 128-output x 128-token
// tile; each wave owns 4 row groups (64 outputs) x 4 token tiles (64 tokens) = 16 MFMA
// accumulators, so every 1 KiB weight fragment and every 1 KiB activation fragment a wave
// loads feeds 4 MFMAs (the decode kernel's 1:1 ratio made the old prefill path 7 % of
// the MFMA peak). Weight fragments come straight from the P16 layout (A operand lane
// order), activation fragments straight from row-major X (B operand: lane l reads row
// l&15, k 8*(l>>4)..+7); the two waves sharing a row set (or a token set) hit each
// other's lines in L1. Next k-step's fragments are in flight while this one multiplies.
// Accumulation is one MFMA chain in k order per output: deterministic, and a token's
// result does not depend on the other tokens of the launch (batch-invariant).
// S k-steps of fragments are in flight per wave (a ring of S register stages): at the
// decoder prefill's 1 216 tokens a launch has 1-2 blocks per CU, one wave per SIMD, so
// the ring depth -- not the MFMA rate -- sets how long each k-step waits for its loads.
// Stage s of a ring turn feeds chain s & 1, so every S gives the same k order per chain.
#ifndef PF_STAGES
#define PF_STAGES 4
#endif
#ifndef PFL_NBUF
#define PFL_NBUF 4
#endif
// prefill epilogue: lane l holds outputs 4*(l>>4)..+3 of each of the wave's 4 row groups
// (from g0) for token l&15 of each of its 4 token tiles (from mb)
template <int EPI>
__device__ __forceinline__ void pf_epilogue(const GemmArgs& a, const f32x4 (&acc)[4][4], int g0, int mb, int lane) {
    constexpr bool GLU = EPI == EPI_GEGLU;
    const int n_out = GLU ? a.N / 2 : a.N;
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
        const int g = g0 + rg;
        if (g >= a.NG) break;
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            const int m = mb + mt * 16 + (lane & 15);
            float v[4];
            int n0;
            if constexpr (GLU) {
                // 8 gate rows then the same 8 features' up rows: the up sums sit 32 lanes up
                f32x4 up;
#pragma unroll
                for (int r = 0; r < 4; ++r) up[r] = __shfl_down(acc[rg][mt][r], 32, 64);
                if (lane >= 32) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = rbf(gelu_tanh(rbf(acc[rg][mt][r]))) * rbf(up[r]);
                n0 = g * 8 + 4 * (lane >> 4);
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = acc[rg][mt][r];
                n0 = g * 16 + 4 * (lane >> 4);
            }
            if (m >= a.M) continue;
            bf16_t o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float x = v[r];
                if constexpr (EPI == EPI_BIAS_BF16 || EPI == EPI_BIAS_GELU) {
                    if (n0 + r < n_out) x = x + bf2f(a.bias[n0 + r]);
                }
                if constexpr (EPI == EPI_BIAS_GELU) x = gelu_erf(rbf(x));
                o[r] = f2bf(x);
            }
            bf16_t* y = (bf16_t*)a.Y + (long)m * a.ldy;
            if (n0 + 3 < n_out && (a.ldy & 3) == 0) {
                uint2 w2;
                w2.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
                w2.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
                *(uint2*)(y + n0) = w2;
            } else {
                for (int r = 0; r < 4; ++r)
                    if (n0 + r < n_out) y[n0 + r] = o[r];
            }
        }
    }
}

template <int EPI, int S>
__global__ __launch_bounds__(256) void gemm_pf_kernel(GemmArgs a) {
    static_assert(S % 2 == 0, "even ring: stage parity = k-step parity");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int g0 = blockIdx.x * 8 + wr * 4;                 // first row group of this wave
    const int mb = blockIdx.y * 128 + wc * 64;              // first token of this wave
    const int KB = a.KB;
    const __amdgpu_buffer_rsrc_t wrs = frag_rsrc(a.W, (uint32_t)a.NG * (uint32_t)KB * 1024u);
    const __amdgpu_buffer_rsrc_t xrs = frag_rsrc(a.X, (uint32_t)a.M * (uint32_t)a.ldx * 2u);
    const int xk = 8 * (lane >> 4);
    int xrow[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) xrow[mt] = (mb + mt * 16 + (lane & 15)) * a.ldx;   // rows >= M: out of range
    auto load = [&](bf16x8_s(&w)[4], bf16x8_s(&x)[4], int kb) __attribute__((always_inline)) {
        const bool ok = kb < KB;
#pragma unroll
        for (int rg = 0; rg < 4; ++rg)
            w[rg] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(
                                                     wrs, ok ? (((g0 + rg) * KB + kb) * 64 + lane) * 16 : (int)0xfffffff0u, 0, 0));
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
            x[mt] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(
                                                     xrs, ok ? (xrow[mt] + kb * 32 + xk) * 2 : (int)0xfffffff0u, 0, 0));
    };
    // two accumulator chains (even / odd k-steps) summed at the end: half-length MFMA
    // chains (K = 9216: 144 instead of 288), so the fp32 accumulation error stays at the
    // level of the sliced decode kernel
    f32x4 acc[4][4], acc2[4][4];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[rg][mt] = acc2[rg][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto mma = [&](const bf16x8_s(&w)[4], const bf16x8_s(&x)[4], f32x4(&c)[4][4]) __attribute__((always_inline)) {
#pragma unroll
        for (int rg = 0; rg < 4; ++rg)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) c[rg][mt] = mfma16(w[rg], x[mt], c[rg][mt]);
    };
    bf16x8_s wq[S][4], xq[S][4];
#pragma unroll
    for (int s = 0; s < S - 1; ++s) load(wq[s], xq[s], s);
    for (int kb = 0; kb < KB; kb += S) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
            load(wq[(s + S - 1) % S], xq[(s + S - 1) % S], kb + s + S - 1);
            mma(wq[s], xq[s], (s & 1) ? acc2 : acc);
        }
    }
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[rg][mt] += acc2[rg][mt];
    pf_epilogue<EPI>(a, acc, g0, mb, lane);
}

// LDS-staged form of the same tile (round 3): each k-step's 8 weight and 8 activation
// fragments of the block (16 KiB) are moved by buffer_load ... lds (no VGPR round trip,
// range-checked like the register form) into a ring of NBUF LDS stages, one fragment per
// wave instruction in MFMA operand lane order, so every wave reads its 4 + 4 fragments back
// with conflict-free ds_read_b128; NBUF - 1 k-steps are in flight, one counted vmcnt and
// one barrier per k-step. Fragments are fetched once per block instead of once per wave
// pair, which is what bounded the register form (load issue, not MFMA). The two
// accumulator chains and every sum are those of gemm_pf_kernel: outputs bitwise equal.
// lgkmcnt(0) too: this wave's ds_reads of the previous k-step's stage must have completed
// before the barrier, because right after it some wave's stage() DMA-writes that same slot.
// With only vmcnt the compiler may sink the MFMAs (and the lgkmcnt wait before them) past
// the barrier; an out-of-range LDS-DMA piece (a token tile's rows >= M) completes at once
// and could overwrite the slot while the read is still pending -- the round-3 run-to-run
// difference of the last token tile.
template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" : : "n"(N) : "memory");
}
template <int EPI, int NBUF>
__global__ __launch_bounds__(256, 2) void gemm_pfl_kernel(GemmArgs a) {
    constexpr int P = NBUF - 1;   // k-steps in flight
    extern __shared__ __attribute__((aligned(16))) char smem[];   // [NBUF][16 fragments][1 KiB]
    // wave-uniform in a scalar register: the LDS destination of buffer_load ... lds (M0) must
    // be, or the compiler wraps every load in a waterfall loop
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int wr = wave >> 1, wc = wave & 1;
    const int gb = blockIdx.x * 8;                          // first row group of the block
    const int tb = blockIdx.y * 128;                        // first token of the block
    const int KB = a.KB;
    const __amdgpu_buffer_rsrc_t wrs = frag_rsrc(a.W, (uint32_t)a.NG * (uint32_t)KB * 1024u);
    const __amdgpu_buffer_rsrc_t xrs = frag_rsrc(a.X, (uint32_t)a.M * (uint32_t)a.ldx * 2u);
    // fragments 4 * wave .. + 3 of every stage: 0-7 the block's row groups, 8-15 its token tiles
    const int xk = 8 * (lane >> 4);
    int src[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int f = 4 * wave + q;
        src[q] = f < 8 ? ((gb + f) * KB * 64 + lane) * 16                       // + kb * 1024
                       : ((tb + (f - 8) * 16 + (lane & 15)) * a.ldx + xk) * 2;    // + kb * 64; rows >= M: out of range
    }
    auto stage = [&](int kb) __attribute__((always_inline)) {
        __attribute__((address_space(3))) char* base =
            (__attribute__((address_space(3))) char*)smem + (kb % NBUF) * 16384 + 4 * wave * 1024;
        const bool live = kb < KB;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (4 * wave + q < 8)   // wave-uniform: waves 0-1 stage weights, 2-3 activations
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, base + q * 1024, 16,
                                                         live ? src[q] + kb * 1024 : (int)0xfffffff0u, 0, 0, 0);
            else
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, base + q * 1024, 16,
                                                         live ? src[q] + kb * 64 : (int)0xfffffff0u, 0, 0, 0);
        }
    };
    f32x4 acc[4][4], acc2[4][4];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[rg][mt] = acc2[rg][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < P; ++p) stage(p);
    auto kstep = [&](int kb, f32x4(&c)[4][4]) __attribute__((always_inline)) {
        // this wave's fragments of k-step kb have landed (the P - 1 later stages may still be
        // in flight); after the barrier every wave's have, and nobody reads stage kb - 1 any more
        wait_vm_barrier<4 * (P - 1)>();
        stage(kb + P);
        const char* buf = smem + (kb % NBUF) * 16384 + lane * 16;
        bf16x8_s w[4], x[4];
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) w[rg] = *(const bf16x8_s*)(buf + (wr * 4 + rg) * 1024);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) x[mt] = *(const bf16x8_s*)(buf + (8 + wc * 4 + mt) * 1024);
#pragma unroll
        for (int rg = 0; rg < 4; ++rg)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) c[rg][mt] = mfma16(w[rg], x[mt], c[rg][mt]);
    };
    // even k-steps into acc, odd into acc2 (gemm_pf_kernel's two chains)
    for (int kb = 0; kb < KB; kb += 2) {   // KB even (gemm_prefill)
        kstep(kb, acc);
        kstep(kb + 1, acc2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the tail's out-of-range stages
#pragma unroll
    for (int rg = 0; rg < 4; ++rg)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[rg][mt] += acc2[rg][mt];
    pf_epilogue<EPI>(a, acc, gb + wr * 4, tb + wc * 64, lane);
}

template <int NBUF>
static int launch_pfl(const GemmArgs& a, int epi, dim3 grid, hipStream_t st) {
    const size_t shm = (size_t)NBUF * 16384;
    switch (epi) {
        case EPI_BF16: hipLaunchKernelGGL((gemm_pfl_kernel<EPI_BF16, NBUF>), grid, dim3(256), shm, st, a); break;
        case EPI_BIAS_BF16: hipLaunchKernelGGL((gemm_pfl_kernel<EPI_BIAS_BF16, NBUF>), grid, dim3(256), shm, st, a); break;
        case EPI_BIAS_GELU: hipLaunchKernelGGL((gemm_pfl_kernel<EPI_BIAS_GELU, NBUF>), grid, dim3(256), shm, st, a); break;
        case EPI_GEGLU: hipLaunchKernelGGL((gemm_pfl_kernel<EPI_GEGLU, NBUF>), grid, dim3(256), shm, st, a); break;
        default: return -4;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int S>
static int launch_pf(const GemmArgs& a, int epi, dim3 grid, hipStream_t st) {
    switch (epi) {
        case EPI_BF16: hipLaunchKernelGGL((gemm_pf_kernel<EPI_BF16, S>), grid, dim3(256), 0, st, a); break;
        case EPI_BIAS_BF16: hipLaunchKernelGGL((gemm_pf_kernel<EPI_BIAS_BF16, S>), grid, dim3(256), 0, st, a); break;
        case EPI_BIAS_GELU: hipLaunchKernelGGL((gemm_pf_kernel<EPI_BIAS_GELU, S>), grid, dim3(256), 0, st, a); break;
        case EPI_GEGLU: hipLaunchKernelGGL((gemm_pf_kernel<EPI_GEGLU, S>), grid, dim3(256), 0, st, a); break;
        default: return -4;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

static int gemm_prefill(const GemmArgs& a, int epi, hipStream_t st) {
    if ((long)a.M * a.ldx * 2 >= 0x7fffffffL || (long)a.NG * a.KB * 1024 >= 0x7fffffffL) return -1;
    const dim3 grid((unsigned)((a.NG + 7) / 8), (unsigned)((a.M + 127) / 128));
    // prefill == 1: the LDS-staged kernel; 2: the register-ring kernel (A/B, tools/probe_pf_lds.py)
    if (a.prefill == 1 && a.ldx % 8 == 0 && a.KB % 2 == 0) return launch_pfl<PFL_NBUF>(a, epi, grid, st);
    // ring depth: PF_STAGES k-steps when they divide KB (no partial ring turn), else 2
    if (a.KB % PF_STAGES == 0) return launch_pf<PF_STAGES>(a, epi, grid, st);
    return launch_pf<2>(a, epi, grid, st);
}

// Decode GEMM whose block stages the X rows of its K slice in LDS once and shares them
// among RG row groups (4 waves each: the 4 k-slices of the KS = 4 order, every slice
// chained in k order and the slices summed in order, so outputs are bitwise those of
// gemm_p16_kernel<MT, 4, 4, EPI, *>). At M = 32 the X fragments are two of every three
// 16-byte loads of the fragment-per-MFMA kernel; here they are read from LDS.
constexpr int DX_XCH = 18;   // X staging chunks per thread
template <int MT, int RG, int EPI>
__global__ __launch_bounds__(256 * RG) void gemm_dx_kernel(GemmArgs a) {
    constexpr int KS = 4, UN = 8, STEP = UN * KS, XCH = (DX_XCH + RG - 1) / RG;
    extern __shared__ bf16_t xs[];
    __shared__ f32x4 red[RG * 4][MT][64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int rgl = wave >> 2, ks = wave & 3;
    const int g = blockIdx.x * RG + rgl;
    const int per = (a.KB + a.splits - 1) / a.splits;
    const int kb_lo = blockIdx.y * per;
    const int kb_hi = min(a.KB, kb_lo + per);
    const int rows = min(16 * MT, a.M);
    const int kspan = max(0, kb_hi - kb_lo);
    const int ldsx = kspan * 32 + 8;
    int kb = kb_lo + ks;
    const __amdgpu_buffer_rsrc_t wr = frag_rsrc(a.W + (long)g * a.KB * 512, (uint32_t)max(kb_hi, 0) * 1024u);
    bf16x8_s wcur[UN];
    {
        // every X chunk of the thread first, then the first weight group (vmcnt retires
        // in issue order: the LDS writes wait for the X rows only)
        const int total = rows * kspan * 4;
        const __amdgpu_buffer_rsrc_t xrs = frag_rsrc(a.X, (uint32_t)rows * a.ldx * 2u);
        bf16x8_s xv[XCH];
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int idx = threadIdx.x + 256 * RG * i;
            const int r = idx / max(1, kspan * 4), c = idx - r * (kspan * 4);
            const int off = idx < total ? (r * a.ldx + kb_lo * 32 + 8 * c) * 2 : 0x7ffffff0;
            xv[i] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) wcur[u] = frag_load(wr, kb + u * KS, lane);
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int idx = threadIdx.x + 256 * RG * i;
            const int r = idx / max(1, kspan * 4), c = idx - r * (kspan * 4);
            if (idx < total) *(bf16x8_s*)(xs + r * ldsx + 8 * c) = xv[i];
        }
    }
    __syncthreads();
    const int xr = lane & 15;
    f32x4 acc[MT];
    const bf16_t* xrow[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        acc[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        xrow[mt] = xs + min(16 * mt + xr, rows - 1) * ldsx + 8 * (lane >> 4) - kb_lo * 32;
    }
    for (; kb < kb_hi; kb += STEP) {
        bf16x8_s wnext[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) wnext[u] = frag_load(wr, kb + STEP + u * KS, lane);
#pragma unroll
        for (int u = 0; u < UN; ++u)
            if (kb + u * KS < kb_hi) {   // uniform
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const bf16x8_s xv = *(const bf16x8_s*)(xrow[mt] + (kb + u * KS) * 32);
                    const bf16x8_s xf = 16 * mt + xr < rows ? xv : (bf16x8_s){0, 0, 0, 0, 0, 0, 0, 0};
                    acc[mt] = mfma16(wcur[u], xf, acc[mt]);
                }
            }
#pragma unroll
        for (int u = 0; u < UN; ++u) wcur[u] = wnext[u];
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wave][mt][lane] = acc[mt];
    __syncthreads();
    if (ks != 0) return;
    const int n_out = a.N;
    const int n0 = g * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + xr;
        if (m >= a.M) continue;
        f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s) s4 += red[rgl * KS + s][mt][lane];
        if constexpr (EPI == EPI_F32) {
            float* y = (float*)a.Y + ((long)blockIdx.y * a.M + m) * a.ldy;
            if (n0 + 3 < n_out) {
                *(f32x4*)(y + n0) = s4;
            } else {
                for (int r = 0; r < 4; ++r)
                    if (n0 + r < n_out) y[n0 + r] = s4[r];
            }
        } else {
            bf16_t* y = (bf16_t*)a.Y + (long)m * a.ldy;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + r;
                if (n >= n_out) continue;
                float x = s4[r];
                if constexpr (EPI == EPI_BIAS_BF16 || EPI == EPI_BIAS_GELU) x = x + bf2f(a.bias[n]);
                if constexpr (EPI == EPI_BIAS_GELU) x = gelu_erf(rbf(x));
                y[n] = f2bf(x);
            }
        }
    }
}

// 1: launched, 0: not eligible. Measured (tools/probe_dx.py, profiles/r02_probe_dx.jsonl):
// at M = 17..32 sharing the staged X between 2 row groups makes the split-K projections
// with K = 2304 faster (qkv 8.97 -> 7.19 us, cross-q 5.52 -> 5.17); at M <= 16, for the
// o projections (16 k-steps per slice) and for down it is slower or equal.
static int try_dx(const GemmArgs& a, int epi, hipStream_t st, int* rc) {
    constexpr int RG = 2;
    if (epi != EPI_F32 || a.M <= 16 || a.M > 32 || a.KB * 32 > 2304 || a.splits < 2) return 0;
    const int per = (a.KB + a.splits - 1) / a.splits;
    if (per < 18 || a.M * per * 4 > 256 * RG * ((DX_XCH + RG - 1) / RG) || a.NG % RG) return 0;
    const size_t shm = (size_t)a.M * (per * 32 + 8) * sizeof(bf16_t);
    auto* fn = gemm_dx_kernel<2, RG, EPI_F32>;
    static bool attr[T5G_MAX_DEVICES] = {};
    const int dev = t5g_cur_device();
    if (dev < 0) return 0;
    if (!attr[dev]) {
        if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) != hipSuccess)
            return 0;
        attr[dev] = true;
    }
    if (shm > 96 * 1024) return 0;
    hipLaunchKernelGGL(fn, dim3((unsigned)(a.NG / RG), (unsigned)a.splits), dim3(256 * RG), shm, st, a);
    *rc = 0;
    return 1;
}

// Dispatch: decode-shaped (M <= 64) streams weights with K split over the
// block's 4 waves (GEGLU: 2 waves per gate/up group); larger M uses 4 row groups
// per block sharing X fragments.
int gemm_p16(const GemmArgs& a_in, int epi, hipStream_t st) {
    GemmArgs a = a_in;
    if (a.M <= 0) return 0;
    if (a.NG % 4 != 0 || a.splits < 1) return -1;
    if (epi == EPI_GEGLU && a.splits != 1) return -1;
    if (epi != EPI_F32 && a.splits != 1) return -1;
    // many-token phases (encoder, decoder prefill): the register-tiled MFMA kernel
    if (a.prefill && epi != EPI_F32) return gemm_prefill(a, epi, st);
    int rc;
    if (try_dx(a, epi, st, &rc)) {
        if (rc) return rc;
    } else if (a.M <= 16) {
        rc = launch_epi<1, false>(a, epi, 1, st);
    } else if (a.M <= 32) {
        rc = launch_epi<2, false>(a, epi, 1, st);
    } else if (a.M <= 64) {
        rc = launch_epi<4, false>(a, epi, 1, st);
    } else {
        rc = launch_epi<4, true>(a, epi, (a.M + 63) / 64, st);
    }
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

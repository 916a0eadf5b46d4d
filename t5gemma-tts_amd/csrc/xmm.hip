// Exact-order Linear on the f32-input MFMA (parity mode; replaces exact.hip's VALU linears).
//
// The reference's F.linear (bf16 on CPU: oneDNN AMX matmul) sums, per output,
// each 32-element chunk of K as two sequential fp32 chains -- the even k (0, 2, ..., 30) and
// the odd k -- then chunk = E + O, chunk sums folded in order within K parts of the
// measured split (ref_ksplit.h), parts folded in order, bias last. On gfx950
// v_mfma_f32_16x16x4_f32 is, bit for bit, a k-ordered fmaf chain from its C input
// (cdna_hip_programming.md §3 "FP32-input MFMA"): D[i][j] = fma(a3 b3, fma(a2 b2,
// fma(a1 b1, fma(a0 b0, C)))). Four of them continue one chain over 16 elements, so per
// chunk and 16 x 16 tile (16 outputs i x 16 rows j) the E chain is 4 MFMAs on the even
// elements and the O chain 4 on the odd ones, exactly the reference's sums.
//
// Operands arrive in the MFMA's lane order with one 16-byte load per lane and chunk:
// * weights in the E16 layout: P16 (1 KiB fragment per 16 rows x 32 k) of the matrix
//   whose chunks have their 16 element pairs transposed 4 x 4 -- lane (q = l >> 4, r = l & 15)
//   holds pairs 4t + q, t = 0..3, of row r: word t is the A operand pair of MFMA t;
// * activations in the X16 layout: per 16-row tile, chunk, row j and q the same four
//   pairs (written in that order by the producing kernel, or by xmm_to_x16).
// The products of two bf16 values are exact in fp32, so the fmaf chain is the reference's
// product-then-add chain. Output D layout: lane (q, j) holds outputs 4q .. 4q + 3 of the
// group for row j.
//
// Two launch shapes:
// * xmm_wave_kernel: one wave per (16-output group, RT row tiles), every chunk of K in
//   order, folds in registers -- prefill / encoder (M > 32: thousands of tiles);
// * xmm_dec_kernel: decode rows (M <= 32): one 512-thread workgroup per group (and K part
//   where the reference splits K at M = 1: the down projection), its 8 waves split the
//   chunks, chunk sums go through LDS, one thread per output folds them in order.
#include "common.h"
#include "exact_dev.h"
#include "exact_math.h"
#include "t5g_kernels.h"

namespace t5g {

// ---- weight repack: E16[g][kb][lane (q, r)][t] = P16[g][kb][lane (t, r)][q] (u32 words)
__global__ void pack_e16_kernel(const uint32_t* __restrict__ p16, uint32_t* __restrict__ e16, long n_words) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_words) return;
    const long frag = i >> 8;
    const int w = (int)(i & 255), l = w >> 2, t = w & 3, r = l & 15, q = l >> 4;
    e16[i] = p16[(frag << 8) + ((t * 16 + r) << 2) + q];
}

int pack_e16(const bf16_t* p16, bf16_t* e16, long bytes, hipStream_t st) {
    if (!p16 || !e16 || bytes % 1024) return -1;
    const long n = bytes / 4;
    hipLaunchKernelGGL(pack_e16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const uint32_t*)p16,
                       (uint32_t*)e16, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---- activations to X16 (rows >= M of the last tile are zero)
__global__ void to_x16_kernel(const bf16_t* __restrict__ X, int ldx, int M, int K, bf16_t* __restrict__ Y) {
    const int KB = K / 32;
    const long n = (long)((M + 15) / 16) * 16 * (K / 2);   // pairs
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const long m = i / (K / 2);
    const int k = (int)(i % (K / 2)) * 2;
    const uint32_t v = m < M ? *(const uint32_t*)(X + m * ldx + k) : 0u;
    *(uint32_t*)(Y + x16_off(m, k, KB)) = v;
}

int to_x16(const bf16_t* X, int ldx, int M, int K, bf16_t* Y, hipStream_t st) {
    if (M <= 0) return 0;
    if (!X || !Y || K % 32 || ldx % 2) return -1;
    const long n = (long)((M + 15) / 16) * 16 * (K / 2);
    hipLaunchKernelGGL(to_x16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, ldx, M, K, Y);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ---- shared pieces -------------------------------------------------------------------
// The K-split part length (chunks) of row m for packed output column n (as exact.hip)
__device__ __forceinline__ int xmm_kbc(const XmmArgs& a, int m, int n) {
    if (a.kb_fixed > 0) return a.kb_fixed;
    const int mu = a.row_len ? a.row_len[a.tok_row ? a.tok_row[m] : m] : 1;
    const uint16_t* tab = (a.kb_b && n >= a.nsplit_col) ? a.kb_b : a.kb_a;
    const int kbc = tab ? tab[min(max(mu, 1), a.kb_len) - 1] : a.KB;
    return kbc <= 0 ? a.KB : kbc;
}

// fold state of one output element (the reference's part / total chain)
struct XFold {
    float tot, part;
    int nb;
};
__device__ __forceinline__ void xfold(XFold& f, int kb, int kbc, float c) {
    if (kb == f.nb) {
        if (kb > 0) f.tot = __fadd_rn(f.tot, f.part);
        f.part = __fadd_rn(0.f, c);
        f.nb += kbc;
    } else {
        f.part = __fadd_rn(f.part, c);
    }
}
__device__ __forceinline__ float xfold_end(const XFold& f, int KB, int kbc) {
    return KB > kbc ? __fadd_rn(f.tot, f.part) : f.part;
}

// Epilogue of lane (q, j): y[reg] = output n0 + reg (n0 = g * 16 + 4q) of row m. Called by
// whole waves (GEGLU pairs lanes q and q + 2: the gate rows 0..7 of the group with the up
// rows 8..15 of the same features).
template <int EPI>
__device__ __forceinline__ void xmm_store(const XmmArgs& a, int g, int q, long m, const float (&y)[4]) {
    if constexpr (EPI == EPI_GEGLU) {
        float up[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) up[r] = xlane<32>(y[r]);
        if (q >= 2 || m >= a.M) return;
        const int f0 = g * 8 + q * 4;
        if (f0 >= a.N / 2) return;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = rbf(__fmul_rn(rbf(t5g_exact::gelu_tanh(rbf(y[r]))), rbf(up[r])));
        const uint32_t w0 = pack2(v[0], v[1]), w1 = pack2(v[2], v[3]);
        if (a.Y) {
            uint32_t* d = (uint32_t*)((bf16_t*)a.Y + m * a.ldy + f0);
            d[0] = w0;
            d[1] = w1;
        }
        if (a.Y16) {
            const int KB2 = a.N / 64;   // chunks of the act row (N / 2 features)
            *(uint32_t*)(a.Y16 + x16_off(m, f0, KB2)) = w0;
            *(uint32_t*)(a.Y16 + x16_off(m, f0 + 2, KB2)) = w1;
        }
        return;
    }
    if (m >= a.M) return;
    const int n0 = g * 16 + q * 4;
    if constexpr (EPI == EPI_F32) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (n0 + r < a.N) ((float*)a.Y)[m * a.ldy + n0 + r] = y[r];
        return;
    }
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int n = min(n0 + r, a.N - 1);
        if constexpr (EPI == EPI_BF16) {
            v[r] = rbf(y[r]);
        } else if constexpr (EPI == EPI_BIAS_BF16) {
            v[r] = rbf(__fadd_rn(y[r], bf2f(a.bias[n])));
        } else {   // EPI_BIAS_GELU: nn.GELU() (erf) on the bf16 Linear output
            const bf16_t h = f2bf(__fadd_rn(y[r], bf2f(a.bias[n])));
            v[r] = bf2f(a.gelu_lut ? a.gelu_lut[h] : f2bf(t5g_exact::gelu_erf(bf2f(h))));
        }
    }
    if (a.Y) {
        bf16_t* d = (bf16_t*)a.Y + m * a.ldy + n0;
        if (n0 + 4 <= a.N && (a.ldy & 3) == 0) {
            *(uint32_t*)d = pack2(v[0], v[1]);
            *((uint32_t*)d + 1) = pack2(v[2], v[3]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (n0 + r < a.N) d[r] = f2bf(v[r]);
        }
    }
    if (a.Y16 && n0 + 4 <= a.N) {
        const int KB2 = a.N / 32;
        *(uint32_t*)(a.Y16 + x16_off(m, n0, KB2)) = pack2(v[0], v[1]);
        *(uint32_t*)(a.Y16 + x16_off(m, n0 + 2, KB2)) = pack2(v[2], v[3]);
    }
}

// ---- one wave per (group, RT row tiles): every chunk in order, fold in registers --------
// 4 waves per workgroup (4 consecutive groups). DEPTH chunks' operands are in flight.
template <int RT, int EPI>
__global__ __launch_bounds__(256) void xmm_wave_kernel(XmmArgs a) {
    constexpr int DEPTH = 4;
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int j = lane & 15, q = lane >> 4;
    const int mt0 = blockIdx.y * RT;
    const int KB = a.KB;
    const u32x4* wp = (const u32x4*)(a.W + (long)g * KB * 512) + lane;
    const u32x4* xp[RT];
    int kbc[RT];
    XFold f[RT][4];
    const int tiles = (a.M + 15) / 16;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
        // a row-tile group past the last tile re-reads the last one (its stores are skipped)
        xp[r] = (const u32x4*)(a.X16 + (long)min(mt0 + r, tiles - 1) * KB * 512) + lane;
        const long m = (long)(mt0 + r) * 16 + j;
        kbc[r] = xmm_kbc(a, (int)min(m, (long)a.M - 1), g * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) f[r][i] = XFold{0.f, 0.f, 0};
    }
    u32x4 wr[DEPTH], xr[DEPTH][RT];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        const int kb = min(d, KB - 1);
        wr[d] = wp[(long)kb * 64];
#pragma unroll
        for (int r = 0; r < RT; ++r) xr[d][r] = xp[r][(long)kb * 64];
    }
    for (int kb0 = 0; kb0 < KB; kb0 += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int kb = kb0 + d;
            if (kb < KB) {
                const u32x4 w = wr[d];
                u32x4 x[RT];
#pragma unroll
                for (int r = 0; r < RT; ++r) x[r] = xr[d][r];
                const int kn = min(kb + DEPTH, KB - 1);
                wr[d] = wp[(long)kn * 64];
#pragma unroll
                for (int r = 0; r < RT; ++r) xr[d][r] = xp[r][(long)kn * 64];
#pragma unroll
                for (int r = 0; r < RT; ++r) {
                    const f32x4_t c = xmm_chunk(w, x[r]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) xfold(f[r][i], kb, kbc[r], c[i]);
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RT; ++r) {
        float y[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) y[i] = xfold_end(f[r][i], KB, kbc[r]);
        xmm_store<EPI>(a, g, q, (long)(mt0 + r) * 16 + j, y);
    }
}

// ---- decode rows (M <= 32): one 512-thread workgroup per (16-output group, K part) ----
// The 8 waves take the chunks of a stage round-robin and issue every chunk's operand loads
// up front (CPW chunks per wave in flight), chunk sums go to LDS as [chunk][row][col]
// (only the ROWS rows that exist: 8 when M <= 8, so two or more workgroups share a CU),
// then thread t < 16 ROWS folds element (row t >> 4, col t & 15) over the chunks in order
// and stores it: consecutive threads write consecutive outputs of a row.
// PART: the group's chunks [p part_kbc, (p + 1) part_kbc) only, folded from 0 into
// part_out[p] -- the reference's part value, summed in order by the consumer.
template <int RT, bool R8>
struct XDecShape {
    static constexpr int NW = 8, CPW = RT == 1 ? 9 : 5, SC = NW * CPW;
    static constexpr int ROWS = R8 ? 8 : 16 * RT, EL = 16 * ROWS;
    static constexpr int LDS = SC * EL * 4;
};

// Epilogue of folder thread (row m, col fcol of group g): y is the folded value
template <int EPI, bool PART>
__device__ __forceinline__ void xdec_store(const XmmArgs& a, int g, int part, long m, int fcol, float y) {
    const int n = g * 16 + fcol;
    if constexpr (PART) {
        if (m < a.M && n < a.N) a.part_out[((long)part * a.M + m) * a.N + n] = y;
        return;
    }
    if constexpr (EPI == EPI_GEGLU) {
        const float up = xlane<8>(y);   // col + 8 of the same row: the up row of this feature
        if (fcol >= 8 || m >= a.M) return;
        const int ft = g * 8 + fcol;
        if (ft >= a.N / 2) return;
        const bf16_t v = f2bf(rbf(__fmul_rn(rbf(t5g_exact::gelu_tanh(rbf(y))), rbf(up))));
        if (a.Y) ((bf16_t*)a.Y)[m * a.ldy + ft] = v;
        if (a.Y16) a.Y16[x16_off(m, ft, a.N / 64)] = v;
        return;
    }
    if (m >= a.M || n >= a.N) return;
    if constexpr (EPI == EPI_F32) {
        ((float*)a.Y)[m * a.ldy + n] = y;
        return;
    }
    float v;
    if constexpr (EPI == EPI_BF16) {
        v = rbf(y);
    } else if constexpr (EPI == EPI_BIAS_BF16) {
        v = rbf(__fadd_rn(y, bf2f(a.bias[n])));
    } else {   // EPI_BIAS_GELU: nn.GELU() (erf) on the bf16 Linear output
        const bf16_t h = f2bf(__fadd_rn(y, bf2f(a.bias[n])));
        v = bf2f(a.gelu_lut ? a.gelu_lut[h] : f2bf(t5g_exact::gelu_erf(bf2f(h))));
    }
    if (a.Y) ((bf16_t*)a.Y)[m * a.ldy + n] = f2bf(v);
    if (a.Y16) a.Y16[x16_off(m, n, a.N / 32)] = f2bf(v);
}

template <int RT, bool R8, int EPI, bool PART, int VAR = 0>
__global__ __launch_bounds__(512) void xmm_dec_kernel(XmmArgs a) {
    using S = XDecShape<RT, R8>;
    constexpr int NW = S::NW, CPW = S::CPW, SC = S::SC, EL = S::EL;
    extern __shared__ float cs[];   // [SC][EL]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, j = lane & 15, q = lane >> 4;
    const int g = blockIdx.x, KB = a.KB;
    const int part = PART ? (int)blockIdx.y : 0;
    const int kb_lo = PART ? part * a.part_kbc : 0;
    const int kb_hi = PART ? min(kb_lo + a.part_kbc, KB) : KB;
    const u32x4* wp = (const u32x4*)(a.W + (long)g * KB * 512) + lane;
    // R8: lanes j >= 8 (rows that do not exist) read lane j - 8's operand: half the bytes
    const u32x4* xp = (const u32x4*)a.X16 + (R8 ? (lane & ~8) : lane);
    const int frow = tid >> 4, fcol = tid & 15;
    const bool folder = tid < EL;
    // decode rows (no per-row lengths) share the K-part length; when it covers the
    // workgroup's chunks every element folds them as one plain chain
    const bool uni = PART || a.kb_fixed > 0 || !a.row_len;
    const int kbc_t = PART ? (1 << 30) : xmm_kbc(a, uni ? 0 : min(frow, a.M - 1), g * 16);
    const bool single = uni && __builtin_amdgcn_readfirstlane(kbc_t) >= kb_hi - kb_lo;
    XFold f{0.f, 0.f, kb_lo};
    u32x4 wr[CPW], xr[CPW][RT];
    auto load = [&](int s0) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            const int kb = min(s0 + w + c * NW, kb_hi - 1);
            wr[c] = wp[(long)kb * 64];
#pragma unroll
            for (int r = 0; r < RT; ++r) xr[c][r] = xp[((long)r * KB + kb) * 64];
        }
    };
    load(kb_lo);
    for (int s0 = kb_lo; s0 < kb_hi; s0 += SC) {
        const int n = min(SC, kb_hi - s0);
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            const int cc = w + c * NW;
            if (cc < n) {
#pragma unroll
                for (int r = 0; r < RT; ++r) {
                    f32x4_t v;
                    if constexpr (VAR == 2) {   // timing variant: no MFMA
#pragma unroll
                        for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(wr[c][i] ^ xr[c][r][i]);
                    } else {
                        v = xmm_chunk(wr[c], xr[c][r]);
                    }
                    if (!R8 || j < 8) *(f32x4_t*)&cs[cc * EL + (r * 16 + j) * 16 + 4 * q] = v;
                }
            }
        }
        if (s0 + SC < kb_hi) load(s0 + SC);   // the next stage's operands fly during the fold
        __syncthreads();
        if (VAR == 1 && folder) {   // timing variant: no fold
            f.part = cs[tid];
        } else if (folder && single) {
            // one K part: part = ((0 + c0) + c1) + ... -- a plain chain (xfold's first step
            // is fadd(0, c0) too), 16 chunk sums read per LDS round trip
            for (int c0 = 0; c0 < n; c0 += 16) {
                float v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) v[u] = cs[min(c0 + u, SC - 1) * EL + tid];
                if (c0 + 16 <= n) {
#pragma unroll
                    for (int u = 0; u < 16; ++u) f.part = __fadd_rn(f.part, v[u]);
                } else {
#pragma unroll
                    for (int u = 0; u < 16; ++u)
                        if (c0 + u < n) f.part = __fadd_rn(f.part, v[u]);
                }
            }
        } else if (folder) {
            for (int c0 = 0; c0 < n; c0 += 8) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = cs[min(c0 + u, SC - 1) * EL + tid];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (c0 + u < n) xfold(f, s0 + c0 + u, kbc_t, v[u]);
            }
        }
        __syncthreads();
    }
    if (folder) xdec_store<EPI, PART>(a, g, part, frow, fcol, (PART || single) ? f.part : xfold_end(f, KB, kbc_t));
}

template <int RT>
static int launch_xmm_wave(const XmmArgs& a, int epi, hipStream_t st) {
    const int tiles = (a.M + 15) / 16;
    const dim3 grid((unsigned)(a.NG / 4), (unsigned)((tiles + RT - 1) / RT)), blk(256);
    switch (epi) {
        case EPI_F32: hipLaunchKernelGGL((xmm_wave_kernel<RT, EPI_F32>), grid, blk, 0, st, a); break;
        case EPI_BF16: hipLaunchKernelGGL((xmm_wave_kernel<RT, EPI_BF16>), grid, blk, 0, st, a); break;
        case EPI_BIAS_BF16: hipLaunchKernelGGL((xmm_wave_kernel<RT, EPI_BIAS_BF16>), grid, blk, 0, st, a); break;
        case EPI_BIAS_GELU: hipLaunchKernelGGL((xmm_wave_kernel<RT, EPI_BIAS_GELU>), grid, blk, 0, st, a); break;
        case EPI_GEGLU: hipLaunchKernelGGL((xmm_wave_kernel<RT, EPI_GEGLU>), grid, blk, 0, st, a); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int RT, bool R8, int EPI, bool PART, int VAR = 0>
static void launch_dec1(const XmmArgs& a, hipStream_t st) {
    using S = XDecShape<RT, R8>;
    auto k = xmm_dec_kernel<RT, R8, EPI, PART, VAR>;
    if (S::LDS > 64 * 1024) {   // once per device: opt in to more than 64 KiB of LDS
        static bool done[64];
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev >= 0 && dev < 64 && !done[dev]) {
            (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS);
            done[dev] = true;
        }
    }
    const int np = PART ? (a.KB + a.part_kbc - 1) / a.part_kbc : 1;
    hipLaunchKernelGGL(k, dim3((unsigned)a.NG, (unsigned)np), dim3(512), S::LDS, st, a);
}

template <int RT, bool R8>
static int launch_xmm_dec(const XmmArgs& a, int epi, hipStream_t st) {
    if (a.part_out) {
        launch_dec1<RT, R8, EPI_F32, true>(a, st);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    if (a.timing_var == 1 || a.timing_var == 2) {
        if (epi != EPI_BF16) return -1;
        if (a.timing_var == 1) launch_dec1<RT, R8, EPI_BF16, false, 1>(a, st);
        else launch_dec1<RT, R8, EPI_BF16, false, 2>(a, st);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    switch (epi) {
        case EPI_F32: launch_dec1<RT, R8, EPI_F32, false>(a, st); break;
        case EPI_BF16: launch_dec1<RT, R8, EPI_BF16, false>(a, st); break;
        case EPI_BIAS_BF16: launch_dec1<RT, R8, EPI_BIAS_BF16, false>(a, st); break;
        case EPI_BIAS_GELU: launch_dec1<RT, R8, EPI_BIAS_GELU, false>(a, st); break;
        case EPI_GEGLU: launch_dec1<RT, R8, EPI_GEGLU, false>(a, st); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int xmm(const XmmArgs& a, int epi, hipStream_t st) {
    if (a.M <= 0) return 0;
    if (!a.X16 || !a.W || (!a.Y && !a.Y16 && !a.part_out) || a.N <= 0 || a.KB <= 0 || a.NG % 4 || a.NG * 16 < a.N) return -1;
    if ((epi == EPI_BIAS_BF16 || epi == EPI_BIAS_GELU) && !a.bias) return -1;
    if (epi == EPI_GEGLU && a.N % 64) return -1;
    if (a.Y16 && (epi == EPI_F32 || (epi == EPI_GEGLU ? a.N % 64 : a.N % 32))) return -1;
    if (a.part_out) {   // parts: decode rows only, fp32 part values (no epilogue)
        if (a.M > 32 || a.part_kbc <= 0 || a.part_kbc >= a.KB || (a.KB + a.part_kbc - 1) / a.part_kbc > 8) return -1;
    }
    // decode rows: K of each group over the 8 waves of a workgroup
    if (a.M <= 8) return launch_xmm_dec<1, true>(a, epi, st);
    if (a.M <= 16) return launch_xmm_dec<1, false>(a, epi, st);
    if (a.M <= 32) return launch_xmm_dec<2, false>(a, epi, st);
    if (a.M <= 16) return launch_xmm_wave<1>(a, epi, st);
    if (a.M <= 32) return launch_xmm_wave<2>(a, epi, st);
    return launch_xmm_wave<4>(a, epi, st);
}

}  // namespace t5g

// Shared fp32 building blocks of the XCodec2 decoder (xc2.hip) and encoder (xc2enc.hip):
// the f32 MFMA GEMM over row-mapped operands, block sums, LayerNorm / RMSNorm rows.
// Internal linkage (anonymous namespace): each translation unit owns its copy.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace xc2 {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// row m of a GEMM -> physical row: (m / T) * seq + (m % T) + off
struct RowMap {
    int T, seq, off;
};
__device__ __forceinline__ long rowaddr(const RowMap& r, int m) {
    int b = m / r.T;
    int t = m - b * r.T;
    return (long)b * r.seq + t + r.off;
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float bsum(float v, float* red) {
    v = wsum(v);
    const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}
__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }

// --------------------------------------------------------------------------- GEMM
// EPI_LOG: log(max(v, 1.1920929e-7)); EPI_GELU: exact (erf) GELU; EPI_LOG10: log10(max(v, 1e-10))
enum { EPI_NONE = 0, EPI_SILU = 1, EPI_RELU = 2, EPI_LOG = 3, EPI_GELU = 4, EPI_LOG10 = 5 };

struct GemmArgs {
    const float* A;
    int lda;
    RowMap am;
    const float* W;   // [N][ldw] row-major
    int ldw;
    const float* bias;
    float* C;
    int ldc;
    RowMap cm;
    const float* resid;   // same map / ld as C (may alias C)
    const int* lens;      // with mask_T > 0: rows with t >= min(lens[b], mask_T) are written as 0
    int mask_T;
    int M, N, K, epi;
    float alpha;          // C = resid + alpha * epi(acc + bias); 0 is taken as 1
};

constexpr int BM = 128, BN = 128, BK = 32, LDT = BK + 4;

// 256 threads = 4 waves in 2x2; each wave owns a 64x64 tile = 2x2 MFMA 32x32 tiles.
// K is consumed in groups of 8: lane half h takes k = 8g + 4h + e in MFMA step e, so
// every operand fetch is one 16-byte LDS read per 4 MFMAs.
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs a) {
    __shared__ float As[2][BM * LDT];
    __shared__ float Ws[2][BN * LDT];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1, li = lane & 31, hh = lane >> 5;
    // XCD-aware order: consecutive tiles of one XCD share A rows in its L2
    const int ntn = (a.N + BN - 1) / BN;
    const int nb = gridDim.x;
    int L = blockIdx.x;
    if ((nb & 7) == 0) L = (L & 7) * (nb >> 3) + (L >> 3);
    const int m0 = (L / ntn) * BM, n0 = (L % ntn) * BN;

    const int lr = tid >> 3, lk = (tid & 7) * 4;
    const float* ap[4];
    const float* wp[4];
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // out-of-range rows read row 0 and are zeroed at LDS store time
        const int m = m0 + lr + 32 * i, n = n0 + lr + 32 * i;
        ap[i] = a.A + (m < a.M ? rowaddr(a.am, m) : rowaddr(a.am, 0)) * a.lda + lk;
        wp[i] = a.W + (long)(n < a.N ? n : 0) * a.ldw + lk;
    }
    const bool am_ok = m0 + BM <= a.M, wn_ok = n0 + BN <= a.N;
    f32x4 ra[4], rw[4];
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nk = a.K / BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ra[i] = *(const f32x4*)(ap[i]);
        rw[i] = *(const f32x4*)(wp[i]);
    }
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        // stage tile kt (registers -> LDS), then prefetch tile kt+1 into registers
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool va = am_ok || m0 + lr + 32 * i < a.M, vw = wn_ok || n0 + lr + 32 * i < a.N;
            *(f32x4*)&As[buf][(lr + 32 * i) * LDT + lk] = va ? ra[i] : z4;
            *(f32x4*)&Ws[buf][(lr + 32 * i) * LDT + lk] = vw ? rw[i] : z4;
        }
        __syncthreads();
        if (kt + 1 < nk) {
            const int k1 = (kt + 1) * BK;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                ra[i] = *(const f32x4*)(ap[i] + k1);
                rw[i] = *(const f32x4*)(wp[i] + k1);
            }
        }
        const float* as = As[buf];
        const float* ws = Ws[buf];
#pragma unroll
        for (int g = 0; g < BK / 8; ++g) {
            f32x4 fa[2], fb[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                fa[t] = *(const f32x4*)&as[(wm * 64 + t * 32 + li) * LDT + 8 * g + 4 * hh];
                fb[t] = *(const f32x4*)&ws[(wn * 64 + t * 32 + li) * LDT + 8 * g + 4 * hh];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][e], fb[j][e], acc[i][j], 0, 0, 0);
        }
    }
    // epilogue: C/D map col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 64 + j * 32 + li;
            const float bn = (a.bias && n < a.N) ? a.bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                float v = acc[i][j][r] + bn;
                if (m >= a.M || n >= a.N) continue;
                if (a.epi == EPI_SILU) v = silu(v);
                else if (a.epi == EPI_RELU) v = fmaxf(v, 0.f);
                else if (a.epi == EPI_LOG) v = logf(fmaxf(v, 1.1920929e-7f));
                else if (a.epi == EPI_GELU) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
                else if (a.epi == EPI_LOG10) v = log10f(fmaxf(v, 1e-10f));
                if (a.alpha != 0.f) v = a.alpha * v;
                const long row = rowaddr(a.cm, m);
                if (a.resid) v = a.resid[row * a.ldc + n] + v;
                if (a.mask_T > 0) {
                    const int b = m / a.cm.T;
                    const int lim = a.lens ? min(a.lens[b], a.mask_T) : a.mask_T;
                    if (m - b * a.cm.T >= lim) v = 0.f;
                }
                a.C[row * a.ldc + n] = v;
            }
        }
}

// measurement only (xc2_time_gemms): when set, every GEMM launch is bracketed by a pair of
// events from this pool and its 2 M N K flops are counted
struct GemmTimer {
    hipEvent_t* ev;   // 2 * cap events
    int cap, n;
    double flops;
};
static GemmTimer* g_gemm_timer = nullptr;

static int gemm(const GemmArgs& a, hipStream_t st) {
    if (a.M <= 0 || a.N <= 0) return 0;
    if (a.K <= 0 || a.K % BK || a.lda % 4 || a.ldw % 4) return -1;
    const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    GemmTimer* t = g_gemm_timer;
    if (t) {
        if (t->n >= t->cap) return -3;
        (void)hipEventRecord(t->ev[2 * t->n], st);
    }
    hipLaunchKernelGGL(gemm_f32_kernel, dim3(tiles), dim3(256), 0, st, a);
    if (t) {
        (void)hipEventRecord(t->ev[2 * t->n + 1], st);
        ++t->n;
        t->flops += 2.0 * a.M * a.N * a.K;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ------------------------------------------------------- RMSNorm / LayerNorm rows
// RMSNorm: [tf] Xcodec2RMSNorm :322-327  (w * (x * rsqrt(mean(x^2) + eps)))
// LayerNorm: nn.LayerNorm(eps 1e-6) before the head (:862).
__global__ __launch_bounds__(256) void rownorm_kernel(const float* X, float* Y, RowMap rm, int C, const float* w,
                                                      const float* bsh, float eps, int layer_norm) {
    __shared__ float red[8];
    const long row = rowaddr(rm, blockIdx.x);
    const int c = threadIdx.x * 4;
    const bool act = c < C;
    f32x4 x = {0.f, 0.f, 0.f, 0.f};
    if (act) x = *(const f32x4*)(X + row * C + c);
    f32x4 y;
    if (layer_norm) {
        const float mean = bsum((x[0] + x[1]) + (x[2] + x[3]), red) / (float)C;
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) ss += act ? (x[e] - mean) * (x[e] - mean) : 0.f;
        const float rstd = 1.0f / sqrtf(bsum(ss, red) / (float)C + eps);
        if (!act) return;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = (x[e] - mean) * rstd * w[c + e] + bsh[c + e];
    } else {
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) ss += x[e] * x[e];
        const float r = 1.0f / sqrtf(bsum(ss, red) / (float)C + eps);
        if (!act) return;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = w[c + e] * (x[e] * r);
    }
    *(f32x4*)(Y + row * C + c) = y;
}


}  // namespace
}  // namespace xc2

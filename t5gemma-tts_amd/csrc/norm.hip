// Row-wise fused residual + T5Gemma RMSNorm(1+w) + embedding kernels.
//
// One block per token row, one thread per 8 contiguous elements (16-byte bf16 /
// 2x16-byte fp32 loads, every load of the thread issued before the first use), so a
// decode-step row (d = 2304: 288 threads) costs one memory round trip plus two
// block reductions. Implements, in the reference's rounding order
// ([tf] T5GemmaRMSNorm :61-78; residual wiring PMDecoderLayer :285-323):
//   v   = ids ? bf16(table[id] * normalizer)            (embed x sqrt(d), [tf] :789-790)
//         : part ? bf16(sum_s part[s])                   (split-K slabs of a Linear)
//         : delta
//   v   = post_w ? bf16((v * (1/sqrt(mean(v^2)+eps))) * (1 + post_w)) : v
//   h   = resid ? bf16(resid + v) : v                    -> resid_out
//   out = pre_w ? bf16((h * (1/sqrt(mean(h^2)+eps))) * (1 + pre_w))   -> normed_out
// Sums reduce in a fixed order, so results are run-to-run deterministic.
#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

constexpr int NSPLIT_MAX = 8;

__device__ __forceinline__ void unpack8(u32x4 w, float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[2 * j] = bf_lo(w[j]);
        v[2 * j + 1] = bf_hi(w[j]);
    }
}
__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
    u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = pack2(v[2 * j], v[2 * j + 1]);
    return w;
}

__device__ __forceinline__ void rms8(float (&v)[8], bool active, int d, u32x4 w8, float eps, float* red) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    float tot = block_sum(active ? ss : 0.f, red);
    float r = 1.0f / sqrtf(tot / (float)d + eps);
    if (!active) return;
    float wf[8];
    unpack8(w8, wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf((v[j] * r) * (1.0f + wf[j]));
}

__global__ __launch_bounds__(1024) void resid_norm_kernel(NormArgs a) {
    __shared__ float red[32];
    const int mi = blockIdx.x;
    const int m = a.out_rows ? a.out_rows[mi] : mi;
    const int d = a.d;
    const int c = threadIdx.x;          // chunk of 8 elements
    const bool active = 8 * c < d;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float r8[8];
    u32x4 rw = {0u, 0u, 0u, 0u}, w_post = {0u, 0u, 0u, 0u}, w_pre = {0u, 0u, 0u, 0u};
    if (active) {
        // every load of the row is issued up front (one memory round trip)
        if (a.post_w) w_post = *(const u32x4*)(a.post_w + 8 * c);
        if (a.pre_w) w_pre = *(const u32x4*)(a.pre_w + 8 * c);
        if (a.resid) rw = *(const u32x4*)(a.resid + (long)m * d + 8 * c);
        if (a.ids) {
            unpack8(*(const u32x4*)(a.table + (long)a.ids[m] * d + 8 * c), v);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = rbf(v[j] * a.scale);
        } else if (a.part) {
            f32x4 p[NSPLIT_MAX][2];
#pragma unroll
            for (int s = 0; s < NSPLIT_MAX; ++s)
                if (s < a.nsplit) {
                    const f32x4* ps = (const f32x4*)(a.part + ((long)s * a.M + m) * a.ldp + 8 * c);
                    p[s][0] = ps[0];
                    p[s][1] = ps[1];
                }
#pragma unroll
            for (int s = 0; s < NSPLIT_MAX; ++s)
                if (s < a.nsplit) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        v[j] += p[s][0][j];
                        v[4 + j] += p[s][1][j];
                    }
                }
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = rbf(v[j]);
        } else {
            unpack8(*(const u32x4*)(a.delta + (long)m * d + 8 * c), v);
        }
    }
    if (a.post_w) rms8(v, active, d, w_post, a.eps, red);
    if (a.resid && active) {
        unpack8(rw, r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rbf(r8[j] + v[j]);
    }
    const long orow = a.out_rows ? (long)mi : (long)m;
    if (a.resid_out && active) *(u32x4*)(a.resid_out + orow * d + 8 * c) = pack8(v);
    if (a.pre_w) {
        rms8(v, active, d, w_pre, a.eps, red);
        if (active) *(u32x4*)(a.normed_out + orow * d + 8 * c) = pack8(v);
    }
}

int resid_norm(const NormArgs& a, hipStream_t st) {
    if (a.M <= 0) return 0;
    if (a.d % 8 || a.d > 8 * 1024 || a.nsplit > NSPLIT_MAX) return -1;
    const int threads = ((a.d / 8 + 63) / 64) * 64;
    hipLaunchKernelGGL(resid_norm_kernel, dim3((unsigned)a.M), dim3(threads), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

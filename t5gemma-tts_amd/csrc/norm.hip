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
#include "exact_dev.h"
#include "exact_math.h"
#include "t5g_kernels.h"

namespace t5g {

T5G_TS_UNIT(norm)

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

// block_sum without its leading barrier: each rms8 call of a launch gets its own `red`
// (nothing reads it before), so one barrier per reduction; the same fixed-order sum
__device__ __forceinline__ float block_sum_once(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int nw = (blockDim.x + 63) >> 6;
    if (l == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i];
    return s;
}

template <bool EXACT>
__device__ __forceinline__ void rms8(float (&v)[8], bool active, int d, u32x4 w8, float eps, float* red, float* sq) {
    if constexpr (EXACT) {
        rms8_exact(v, active, d, w8, eps, sq);   // exact_dev.h (shared with xlayer.hip)
        return;
    }
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    const float tot = block_sum_once(active ? ss : 0.f, red);
    float r = 1.0f / sqrtf(tot / (float)d + eps);
    if (!active) return;
    float wf[8];
    unpack8(w8, wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf((v[j] * r) * (1.0f + wf[j]));
}

// Every global load is unconditional and issued before the first use: optional
// operands are replaced host-side by a valid stand-in pointer (flags say what is real)
// and idle threads read the last chunk. A load guarded by a branch makes the
// compiler wait for every load in flight at the branch join (vmcnt(0)), which
// serialised two memory round trips here.
template <int NS, int SRC, bool EXACT = false>   // NS: split-K slabs of the part path; SRC: 0 delta, 1 ids, 2 part
__global__ __launch_bounds__(1024) void resid_norm_kernel(NormArgs a, int has_post, int has_resid, int has_pre) {
    __shared__ float red[2][32];   // one per RMSNorm of the launch
    __shared__ float sq[EXACT ? 8 * 1024 + 32 : 1];   // exact mode: squares + accumulator lanes
    T5G_TS(0);
    const int mi = blockIdx.x;
    if (a.rope_tab) {   // the decode step's per-row cos/sin table (used by every layer's attention)
        const int H2 = a.rope_D / 2;
        for (int i = threadIdx.x; i < H2; i += blockDim.x) {
            const float ang = a.rope_inv_freq[i] * a.rope_pos[mi];
            a.rope_tab[(long)mi * a.rope_D + i] =
                EXACT ? t5g_exact::rope_trig(ang, 0, a.trig_exc, a.n_trig_exc) : rbf(cosf(ang));
            a.rope_tab[(long)mi * a.rope_D + H2 + i] =
                EXACT ? t5g_exact::rope_trig(ang, 1, a.trig_exc, a.n_trig_exc) : rbf(sinf(ang));
        }
    }
    const int m = a.out_rows ? a.out_rows[mi] : mi;
    const int d = a.d;
    const int c = threadIdx.x;          // chunk of 8 elements
    const bool active = 8 * c < d;
    const int cc = active ? c : d / 8 - 1;   // idle threads re-read the last chunk
    const u32x4 w_post = *(const u32x4*)(a.post_w + 8 * cc);
    const u32x4 w_pre = *(const u32x4*)(a.pre_w + 8 * cc);
    const u32x4 rw = *(const u32x4*)(a.resid + (long)m * d + 8 * cc);
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (SRC == 1) {
        // the host rejects out-of-range ids (engine.py); the clamp only keeps a bad id
        // passed through the C ABI from reading outside the table
        const int id = min(max(a.ids[m], 0), a.n_table - 1);
        unpack8(*(const u32x4*)(a.table + (long)id * d + 8 * cc), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rbf(v[j] * a.scale);
    } else if constexpr (SRC == 2) {
        f32x4 p[NS > 0 ? NS : 1][2];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const f32x4* ps = (const f32x4*)(a.part + ((long)s * a.M + m) * a.ldp + 8 * cc);
            p[s][0] = ps[0];
            p[s][1] = ps[1];
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[j] = __fadd_rn(v[j], p[s][0][j]);
                v[4 + j] = __fadd_rn(v[4 + j], p[s][1][j]);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rbf(v[j]);
    } else {
        unpack8(*(const u32x4*)(a.delta + (long)m * d + 8 * cc), v);
    }
    if (has_post) rms8<EXACT>(v, active, d, w_post, a.eps, red[0], sq);
    T5G_TS(1);
    if (has_resid) {
        float r8[8];
        unpack8(rw, r8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rbf(r8[j] + v[j]);
    }
    const long orow = a.out_rows ? (long)mi : (long)m;
    if (a.resid_out && active) *(u32x4*)(a.resid_out + orow * d + 8 * c) = pack8(v);
    if (has_pre) {
        rms8<EXACT>(v, active, d, w_pre, a.eps, red[1], sq);
        if (active) {
            const u32x4 pk = pack8(v);
            *(u32x4*)(a.normed_out + orow * d + 8 * c) = pk;
            if (a.normed_x16) {   // the next exact Linear's operand order (xmm.hip): pair j -> slot q = j
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) *(uint32_t*)(a.normed_x16 + x16_off(orow, 8 * c + 2 * jj, d / 32)) = pk[jj];
            }
        }
    }
    T5G_TS(2);
}

int resid_norm(const NormArgs& a_in, hipStream_t st) {
    NormArgs a = a_in;
    if (a.M <= 0) return 0;
    if (a.d % 8 || a.d > 8 * 1024 || a.nsplit > NSPLIT_MAX) return -1;
    if (!a.resid_out && !a.normed_out) return -1;
    if (a.pre_w && !a.normed_out) return -1;
    const int has_post = a.post_w != nullptr, has_resid = a.resid != nullptr, has_pre = a.pre_w != nullptr;
    // stand-ins for absent operands: any readable buffer of the same extent
    const bf16_t* any_w = a.pre_w ? a.pre_w : a.post_w;
    const bf16_t* any_row = a.resid_out ? a.resid_out : a.normed_out;
    if (!any_w) any_w = any_row;
    if (!a.post_w) a.post_w = any_w;
    if (!a.pre_w) a.pre_w = any_w;
    if (!a.resid) a.resid = a.out_rows ? (a.delta ? a.delta : any_row) : any_row;
    const int threads = ((a.d / 8 + 63) / 64) * 64;
    const int src = a.ids ? 1 : (a.part ? 2 : 0);
    if (src == 0 && !a.delta) return -1;
    if (src == 1 && (!a.table || a.n_table <= 0)) return -1;
    if (src == 2 && (a.nsplit < 1 || a.nsplit > 8)) return -1;
    const dim3 g((unsigned)a.M), b(threads);
#define T5G_NORM(NS_, SRC_) \
    hipLaunchKernelGGL((resid_norm_kernel<NS_, SRC_>), g, b, 0, st, a, has_post, has_resid, has_pre)
    if (a.exact) {
        // parity mode: the reference's CPU sum order. Part slabs: the K parts of an exact
        // Linear (xmm part_out), v = bf16((0 + p0) + p1 ...) = the reference's fold of parts
        if (a.d > 8 * 1024 || (src == 2 && a.nsplit > 4)) return -1;
        if (src == 0) hipLaunchKernelGGL((resid_norm_kernel<0, 0, true>), g, b, 0, st, a, has_post, has_resid, has_pre);
        else if (src == 1) hipLaunchKernelGGL((resid_norm_kernel<0, 1, true>), g, b, 0, st, a, has_post, has_resid, has_pre);
        else if (a.nsplit == 1) hipLaunchKernelGGL((resid_norm_kernel<1, 2, true>), g, b, 0, st, a, has_post, has_resid, has_pre);
        else if (a.nsplit == 2) hipLaunchKernelGGL((resid_norm_kernel<2, 2, true>), g, b, 0, st, a, has_post, has_resid, has_pre);
        else if (a.nsplit == 3) hipLaunchKernelGGL((resid_norm_kernel<3, 2, true>), g, b, 0, st, a, has_post, has_resid, has_pre);
        else hipLaunchKernelGGL((resid_norm_kernel<4, 2, true>), g, b, 0, st, a, has_post, has_resid, has_pre);
    } else if (src == 0) T5G_NORM(0, 0);
    else if (src == 1) T5G_NORM(0, 1);
    else switch (a.nsplit) {
        case 1: T5G_NORM(1, 2); break;
        case 2: T5G_NORM(2, 2); break;
        case 3: T5G_NORM(3, 2); break;
        case 4: T5G_NORM(4, 2); break;
        case 5: T5G_NORM(5, 2); break;
        case 6: T5G_NORM(6, 2); break;
        case 7: T5G_NORM(7, 2); break;
        default: T5G_NORM(8, 2); break;
    }
#undef T5G_NORM
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

// ARCHIVED (round 6, not built): the side-stream Infinity Cache prefetch measured in
// DESIGN.md §4.6 -- it made every layer launch slower and was removed with its engine
// plumbing (t5g_engine_set_prefetch, PrefetchArgs in t5g_kernels.h, pf_fork / pf_join).
// Infinity Cache (MALL) prefetch of the next decoder layer's bytes, run beside the current
// layer's persistent launch on a second stream.
//
// A decode layer launch (fused_block_kernel / xlayer_kernel) spends most of its time in a
// chain of dependent stages (o-projection -> norms -> cross q -> cross attention -> ...)
// whose weight reads pay HBM latency, and HBM sits at ~2.6 TB/s of its ~6 TB/s meanwhile.
// The same launch repeated on ONE layer (its ~175 MB then resident in the 256 MiB Infinity
// Cache) takes 55 instead of 67 us (fast path) and 67 instead of 91 us (parity path)
// (tools/probe_mall_layer.py). This kernel streams layer l + 1's weights
// through the Infinity Cache while layer l runs, in the order layer l + 1 consumes them.
//
// Every byte is read with a plain vector buffer load into registers and folded into an xor
// that is stored only if it equals a constant (so the loads are kept); nothing is written
// otherwise. A load past a region's end reads 0 (buffer bounds), never faults.
// Co-residency: 4 waves of <= 64 VGPRs and no LDS per workgroup, so it fits beside one
// persistent-launch workgroup per CU (fused: 2 waves x 168 VGPRs per SIMD; xlayer: 2 x 216)
// and never keeps one of those from becoming resident.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

constexpr int PF_WAVES = 4;    // waves per workgroup (one per SIMD)
constexpr int PF_DEPTH = 10;   // 1 KiB wave loads in flight per wave (<= 64 VGPRs)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pf_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <int AUX>
__global__ __launch_bounds__(PF_WAVES * 64) void mall_prefetch_kernel(PrefetchArgs a) {
    const int lane = threadIdx.x & 63;
    const int w = (int)blockIdx.x * PF_WAVES + (int)(threadIdx.x >> 6);
    const int W = (int)gridDim.x * PF_WAVES;
    uint32_t acc = 0;
    for (int r = 0; r < a.n; ++r) {
        const __amdgpu_buffer_rsrc_t rs = pf_rsrc(a.base[r], a.bytes[r]);
        const int nch = (int)((a.bytes[r] + 1023u) >> 10);
        for (int c0 = w; c0 < nch; c0 += W * PF_DEPTH) {
            u32x4 v[PF_DEPTH];
#pragma unroll
            for (int u = 0; u < PF_DEPTH; ++u)
                v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, ((c0 + u * W) << 10) + lane * 16, 0, AUX));
#pragma unroll
            for (int u = 0; u < PF_DEPTH; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
        }
    }
    if (acc == 0x9e3779b9u && lane == 0) a.sink[0] = acc;
}

int mall_prefetch(const PrefetchArgs& a, int grid, int nt, hipStream_t st) {
    if (a.n <= 0) return 0;
    if (a.n > PF_MAX_REGIONS || !a.sink || grid <= 0) return -1;
    for (int r = 0; r < a.n; ++r)
        if (!a.base[r] || a.bytes[r] > 0x40000000u) return -1;   // byte offsets stay in int range
    if (nt) hipLaunchKernelGGL(mall_prefetch_kernel<2>, dim3((unsigned)grid), dim3(PF_WAVES * 64), 0, st, a);
    else hipLaunchKernelGGL(mall_prefetch_kernel<0>, dim3((unsigned)grid), dim3(PF_WAVES * 64), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

// The parity layer's gate/up stage (xlayer.hip stage G) in isolation: 1 152 groups of 16
// outputs x 72 exact chunks (K = 2 304) at 8 rows, weights streamed from HBM (4 weight sets
// rotated, 340 MB > the 256 MiB Infinity Cache), one 512-thread workgroup per CU, 248 workers
// with contiguous task runs, chunk sums folded in order by 128 folder threads (xl_fold) --
// the exact E / O chunk arithmetic in three forms, every one bitwise equal:
//   0  the product: v_mfma_f32_16x16x4_f32 E / O chains (exact_dev.h xmm_chunk), weights of a
//      pass double-buffered in registers in the E16 lane order, X16 window in LDS
//   1  VALU v_fma_f32: lane = (output j, row pair r), the four E16 fragments of output j
//      loaded by the 4 lanes that need them (4 x 16 B per chunk per lane), a 9-slot register
//      ring reloaded in place one pass ahead; X as f32 in LDS, one ds_read_b128 per k pair
//   2  as 1 with the E16 fragment loaded once (16 B per lane) and all-gathered over the four
//      16-lane rows with v_permlane32/16_swap
// Prints us per stage and the bitwise comparison of the folded outputs against variant 0.
// Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 -I t5gemma-tts_amd/csrc tools/micro_gstage.hip -o tools/bin/micro_gstage
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "common.h"
#include "exact_dev.h"

using namespace t5g;

constexpr int NG = 1152, KB = 72, M = 8, NW = 248, NSET = 4;
constexpr int CPW = 9;   // chunks per wave per pass
constexpr int EL = 128;  // chunk-sum elements: 8 rows x 16 outputs
constexpr size_t WSET = (size_t)NG * KB * 1024;   // bytes per weight set

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void run(int n, int workers, int w, int& lo, int& hi) {
    const int base = n / workers, extra = n - base * workers;
    lo = w * base + min(w, extra);
    hi = lo + base + (w < extra ? 1 : 0);
}

// fold of one pass (folder thread tid < 128), as xlayer.hip xl_fold
__device__ __forceinline__ float fold(const float* cs, int n, int tid, float part) {
    for (int c0 = 0; c0 < n; c0 += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = cs[min(c0 + u, KB - 1) * EL + tid];
        if (c0 + 16 <= n) {
#pragma unroll
            for (int u = 0; u < 16; ++u) part = __fadd_rn(part, v[u]);
        } else {
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (c0 + u < n) part = __fadd_rn(part, v[u]);
        }
    }
    return part;
}

// ---------------------------------------------------------------- variant 0: MFMA
struct W9 {
    u32x4 w[CPW];
};
template <int STRIDED, int AUX, int MODE = 0>
__global__ __launch_bounds__(512) void g_mfma(const bf16_t* __restrict__ Wset, const u32x4* __restrict__ X16,
                                              float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    u32x4* xs = (u32x4*)smem;                       // 72 chunks x 32 lanes x 16 B = 36 KB
    float* cs0 = (float*)(smem + 72 * 1024);
    float* cs1 = cs0 + KB * EL;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, bu = blockIdx.x;
    if (bu >= NW) return;
    int t0, t1;
    if (STRIDED) {   // task i of worker bu = group bu + i * NW (the per-op GEMV's unit order)
        t0 = 0;
        t1 = (NG - bu + NW - 1) / NW;
    } else {
        run(NG, NW, bu, t0, t1);
    }
    auto gid = [&](int i) { return STRIDED ? bu + i * NW : i; };
    const __amdgpu_buffer_rsrc_t wr = rsrc(Wset, (uint32_t)WSET);
    auto issue = [&](W9& o, int i) {
        const int g = gid(i);
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            int off = ((g * KB + wave + c * 8) * 64 + lane) * 16;
            asm volatile("" : "+v"(off));
            o.w[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, AUX));
        }
    };
    W9 wa, wb;
    issue(wa, t0);
    for (int i = tid; i < KB * 32; i += 512) xs[i] = X16[i];
    lds_barrier();
    float acc = 0.f;
    const int j = lane & 15, q = lane >> 4;
    const u32x4* xl = xs + q * 8 + (lane & 7);
    auto pass = [&](W9& cur, W9& nxt, int g, float* cs) {
        if (MODE == 3) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                nxt.w[c] = cur.w[c];
                asm volatile("" : "+v"(nxt.w[c]));
            }
        } else if (g + 1 < t1) issue(nxt, g + 1);
        if constexpr (MODE == 0) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                const int cc = wave + c * 8;
                const f32x4_t v = xmm_chunk(cur.w[c], xl[cc * 32]);
                if (j < 8) *(f32x4_t*)&cs[cc * EL + j * 16 + 4 * q] = v;
            }
        } else {
            u32x4 x = cur.w[0];
#pragma unroll
            for (int c = 1; c < CPW; ++c) x ^= cur.w[c];
            const f32x4_t v = {__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[2]), __uint_as_float(x[3])};
            if (j < 8) *(f32x4_t*)&cs[wave * EL + j * 16 + 4 * q] = v;
            if constexpr (MODE == 2) return;
        }
        lds_barrier();
        if (tid < EL) {
            acc = fold(cs, KB, tid, 0.f);
            Y[((long)gid(g) * 16 + (tid & 15)) * M + (tid >> 4)] = acc;
        }
    };
    for (int g = t0; g < t1; g += 2) {
        pass(wa, wb, g, cs0);
        if (g + 1 < t1) pass(wb, wa, g + 1, cs1);
    }
}

// ---------------------------------------------------------------- variants 1 / 2: VALU
// X f32 window: xf[(c * 16 + p) * 4 + r] = {x[2r][2p], x[2r+1][2p], x[2r][2p+1], x[2r+1][2p+1]}
// (k = 32 c + 2 p): one ds_read_b128 per k pair gives the lane its two rows' E and O operands
__device__ __forceinline__ void chunk_valu(const u32x4 (&w)[4], const f32x4* xp, float& c0, float& c1) {
    float e0 = 0.f, e1 = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) {
        const uint32_t ww = w[p & 3][p >> 2];
        const float wl = bf_lo(ww), wh = bf_hi(ww);
        const f32x4 x = xp[p * 4];
        e0 = fmaf(wl, x[0], e0);
        e1 = fmaf(wl, x[1], e1);
        o0 = fmaf(wh, x[2], o0);
        o1 = fmaf(wh, x[3], o1);
    }
    c0 = __fadd_rn(e0, o0);
    c1 = __fadd_rn(e1, o1);
}

template <int VAR>
__global__ __launch_bounds__(512) void g_valu(const bf16_t* __restrict__ Wset, const f32x4* __restrict__ Xf,
                                              float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f32x4* xs = (f32x4*)smem;                       // 72 chunks x 1 KB
    float* cs0 = (float*)(smem + 72 * 1024);
    float* cs1 = cs0 + KB * EL;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, bu = blockIdx.x;
    if (bu >= NW) return;
    int t0, t1;
    run(NG, NW, bu, t0, t1);
    const int j = lane & 15, r = lane >> 4;
    const __amdgpu_buffer_rsrc_t wr = rsrc(Wset, (uint32_t)WSET);
    // VAR 1: the four 16-B pieces of output j's fragment (lanes q * 16 + j of E16)
    // VAR 2: this lane's own piece (E16 lane order), gathered after the load
    constexpr int NP = VAR == 2 ? 1 : 4;
    u32x4 w[CPW][NP];
    auto issue = [&](int c, int g, bool live) {
        const int cc = wave + c * 8;
        int off = live ? (g * KB + cc) * 1024 : 0x7ffff000;   // past num_records: no fetch, zeros
#pragma unroll
        for (int q = 0; q < NP; ++q) {
            int o = off + (VAR != 2 ? (q * 16 + j) : lane) * 16;
            asm volatile("" : "+v"(o));
            w[c][q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, o, 0, 0));
        }
    };
#pragma unroll
    for (int c = 0; c < CPW; ++c) issue(c, t0, true);
    for (int i = tid; i < KB * 64; i += 512) xs[i] = Xf[i];
    lds_barrier();
    const f32x4* xl = xs + r;
    for (int g = t0; g < t1; ++g) {
        float* cs = ((g - t0) & 1) ? cs1 : cs0;
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            const int cc = wave + c * 8;
            u32x4 w4[4];
            if constexpr (VAR != 2) {
#pragma unroll
                for (int q = 0; q < 4; ++q) w4[q] = w[c][0 + q];
            } else {
                // all-gather of the 4 rows' pieces: row q's word t = pair 4t + q of output j
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t a = w[c][0][t];
                    const auto s32 = __builtin_amdgcn_permlane32_swap(a, a, false, false);   // [a0 a1 a0 a1], [a2 a3 a2 a3]
                    const auto s0 = __builtin_amdgcn_permlane16_swap(s32[0], s32[0], false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(s32[1], s32[1], false, false);
                    w4[0][t] = s0[0];
                    w4[1][t] = s0[1];
                    w4[2][t] = s1[0];
                    w4[3][t] = s1[1];
                }
            }
            float c0, c1;
            chunk_valu(w4, xl + cc * 64, c0, c1);
            cs[cc * EL + (2 * r) * 16 + j] = c0;
            cs[cc * EL + (2 * r + 1) * 16 + j] = c1;
            if constexpr (VAR == 11) {
#pragma unroll
                for (int q2 = 0; q2 < 4; ++q2) asm volatile("" : "+v"(w[c][q2]));
            } else {
                issue(c, g + 1, g + 1 < t1);
            }
        }
        lds_barrier();
        if (tid < EL) {
            const float acc = fold(cs, KB, tid, 0.f);
            Y[((long)g * 16 + (tid & 15)) * M + (tid >> 4)] = acc;
        }
    }
}


// ---------------------------------------------------------------- variants 3 / 4: 3 passes in flight
// the E16 fragment once per lane (16 B per chunk, 4 VGPRs): a ring of 3 passes x 9 chunks held
// in registers, slot (pass % 3, chunk) reloaded with pass + 3's chunk right after its use, so
// ~2.5 passes (180 KB per CU) stay in flight. VAR 3: VALU via the permlane all-gather; VAR 4:
// the MFMA E / O chains on the same registers.
template <int VAR>
__global__ __launch_bounds__(512) void g_ring(const bf16_t* __restrict__ Wset, const f32x4* __restrict__ Xf,
                                              const u32x4* __restrict__ X16, float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f32x4* xs = (f32x4*)smem;                       // VAR 3: 72 chunks x 1 KB f32; VAR 4: X16 36 KB
    float* cs0 = (float*)(smem + 72 * 1024);
    float* cs1 = cs0 + KB * EL;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, bu = blockIdx.x;
    if (bu >= NW) return;
    int t0, t1;
    run(NG, NW, bu, t0, t1);
    const int j = lane & 15, r = lane >> 4, q = lane >> 4;
    const __amdgpu_buffer_rsrc_t wr = rsrc(Wset, (uint32_t)WSET);
    u32x4 ring[3][CPW];
    auto issue = [&](u32x4& dst, int c, int g) {
        const int cc = wave + c * 8;
        int off = g < t1 ? ((g * KB + cc) * 64 + lane) * 16 : 0x7ffff000;
        asm volatile("" : "+v"(off));
        dst = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
    };
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int c = 0; c < CPW; ++c) issue(ring[u][c], c, t0 + u);
    if constexpr (VAR == 3) {
        for (int i = tid; i < KB * 64; i += 512) xs[i] = Xf[i];
    } else {
        for (int i = tid; i < KB * 32; i += 512) ((u32x4*)xs)[i] = X16[i];
    }
    lds_barrier();
    auto pass = [&](u32x4 (&w)[CPW], int g, float* cs) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            const int cc = wave + c * 8;
            if constexpr (VAR == 3) {
                u32x4 w4[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t a = w[c][t];
                    const auto s32 = __builtin_amdgcn_permlane32_swap(a, a, false, false);
                    const auto s0 = __builtin_amdgcn_permlane16_swap(s32[0], s32[0], false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(s32[1], s32[1], false, false);
                    w4[0][t] = s0[0];
                    w4[1][t] = s0[1];
                    w4[2][t] = s1[0];
                    w4[3][t] = s1[1];
                }
                float c0, c1;
                chunk_valu(w4, xs + r + cc * 64, c0, c1);
                cs[cc * EL + (2 * r) * 16 + j] = c0;
                cs[cc * EL + (2 * r + 1) * 16 + j] = c1;
            } else {
                const u32x4* xl = (const u32x4*)xs + q * 8 + (lane & 7);
                const f32x4_t v = xmm_chunk(w[c], xl[cc * 32]);
                if (j < 8) *(f32x4_t*)&cs[cc * EL + j * 16 + 4 * q] = v;
            }
            issue(w[c], c, g + 3);
        }
        lds_barrier();
        if (tid < EL) {
            const float acc = fold(cs, KB, tid, 0.f);
            Y[((long)g * 16 + (tid & 15)) * M + (tid >> 4)] = acc;
        }
    };
    for (int g = t0; g < t1; g += 3) {
        pass(ring[0], g, ((g - t0) & 1) ? cs1 : cs0);
        if (g + 1 < t1) pass(ring[1], g + 1, ((g + 1 - t0) & 1) ? cs1 : cs0);
        if (g + 2 < t1) pass(ring[2], g + 2, ((g + 2 - t0) & 1) ? cs1 : cs0);
    }
}


// ---------------------------------------------------------------- variant 12 / 13: lane = output
// a pass = 64 outputs (4 groups) x 72 chunks; lane o = output 16 gi + j holds all 16 k pairs of
// its output (the four 16-B pieces q * 16 + j of group gi's E16 fragment, 4 loads per chunk, no
// replication) and all 8 rows (E / O accumulators), X f32 [chunk][k][8 rows] read by uniform
// (broadcast) ds_read_b128. Rounds: every wave computes one chunk per round (chunk 8 s + wave),
// writes its 8 rows' chunk sums to an LDS slot, and after the round's barrier wave w folds row w
// of the round's 8 chunks in order. Worker bu: groups [4 bu, 4 bu + 4), then (bu < 160) the
// 16-output pass of group 992 + bu (lanes >= 16 idle). Weights of round n + R requested at round n.
template <int R>
__global__ __launch_bounds__(512) void g_lo(const bf16_t* __restrict__ Wset, const float* __restrict__ Xk,
                                            float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* xs = (float*)smem;                               // [72][32][8] f32 = 72 KB
    float* cs = (float*)(smem + 72 * 1024);                 // [2][8 chunks][8 rows][64] = 32 KB
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, bu = blockIdx.x;
    if (bu >= NW) return;
    const int npass = bu < NG - 4 * NW ? 2 : 1, nround = npass * CPW;
    const int gi = lane >> 4, j = lane & 15;
    const __amdgpu_buffer_rsrc_t wr = rsrc(Wset, (uint32_t)WSET);
    auto g0_of = [&](int pass) { return pass == 0 ? 4 * bu : 4 * NW + bu; };
    auto issue = [&](u32x4 (&w)[4], int n) {
        const int pass = n / CPW, sc = n - pass * CPW, cc = wave + 8 * sc;
        const bool live = n < nround && (pass == 0 || gi == 0);
        const int base = live ? ((g0_of(pass) + gi) * KB + cc) * 1024 + j * 16 : 0x7ffff000;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            int o = base + q * 256;
            asm volatile("" : "+v"(o));
            w[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, o, 0, 2));
        }
    };
    u32x4 ring[R][4];
#pragma unroll
    for (int u = 0; u < R; ++u) issue(ring[u], u);
    for (int i = tid; i < KB * 256; i += 512) xs[i] = Xk[i];
    lds_barrier();
    float acc = 0.f;
    auto round = [&](u32x4 (&w)[4], int n) {
        const int pass = n / CPW, sc = n - pass * CPW, cc = wave + 8 * sc;
        float e[8], o[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) e[m] = o[m] = 0.f;
        const f32x4* xp = (const f32x4*)(xs + cc * 256);
#pragma unroll
        for (int p = 0; p < 16; ++p) {
            const uint32_t ww = w[p & 3][p >> 2];
            const float wl = bf_lo(ww), wh = bf_hi(ww);
            const f32x4 xa = xp[p * 4], xb = xp[p * 4 + 1], xc = xp[p * 4 + 2], xd = xp[p * 4 + 3];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                e[m] = fmaf(wl, xa[m], e[m]);
                e[4 + m] = fmaf(wl, xb[m], e[4 + m]);
                o[m] = fmaf(wh, xc[m], o[m]);
                o[4 + m] = fmaf(wh, xd[m], o[4 + m]);
            }
        }
        float* slot = cs + (n & 1) * 4096;
#pragma unroll
        for (int m = 0; m < 8; ++m) slot[(wave * 8 + m) * 64 + lane] = __fadd_rn(e[m], o[m]);
        issue(w, n + R);
        lds_barrier();
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = slot[(c * 8 + wave) * 64 + lane];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc = __fadd_rn(acc, v[c]);
        if (sc == CPW - 1) {
            if (pass == 0 || gi == 0) Y[((long)(g0_of(pass) + gi) * 16 + j) * M + wave] = acc;
            acc = 0.f;
        }
    };
    for (int n = 0; n < nround; n += R) {
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (n + u < nround) round(ring[u], n + u);
    }
}


// ---------------------------------------------------------------- variant 14 / 15: prefetch kept
// variant 0 with every weight request unconditional (a pass past the worker's run requests an
// out-of-range offset: no fetch) and every pass of the unrolled pair run (compute, fold and
// store predicated): the compiler's vmcnt for a chunk then counts the next pass's requests as
// younger, instead of waiting for them (a conditional issue merges to the smaller count)
template <int AUX, int BIS = 0>
__global__ __launch_bounds__(512) void g_fix(const bf16_t* __restrict__ Wset, const u32x4* __restrict__ X16,
                                             float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    u32x4* xs = (u32x4*)smem;
    float* cs0 = (float*)(smem + 72 * 1024);
    float* cs1 = cs0 + KB * EL;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, bu = blockIdx.x;
    if (bu >= NW) return;
    int t0, t1;
    run(NG, NW, bu, t0, t1);
    const __amdgpu_buffer_rsrc_t wr = rsrc(Wset, (uint32_t)WSET);
    auto issue = [&](W9& o, int g) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            int off = g < t1 ? ((g * KB + wave + c * 8) * 64 + lane) * 16 : 0x7ffff000;
            asm volatile("" : "+v"(off));
            o.w[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, AUX));
        }
    };
    W9 wa, wb;
    issue(wa, t0);
    for (int i = tid; i < KB * 32; i += 512) xs[i] = X16[i];
    lds_barrier();
    const int j = lane & 15, q = lane >> 4;
    const u32x4* xl = xs + q * 8 + (lane & 7);
    auto pass = [&](W9& cur, W9& nxt, int g, float* cs) {
        issue(nxt, g + 1);
        if (g < t1) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                const int cc = wave + c * 8;
                u32x4 xv = (BIS & 4) ? u32x4{0x3f80u, 0x3f80u, 0x3f80u, 0x3f80u} : xl[cc * 32];
                if ((BIS & 8) && j >= 8) xv = u32x4{0u, 0u, 0u, 0u};   // the duplicate columns zero (no toggling)
                f32x4_t v;
                if constexpr (BIS & 1) {
                    f32x4_t e = {0.f, 0.f, 0.f, 0.f}, o = e;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        e = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(cur.w[c][t]), __uint_as_float(xv[t]), e, 0, 0, 0);
                        o = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(cur.w[c][t] ^ 1u), __uint_as_float(xv[t]), o, 0, 0, 0);
                    }
                    v = e + o;
                } else {
                    v = xmm_chunk(cur.w[c], xv);
                }
                if (j < 8) *(f32x4_t*)&cs[cc * EL + j * 16 + 4 * q] = v;
            }
        }
        lds_barrier();
        if ((BIS & 2) && g < t1 && tid < EL) {
            Y[((long)g * 16 + (tid & 15)) * M + (tid >> 4)] = cs[tid];
        } else if (g < t1 && tid < EL) {
            const float acc = fold(cs, KB, tid, 0.f);
            Y[((long)g * 16 + (tid & 15)) * M + (tid >> 4)] = acc;
        }
    };
    for (int g = t0; g < t1; g += 2) {
        pass(wa, wb, g, cs0);
        pass(wb, wa, g + 1, cs1);
    }
}


// ---------------------------------------------------------------- variants 16 / 17: interaction
// the stream of variant 15 consumed by a cheap xor (as variant 9), beside independent work of the
// product's size per chunk: 16: 8 v_mfma_f32_16x16x4_f32 on register operands not fed by the
// loads; 17: 64 v_fma_f32 likewise -- whether the matrix or vector work itself slows the stream
template <int KIND>
__global__ __launch_bounds__(512) void g_side(const bf16_t* __restrict__ Wset, float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* cs0 = (float*)(smem + 72 * 1024);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, bu = blockIdx.x;
    if (bu >= NW) return;
    int t0, t1;
    run(NG, NW, bu, t0, t1);
    const __amdgpu_buffer_rsrc_t wr = rsrc(Wset, (uint32_t)WSET);
    auto issue = [&](W9& o, int g) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            int off = g < t1 ? ((g * KB + wave + c * 8) * 64 + lane) * 16 : 0x7ffff000;
            asm volatile("" : "+v"(off));
            o.w[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 2));
        }
    };
    W9 wa, wb;
    issue(wa, t0);
    f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
    float fa = (float)lane, fb = 1.0001f;
    u32x4 sink = {0u, 0u, 0u, 0u};
    auto pass = [&](W9& cur, W9& nxt, int g) {
        issue(nxt, g + 1);
        if (g < t1) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                if constexpr (KIND == 16) {
#pragma unroll
                    for (int t = 0; t < 8; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, acc, 0, 0, 0);
                } else if constexpr (KIND == 18) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, acc, 0, 0, 0);
                } else if constexpr (KIND == 19) {
#pragma unroll
                    for (int t = 0; t < 16; ++t) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(fa, fb, acc, 0, 0, 0);
                } else if constexpr (KIND == 20) {
                    // the product's chunk: two chains of 4 interleaved (E / O), operands from the loads
                    f32x4_t e = {0.f, 0.f, 0.f, 0.f}, o = e;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        e = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fb, e, 0, 0, 0);
                        o = __builtin_amdgcn_mfma_f32_16x16x4f32(fb, fa, o, 0, 0, 0);
                    }
                    acc += e + o;
                } else {
#pragma unroll
                    for (int t = 0; t < 64; ++t) fa = fmaf(fa, fb, 0.5f);
                }
                sink ^= cur.w[c];
            }
        }
        asm volatile("s_barrier" ::: "memory");
    };
    for (int g = t0; g < t1; g += 2) {
        pass(wa, wb, g);
        pass(wb, wa, g + 1);
    }
    cs0[tid] = acc[0] + acc[1] + fa + __uint_as_float(sink[0] ^ sink[1] ^ sink[2] ^ sink[3]);
    if (cs0[(tid + 1) & 511] == 123.f) Y[0] = 1.f;
}


// ---------------------------------------------------------------- variant 25: 2 passes ahead
// variant 15 with three register buffers: pass g requests pass g + 2's weights (unconditional,
// out of range past the run), every pass of the 3-way unrolled loop runs (compute predicated)
template <int AUX>
__global__ __launch_bounds__(512) void g_fix3(const bf16_t* __restrict__ Wset, const u32x4* __restrict__ X16,
                                              float* __restrict__ Y) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    u32x4* xs = (u32x4*)smem;
    float* cs0 = (float*)(smem + 72 * 1024);
    float* cs1 = cs0 + KB * EL;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, bu = blockIdx.x;
    if (bu >= NW) return;
    int t0, t1;
    run(NG, NW, bu, t0, t1);
    const __amdgpu_buffer_rsrc_t wr = rsrc(Wset, (uint32_t)WSET);
    auto issue = [&](W9& o, int g) {
#pragma unroll
        for (int c = 0; c < CPW; ++c) {
            int off = g < t1 ? ((g * KB + wave + c * 8) * 64 + lane) * 16 : 0x7ffff000;
            asm volatile("" : "+v"(off));
            o.w[c] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, AUX));
        }
    };
    W9 wa, wb, wc;
    issue(wa, t0);
    issue(wb, t0 + 1);
    for (int i = tid; i < KB * 32; i += 512) xs[i] = X16[i];
    lds_barrier();
    const int j = lane & 15, q = lane >> 4;
    const u32x4* xl = xs + q * 8 + (lane & 7);
    auto pass = [&](W9& cur, W9& nxt2, int g) {
        float* cs = ((g - t0) & 1) ? cs1 : cs0;
        issue(nxt2, g + 2);
        if (g < t1) {
#pragma unroll
            for (int c = 0; c < CPW; ++c) {
                const int cc = wave + c * 8;
                const f32x4_t v = xmm_chunk(cur.w[c], xl[cc * 32]);
                if (j < 8) *(f32x4_t*)&cs[cc * EL + j * 16 + 4 * q] = v;
            }
        }
        lds_barrier();
        if (g < t1 && tid < EL) {
            const float acc = fold(cs, KB, tid, 0.f);
            Y[((long)g * 16 + (tid & 15)) * M + (tid >> 4)] = acc;
        }
    };
    for (int g = t0; g < t1; g += 3) {
        pass(wa, wc, g);
        pass(wb, wa, g + 1);
        pass(wc, wb, g + 2);
    }
}

static uint32_t hs(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
static uint16_t rb(uint32_t s) {   // a random finite bf16 of moderate range
    const uint32_t h = hs(s);
    const float m = (float)((int)(h & 0xffff) - 32768) / 32768.0f;
    const int e = (int)((h >> 16) % 8) - 4;
    float f = ldexpf(m, e);
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)(u >> 16);
}

int main(int argc, char** argv) {
    // argv[1]: weight sets rotated over (1: the same 85 MB set every launch, resident in the
    // Infinity Cache; NSET: every launch from HBM)
    const int rot = argc > 1 ? max(1, min(NSET, atoi(argv[1]))) : NSET;
    // weights: random bf16, the same bytes read as E16 by every variant
    std::vector<uint16_t> hw(WSET / 2);
    bf16_t* dW;
    hipMalloc(&dW, WSET * NSET);
    for (int s = 0; s < NSET; ++s) {
        for (size_t i = 0; i < hw.size(); ++i) hw[i] = rb((uint32_t)(i * 2654435761u + s * 977u + 11));
        hipMemcpy((char*)dW + WSET * s, hw.data(), WSET, hipMemcpyHostToDevice);
    }
    // X [8][2304] bf16 -> X16 and the f32 window
    std::vector<uint16_t> x(M * KB * 32);
    for (size_t i = 0; i < x.size(); ++i) x[i] = rb((uint32_t)(i * 7919u + 5));
    auto xf = [&](int m, int k) {
        uint32_t u = (uint32_t)x[m * KB * 32 + k] << 16;
        float f;
        memcpy(&f, &u, 4);
        return f;
    };
    std::vector<uint32_t> h16(KB * 32 * 4);
    for (int c = 0; c < KB; ++c)
        for (int q = 0; q < 4; ++q)
            for (int m = 0; m < 8; ++m)
                for (int t = 0; t < 4; ++t) {
                    const int p = 4 * t + q, k = 32 * c + 2 * p;
                    h16[((c * 32) + q * 8 + m) * 4 + t] = (uint32_t)x[m * KB * 32 + k] | ((uint32_t)x[m * KB * 32 + k + 1] << 16);
                }
    std::vector<float> hf(KB * 64 * 4);
    for (int c = 0; c < KB; ++c)
        for (int p = 0; p < 16; ++p)
            for (int r = 0; r < 4; ++r) {
                const int k = 32 * c + 2 * p, b = ((c * 16 + p) * 4 + r) * 4;
                hf[b + 0] = xf(2 * r, k);
                hf[b + 1] = xf(2 * r + 1, k);
                hf[b + 2] = xf(2 * r, k + 1);
                hf[b + 3] = xf(2 * r + 1, k + 1);
            }
    std::vector<float> hk(KB * 32 * 8);
    for (int c = 0; c < KB; ++c)
        for (int k = 0; k < 32; ++k)
            for (int m = 0; m < 8; ++m) hk[(c * 32 + k) * 8 + m] = xf(m, 32 * c + k);
    float* dXk;
    hipMalloc(&dXk, hk.size() * 4);
    hipMemcpy(dXk, hk.data(), hk.size() * 4, hipMemcpyHostToDevice);
    u32x4* dX16;
    f32x4* dXf;
    hipMalloc(&dX16, h16.size() * 4);
    hipMalloc(&dXf, hf.size() * 4);
    hipMemcpy(dX16, h16.data(), h16.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dXf, hf.data(), hf.size() * 4, hipMemcpyHostToDevice);
    constexpr int NV = 28;
    float* dY[NV];
    for (int v = 0; v < NV; ++v) {
        hipMalloc(&dY[v], (size_t)NG * 16 * M * 4);
        hipMemset(dY[v], 0, (size_t)NG * 16 * M * 4);
    }
    const size_t shm = 72 * 1024 + 2 * KB * EL * 4;
    hipFuncSetAttribute((const void*)g_mfma<0, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_mfma<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_mfma<1, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_mfma<0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_mfma<0, 2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_mfma<0, 2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_mfma<0, 2, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_valu<11>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_lo<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_lo<9>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_side<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_side<17>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_side<18>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_side<19>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_side<20>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix<2, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix<2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix<2, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix<2, 7>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix3<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix3<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_fix<2, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_valu<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_valu<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_ring<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    hipFuncSetAttribute((const void*)g_ring<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    const char* names[NV] = {"MFMA 16x16x4 E/O (product)", "VALU lane=(out,row pair), 4x16B loads",
                             "VALU lane=(out,row pair), 16B load + permlane gather", "VALU gather, 3-pass register ring",
                             "MFMA, 3-pass register ring", "MFMA, strided tasks", "MFMA, strided tasks, nt loads",
                             "MFMA, contiguous runs, nt loads", "no MFMA (xor), fold, nt", "stream only (xor), nt",
                             "MFMA compute + fold only (no loads)", "VALU var 1 compute + fold only (no loads)",
                             "VALU lane=output, 64-out passes, rounds, ring 3", "VALU lane=output, ring 9",
                             "MFMA, unconditional prefetch", "MFMA, unconditional prefetch, nt",
                             "stream (nt) + independent MFMAs", "stream (nt) + independent VALU fma",
                             "stream + 4 indep. 16x16x4 per chunk", "stream + 16 indep. 4x4x1 per chunk",
                             "stream + 2 chains of 4 16x16x4 per chunk", "var 15, no weight conversion",
                             "var 15, no fold", "var 15, x constant (no LDS x)", "var 15, none of the three",
                             "MFMA, 2 passes ahead, nt", "MFMA, 2 passes ahead", "var 15, duplicate B columns zero"};
    std::vector<float> ref((size_t)NG * 16 * M), got((size_t)NG * 16 * M);
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < NV; ++v) {
            if (v != 0 && v != 9 && v != 10 && v != 15 && v != 24) continue;
            auto launch = [&](int s) {
                const bf16_t* W = (const bf16_t*)((char*)dW + WSET * s);
                if (v == 0) hipLaunchKernelGGL((g_mfma<0, 0>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 5) hipLaunchKernelGGL((g_mfma<1, 0>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 6) hipLaunchKernelGGL((g_mfma<1, 2>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 7) hipLaunchKernelGGL((g_mfma<0, 2>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 8) hipLaunchKernelGGL((g_mfma<0, 2, 1>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 9) hipLaunchKernelGGL((g_mfma<0, 2, 2>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 10) hipLaunchKernelGGL((g_mfma<0, 2, 3>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 11) hipLaunchKernelGGL(g_valu<11>, dim3(256), dim3(512), shm, 0, W, dXf, dY[v]);
                else if (v == 12) hipLaunchKernelGGL(g_lo<3>, dim3(256), dim3(512), shm, 0, W, dXk, dY[v]);
                else if (v == 13) hipLaunchKernelGGL(g_lo<9>, dim3(256), dim3(512), shm, 0, W, dXk, dY[v]);
                else if (v == 14) hipLaunchKernelGGL(g_fix<0>, dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 15) hipLaunchKernelGGL(g_fix<2>, dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 16) hipLaunchKernelGGL(g_side<16>, dim3(256), dim3(512), shm, 0, W, dY[v]);
                else if (v == 17) hipLaunchKernelGGL(g_side<17>, dim3(256), dim3(512), shm, 0, W, dY[v]);
                else if (v == 18) hipLaunchKernelGGL(g_side<18>, dim3(256), dim3(512), shm, 0, W, dY[v]);
                else if (v == 19) hipLaunchKernelGGL(g_side<19>, dim3(256), dim3(512), shm, 0, W, dY[v]);
                else if (v == 20) hipLaunchKernelGGL(g_side<20>, dim3(256), dim3(512), shm, 0, W, dY[v]);
                else if (v == 21) hipLaunchKernelGGL((g_fix<2, 1>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 22) hipLaunchKernelGGL((g_fix<2, 2>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 23) hipLaunchKernelGGL((g_fix<2, 4>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 24) hipLaunchKernelGGL((g_fix<2, 7>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 25) hipLaunchKernelGGL(g_fix3<2>, dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 26) hipLaunchKernelGGL(g_fix3<0>, dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 27) hipLaunchKernelGGL((g_fix<2, 8>), dim3(256), dim3(512), shm, 0, W, dX16, dY[v]);
                else if (v == 1) hipLaunchKernelGGL(g_valu<1>, dim3(256), dim3(512), shm, 0, W, dXf, dY[v]);
                else if (v == 2) hipLaunchKernelGGL(g_valu<2>, dim3(256), dim3(512), shm, 0, W, dXf, dY[v]);
                else if (v == 3) hipLaunchKernelGGL(g_ring<3>, dim3(256), dim3(512), shm, 0, W, dXf, dX16, dY[v]);
                else if (v == 4) hipLaunchKernelGGL(g_ring<4>, dim3(256), dim3(512), shm, 0, W, dXf, dX16, dY[v]);
            };
            for (int s = 0; s < NSET; ++s) launch(s);
            hipDeviceSynchronize();
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            const int iters = 40;
            hipEventRecord(e0);
            for (int i = 0; i < iters; ++i) launch(i % rot);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const hipError_t err = hipGetLastError();
            const double us = ms * 1000.0 / iters;
            printf("rot %d rep %d var %d %-52s %7.2f us/stage  %6.1f GB/s  (%s)\n", rot, rep, v, names[v], us,
                   (double)WSET / (us * 1e3), hipGetErrorString(err));
            // outputs of the last launch (weight set (iters - 1) % rot) vs variant 0's
            hipMemcpy(v == 0 ? ref.data() : got.data(), dY[v], ref.size() * 4, hipMemcpyDeviceToHost);
            if (v > 0) {
                size_t bad = 0;
                for (size_t i = 0; i < ref.size(); ++i) bad += memcmp(&ref[i], &got[i], 4) != 0;
                printf("      bitwise vs variant 0: %zu / %zu differ\n", bad, ref.size());
            }
            fflush(stdout);
        }
    return 0;
}

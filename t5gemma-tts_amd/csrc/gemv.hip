// Decode-step weight-streaming GEMM (M <= 16 rows): Y[M][N] = X[M][K] . W[N][K]^T on
// v_mfma_f32_16x16x32_bf16 over the P16 packed weights (gemm.hip), at most one block per
// CU. A block owns whole row-group "units" (16 outputs each, GeGLU: 8 gate + the same 8
// features' up rows) for its K range: its NW waves split each group's K stream (k-step kb
// belongs to wave kb % WPG) and reduce through LDS in fixed wave order, so every output
// is deterministic and independent of the batch composition. The X rows (<= 16 x K bf16)
// are staged through LDS once per block while the first weight fragments are in flight.
// Optional split-K over blockIdx.y writes fp32 slabs (EPI_F32) for the consumer to sum.
// The decode step runs its gate/up projection here (engine.hip decoder_pass).
#include <algorithm>
#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

// Work split: the NG/RG "units" (RG row groups each) are dealt round-robin to at most
// one block per CU (grid <= #CUs), so the prologue runs once per CU however many units
// a block streams; each wave's k-steps over its units form ONE register-double-buffered
// stream (UN fragments in flight, the next unit's fragments already requested while the
// current unit finishes). A unit's partial sums go to LDS when its last k-step is done.
template <int NW, int RG, int EPI, int UN>
__global__ __launch_bounds__(NW * 64) void gemv_dec_kernel(DecGemmArgs a) {
    constexpr int WPG = NW / RG;   // waves sharing one row group's K stream
    extern __shared__ __attribute__((aligned(16))) char smem[];   // one LDS object (no extra waits)
    const int nb = (int)gridDim.x;
    const int bu = (int)blockIdx.x;
    const int nunits = a.NG / RG;
    const int nu = (nunits - bu + nb - 1) / nb;   // units of this block
    const int umax = (nunits + nb - 1) / nb;
    f32x4* red = (f32x4*)smem;                               // [umax][NW][64]
    bf16_t* xs = (bf16_t*)(smem + (size_t)umax * NW * 1024);  // [M][K + 8] staged / normed X rows

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int gw = wave / WPG, ks = wave % WPG;
    const int KB = a.KB;
    // split-K (EPI_F32 only): blockIdx.y owns k-steps [kb_lo, kb_lo + KBs), fp32 slab y
    const int per = (KB + a.splits - 1) / a.splits;
    const int kb_lo = (int)blockIdx.y * per;
    const int KBs = max(0, min(KB, kb_lo + per) - kb_lo);
    const int spu = (KBs + WPG - 1) / WPG;   // k-steps per unit of every wave
    const int total = nu * spu;
    const int ldsx = KBs * 32 + 8;   // +16 B row pad spreads the 16 row reads over banks
    const int xr = lane & 15;
    const __amdgpu_buffer_rsrc_t wr = frag_rsrc(a.W, (uint32_t)a.NG * (uint32_t)KB * 1024u);
    // byte offset of this lane's fragment for (unit i, step j); past the stream -> out of
    // range of the descriptor: zeros, no traffic
    auto woff = [&](int i, int j) -> int __attribute__((always_inline)) {
        const int kb = ks + j * WPG;
        const int g = (bu + i * nb) * RG + gw;
        return (i < nu && kb < KBs) ? ((g * KB + kb_lo + kb) * 64 + lane) * 16 : (int)0xfffffff0u;
    };
    auto wload = [&](int off) __attribute__((always_inline)) {
        return __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 2));   // nt
    };

    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int ip = 0, jp = 0;   // (unit, step) of the next fragment to request
    int ic = 0, jc = 0;   // (unit, step) of the next fragment to multiply
    auto adv = [&](int& i, int& j) __attribute__((always_inline)) {
        if (++j == spu) {
            j = 0;
            ++i;
        }
    };
    // after the MFMA of (ic, jc): a finished unit's partial sums go to LDS
    auto retire = [&]() __attribute__((always_inline)) {
        if (jc == spu - 1) {   // wave-uniform
            // the padded tail of the stream (steps past nu units, loop rounds to 2*UN)
            // must not store: red holds umax units and the staged X rows follow it in
            // LDS, still being read by the other waves (intermittent wrong outputs)
            if (ic < nu) red[(ic * NW + wave) * 64 + lane] = acc;
            acc = (f32x4){0.f, 0.f, 0.f, 0.f};
        }
        adv(ic, jc);
    };
    // The stream is padded to whole batches: steps past it load zeros (out of the
    // descriptor), and their MFMAs add exact zeros, so no per-step predicate. The two
    // batches A/B are explicit ping-pong registers: no copy between them, so waits are
    // counted (vmcnt(UN)) and a full batch stays in flight behind the one multiplied.
    bf16x8_s wa[UN], wb[UN];
    auto wbatch = [&](bf16x8_s(&w)[UN]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < UN; ++u) {
            w[u] = wload(woff(ip, jp));
            adv(ip, jp);
        }
    };
    {
        // X staging loads first (oldest in the in-order vmcnt queue), then the first
        // weight batch, so the staging stores run while weights stream in: every chunk of
        // the block's rows, all requested at once
        constexpr int XCH = 10;
        const int CH = KBs * 4, tot = a.M * CH;
        const bf16_t* X0 = a.X + kb_lo * 32;
        u32x4 xv[XCH];
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int idx = max(0, min((int)threadIdx.x + NW * 64 * i, tot - 1));
            const int r = idx / max(CH, 1), c = idx - r * CH;
            xv[i] = *(const u32x4*)(X0 + (long)r * a.ldx + 8 * c);
        }
        wbatch(wa);
#pragma unroll
        for (int i = 0; i < XCH; ++i) {
            const int idx = (int)threadIdx.x + NW * 64 * i;
            if (idx < tot) {
                const int r = idx / CH, c = idx - r * CH;
                *(u32x4*)(xs + r * ldsx + 8 * c) = xv[i];
            }
        }
        __syncthreads();
        // X fragment of k-step kb for this lane (rows >= M read row M-1 and are zeroed;
        // steps past K read the last valid k-step: multiplied by zero weights)
        const bf16_t* xrow = xs + min(xr, a.M - 1) * ldsx + 8 * (lane >> 4);
        const bool xlive = xr < a.M;
        auto mul = [&](bf16x8_s(&w)[UN]) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const int kb = max(0, min(ks + jc * WPG, KBs - 1));
                const bf16x8_s xv = *(const bf16x8_s*)(xrow + kb * 32);
                acc = mfma16(w[u], xlive ? xv : (bf16x8_s){0, 0, 0, 0, 0, 0, 0, 0}, acc);
                retire();
            }
        };
        for (int q = 0; q < total; q += 2 * UN) {
            wbatch(wb);
            mul(wa);
            wbatch(wa);
            mul(wb);
        }
    }
    __syncthreads();

    // GeGLU: a row group is 8 gate rows then the same 8 features' up rows, so one row
    // group is one output group of 8 features: lanes 0-31 hold its gate sums, lanes 32-63
    // the up sums of the same (feature, batch row)
    constexpr bool GLU = EPI == EPI_GEGLU;
    constexpr int OG = RG;   // output groups per unit
    const int m = xr;
    if (m >= a.M || (GLU && lane >= 32)) return;
    const int n_out = GLU ? a.N / 2 : a.N;
    for (int t = wave; t < nu * OG; t += NW) {
        const int i = t / OG, og = t - i * OG;
        const f32x4* ri = red + (size_t)i * NW * 64 + lane;
        const int n0 = ((bu + i * nb) * OG + og) * (GLU ? 8 : 16) + 4 * (lane >> 4);
        float v[4];
        if constexpr (GLU) {
            f32x4 gs = {0.f, 0.f, 0.f, 0.f}, us = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < WPG; ++s) {
                gs += ri[(og * WPG + s) * 64];
                us += ri[(og * WPG + s) * 64 + 32];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = rbf(gelu_tanh(rbf(gs[r]))) * rbf(us[r]);
        } else {
            f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < WPG; ++s) s4 += ri[(og * WPG + s) * 64];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = s4[r];
        }
        if constexpr (EPI == EPI_F32) {
            float* y = (float*)a.Y + ((long)blockIdx.y * a.M + m) * a.ldy;
            if (n0 + 3 < n_out && (a.ldy & 3) == 0) {
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
                if constexpr (EPI == EPI_BIAS_BF16 || EPI == EPI_BIAS_GELU) {
                    if (n0 + r < n_out) x = x + bf2f(a.bias[n0 + r]);
                }
                if constexpr (EPI == EPI_BIAS_GELU) x = gelu_erf(rbf(x));
                o[r] = f2bf(x);
            }
            bf16_t* y = (bf16_t*)a.Y + (long)m * a.ldy;
            if (n0 + 3 < n_out && (a.ldy & 3) == 0) {
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
}

// ---------------------------------------------------------------------------
// Register-resident X variant for 1..32 rows (MT = 1 or 2 sixteen-row MFMA tiles): all
// NW waves share each unit's K stream (wave ks takes k-steps ks, ks + NW, ...: SPU of
// them, a compile-time count, so one unit = one batch of SPU fragments per wave), and the
// X fragments of a wave's k-steps never change from unit to unit -- they are loaded once
// into registers before the stream starts. No X staging in LDS (32 rows x K = 2304 would
// not fit beside the partial sums) and no barrier before the first MFMA. Batches are
// double-buffered per unit: unit i + 1's fragments are in flight while unit i multiplies.
// Per-row results are bitwise those of gemv_dec_kernel (same k-step order per wave, same
// fixed-order wave reduction).
// UMAX > 0: every unit's weight batch is requested before the first multiply (up to UMAX
// units per block held in registers) instead of one unit ahead -- the block's whole weight
// stream is in flight from the start.
template <int NW, int MT, int EPI, int SPU, int UMAX = 0>
__global__ __launch_bounds__(NW * 64) void gemv_rx_kernel(DecGemmArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f32x4* red = (f32x4*)smem;   // [umax][MT][NW][64]
    const int nb = (int)gridDim.x, bu = (int)blockIdx.x;
    const int nu = (a.NG - bu + nb - 1) / nb;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int KB = a.KB;
    const int per = (KB + a.splits - 1) / a.splits;
    const int kb_lo = (int)blockIdx.y * per;
    const int KBs = max(0, min(KB, kb_lo + per) - kb_lo);
    const int xr = lane & 15;
    const __amdgpu_buffer_rsrc_t wr = frag_rsrc(a.W, (uint32_t)a.NG * (uint32_t)KB * 1024u);
    auto wbatch = [&](int i, bf16x8_s(&w)[SPU]) __attribute__((always_inline)) {
        const int g = bu + i * nb;
#pragma unroll
        for (int j = 0; j < SPU; ++j) {
            const int kb = wave + j * NW;
            const int off = (i < nu && kb < KBs) ? ((g * KB + kb_lo + kb) * 64 + lane) * 16 : (int)0xfffffff0u;
            w[j] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 2));
        }
    };
    bf16x8_s wa[SPU], wb[SPU];
    bf16x8_s wall[UMAX > 0 ? UMAX : 1][SPU];
    if constexpr (UMAX > 0) {
#pragma unroll
        for (int i = 0; i < UMAX; ++i) wbatch(i, wall[i]);
    } else {
        wbatch(0, wa);
    }
    // this wave's X fragments (rows >= M and k-steps past the slice are zero)
    bf16x8_s xf[MT][SPU];
    const bf16x8_s z8 = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int row = 16 * t + xr;
        const bf16_t* xp = a.X + (long)min(row, a.M - 1) * a.ldx + kb_lo * 32 + 8 * (lane >> 4);
#pragma unroll
        for (int j = 0; j < SPU; ++j) {
            const int kb = min(wave + j * NW, KBs - 1);
            const bf16x8_s v = *(const bf16x8_s*)(xp + kb * 32);
            xf[t][j] = (row < a.M && wave + j * NW < KBs) ? v : z8;
        }
    }
    auto mul = [&](int i, bf16x8_s(&w)[SPU]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < SPU; ++j) acc = mfma16(w[j], xf[t][j], acc);
            if (i < nu) red[((i * MT + t) * NW + wave) * 64 + lane] = acc;
        }
    };
    if constexpr (UMAX > 0) {
#pragma unroll
        for (int i = 0; i < UMAX; ++i) mul(i, wall[i]);   // units past nu: zero batches, results dropped
    } else {
        for (int i = 0; i < nu; i += 2) {
            wbatch(i + 1, wb);
            mul(i, wa);
            wbatch(i + 2, wa);
            mul(i + 1, wb);
        }
    }
    __syncthreads();

    constexpr bool GLU = EPI == EPI_GEGLU;
    if (GLU && lane >= 32) return;
    const int n_out = GLU ? a.N / 2 : a.N;
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int m = 16 * t + xr;
        if (m >= a.M) continue;
        for (int i = wave; i < nu; i += NW) {
            const f32x4* ri = red + (size_t)(i * MT + t) * NW * 64 + lane;
            const int n0 = (bu + i * nb) * (GLU ? 8 : 16) + 4 * (lane >> 4);
            float v[4];
            if constexpr (GLU) {
                f32x4 gs = {0.f, 0.f, 0.f, 0.f}, us = gs;
#pragma unroll
                for (int s2 = 0; s2 < NW; ++s2) {
                    gs += ri[s2 * 64];
                    us += ri[s2 * 64 + 32];
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = rbf(gelu_tanh(rbf(gs[r]))) * rbf(us[r]);
            } else {
                f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s2 = 0; s2 < NW; ++s2) s4 += ri[s2 * 64];
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = s4[r];
            }
            if constexpr (EPI == EPI_F32) {
                float* y = (float*)a.Y + ((long)blockIdx.y * a.M + m) * a.ldy;
                for (int r = 0; r < 4; ++r)
                    if (n0 + r < n_out) y[n0 + r] = v[r];
            } else {
                bf16_t* y = (bf16_t*)a.Y + (long)m * a.ldy;
                for (int r = 0; r < 4; ++r) {
                    float x = v[r];
                    if constexpr (EPI == EPI_BIAS_BF16 || EPI == EPI_BIAS_GELU) {
                        if (n0 + r < n_out) x = x + bf2f(a.bias[n0 + r]);
                    }
                    if constexpr (EPI == EPI_BIAS_GELU) x = gelu_erf(rbf(x));
                    if (n0 + r < n_out) y[n0 + r] = f2bf(x);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
constexpr size_t GD_LDS_MAX = 160 * 1024;   // gfx950: 160 KB LDS per workgroup

static int cu_count() {
    static int n[T5G_MAX_DEVICES] = {};
    const int dev = t5g_cur_device();
    if (dev < 0) return 256;
    if (!n[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        n[dev] = v;
    }
    return n[dev];
}

// blocks of one launch: <= one per CU (the X rows are staged once per block)
static int gd_grid(const DecGemmArgs& a, int rg) {
    const int units = a.NG / rg;
    if (a.splits > 1) return units;   // split-K: one unit per block
    const int cap = a.max_grid > 0 ? a.max_grid : cu_count();
    return units < cap ? units : cap;
}

template <int NW, int RG, int EPI, int UN>
static void launch_gd_un(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    auto* fn = gemv_dec_kernel<NW, RG, EPI, UN>;
    static bool attr[T5G_MAX_DEVICES] = {};   // one opt-in per instantiation and device
    const int dev = t5g_cur_device();
    if (dev >= 0 && !attr[dev]) {
        (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GD_LDS_MAX);
        attr[dev] = true;
    }
    hipLaunchKernelGGL(fn, dim3((unsigned)gd_grid(a, RG), (unsigned)a.splits), dim3(NW * 64), shm, st, a);
}

// fragments in flight per wave, kept spill-free (VGPR budget 512 / waves per SIMD)
template <int NW, int RG, int EPI>
static void launch_gd(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    constexpr int UND = NW >= 16 ? 8 : 16;
    if (UND == 16 && a.un == 8) launch_gd_un<NW, RG, EPI, 8>(a, shm, st);
    else launch_gd_un<NW, RG, EPI, UND>(a, shm, st);
}

template <int EPI>
static int launch_nw(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    // one row group per unit: at 2b-2b gate/up 1152 units balance over the CUs (4.5 per
    // block) far better than 576 two-group units
    if (a.nw == 4) launch_gd<4, 1, EPI>(a, shm, st);
    else if (a.nw == 8) launch_gd<8, 1, EPI>(a, shm, st);
    else if (a.nw == 16 && EPI != EPI_GEGLU) launch_gd<16, 1, EPI>(a, shm, st);
    else return -1;
    return 0;
}

size_t gemv_dec_lds_bytes(const DecGemmArgs& a, int rg) {
    const int grid = gd_grid(a, rg);
    const int umax = (a.NG / rg + grid - 1) / grid;
    const int per = (a.KB + a.splits - 1) / a.splits;
    return (size_t)umax * a.nw * 64 * 16 + (size_t)a.M * (per * 32 + 8) * sizeof(bf16_t);
}

// the register-resident-X kernel for the shapes it is instantiated for: PER k-steps per
// K slice (72: K = 2304 unsplit; 36: the down projection's K = 9216 in 8 slices; 8 / 16 /
// 18 / 32: the attention projections' slices), SPU =
// PER / NW per wave -- 0 if launched. Split-K launches put cu_count / splits blocks on each
// slice, so every block streams several units against one register-held X slice.
template <int NW, int MT, int EPI, int PER>
static int launch_rx_nw(const DecGemmArgs& a, hipStream_t st) {
    static_assert(PER % NW == 0, "whole k-step batches per wave");
    constexpr int SPU = PER / NW;
    const int cap = a.max_grid > 0 ? a.max_grid : cu_count();
    const int grid = a.splits > 1 ? std::max(1, std::min(a.NG, cap / a.splits)) : gd_grid(a, 1);
    const int umax = (a.NG + grid - 1) / grid;
    const size_t shm = (size_t)umax * MT * NW * 64 * 16;
    if (shm > GD_LDS_MAX) return -1;
    // un = -1 (tuning): the whole per-block weight stream requested up front, for blocks of
    // <= 5 units whose batches fit the register budget (SPU * 5 fragments per wave)
    bool all = false;
    auto* fn = gemv_rx_kernel<NW, MT, EPI, SPU, 0>;
    if constexpr (MT == 1 && SPU <= 6) {
        all = a.un == -1 && umax <= 5;
        if (all) fn = gemv_rx_kernel<NW, MT, EPI, SPU, 5>;
    }
    static bool attr[T5G_MAX_DEVICES][2] = {};
    const int dev = t5g_cur_device();
    if (dev >= 0 && !attr[dev][all]) {
        (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GD_LDS_MAX);
        attr[dev][all] = true;
    }
    hipLaunchKernelGGL(fn, dim3((unsigned)grid, (unsigned)a.splits), dim3(NW * 64), shm, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
// a.nw picks the waves sharing each unit's K stream (the PER k-steps split evenly; the
// decode gate/up runs 12: 17.9 vs 18.5 us for 8 at 8 rows, tools/probe_rx_nw.py)
template <int MT, int EPI, int PER>
static int launch_rx(const DecGemmArgs& a, hipStream_t st) {
    switch (a.nw) {
        case 4: if constexpr (PER % 4 == 0) return launch_rx_nw<4, MT, EPI, PER>(a, st); else return -1;
        case 6: if constexpr (PER % 6 == 0) return launch_rx_nw<6, MT, EPI, PER>(a, st); else return -1;
        case 9: if constexpr (PER % 9 == 0) return launch_rx_nw<9, MT, EPI, PER>(a, st); else return -1;
        case 12: if constexpr (PER % 12 == 0) return launch_rx_nw<12, MT, EPI, PER>(a, st); else return -1;
        case 8: if constexpr (PER % 8 == 0) return launch_rx_nw<8, MT, EPI, PER>(a, st); else return -1;
        default: return -1;   // a wave split the kernel is not built for (a different sum order)
    }
}
template <int MT>
static int launch_rx_slabs(const DecGemmArgs& a, int per, hipStream_t st) {
    switch (per) {
        case 8: return launch_rx<MT, EPI_F32, 8>(a, st);
        case 16: return launch_rx<MT, EPI_F32, 16>(a, st);
        case 18: return launch_rx<MT, EPI_F32, 18>(a, st);
        case 32: return launch_rx<MT, EPI_F32, 32>(a, st);
        case 36: return launch_rx<MT, EPI_F32, 36>(a, st);
        default: return -1;
    }
}

int gemv_rx(const DecGemmArgs& a, int epi, hipStream_t st) {
    if (a.M <= 0 || a.M > 32 || a.K != a.KB * 32 || a.NG % 4 || a.NG * 16 < a.N) return -1;
    if (a.splits < 1 || a.KB % a.splits) return -1;
    const int per = a.KB / a.splits;
    // unsplit K = 2304 (any epilogue), or fp32 slabs of 8 / 16 / 18 / 32 / 36-k-step
    // slices (the decode projections' split-K shapes)
    if (!(per == 72 && a.splits == 1) && !(a.splits > 1 && epi == EPI_F32)) return -1;
    if (!a.X || a.ldx < a.K || a.ldx % 8) return -1;
    if ((epi == EPI_BIAS_BF16 || epi == EPI_BIAS_GELU) && !a.bias) return -1;
    const bool two = a.M > 16;
    switch (epi) {
        case EPI_BF16: return two ? launch_rx<2, EPI_BF16, 72>(a, st) : launch_rx<1, EPI_BF16, 72>(a, st);
        case EPI_BIAS_BF16: return two ? launch_rx<2, EPI_BIAS_BF16, 72>(a, st) : launch_rx<1, EPI_BIAS_BF16, 72>(a, st);
        case EPI_BIAS_GELU: return two ? launch_rx<2, EPI_BIAS_GELU, 72>(a, st) : launch_rx<1, EPI_BIAS_GELU, 72>(a, st);
        case EPI_GEGLU: return two ? launch_rx<2, EPI_GEGLU, 72>(a, st) : launch_rx<1, EPI_GEGLU, 72>(a, st);
        case EPI_F32: return two ? launch_rx_slabs<2>(a, per, st) : launch_rx_slabs<1>(a, per, st);
        default: return -1;
    }
}

int gemv_dec(const DecGemmArgs& a, int epi, hipStream_t st) {
    if (a.M <= 0) return 0;
    if (a.layout_rx) return gemv_rx(a, epi, st);
    if (a.M > 16 || a.K % 32 || a.KB * 32 != a.K || a.NG % 4 || a.NG * 16 < a.N) return -1;
    if (a.splits < 1 || a.splits > 64 || (a.splits > 1 && epi != EPI_F32)) return -1;
    if (a.nw != 4 && a.nw != 8 && a.nw != 16) return -1;
    if (!a.X || a.ldx < a.K || a.ldx % 8) return -1;
    if ((epi == EPI_BIAS_BF16 || epi == EPI_BIAS_GELU) && !a.bias) return -1;
    const size_t shm = gemv_dec_lds_bytes(a, 1);
    if (shm > GD_LDS_MAX) return -1;
    if (a.M * ((a.KB + a.splits - 1) / a.splits) * 4 > a.nw * 64 * 10) return -1;   // XCH staging chunks
    int rc;
    switch (epi) {
        case EPI_BF16: rc = launch_nw<EPI_BF16>(a, shm, st); break;
        case EPI_BIAS_BF16: rc = launch_nw<EPI_BIAS_BF16>(a, shm, st); break;
        case EPI_GEGLU: rc = launch_nw<EPI_GEGLU>(a, shm, st); break;
        case EPI_F32: rc = launch_nw<EPI_F32>(a, shm, st); break;
        default: return -1;
    }
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

// Decode MLP half of a decoder layer as ONE persistent launch (one workgroup per CU):
//
//   stage N (M workgroups):  h = h + RMSNorm_post(sum of the cross-o slabs); xn = RMSNorm_pre(h)
//   stage G (every workgroup): act = GeGLU(xn . Wgate/up^T)            (gemv_rx_kernel's units)
//   stage D (every workgroup): down slabs[s] = act[:, slice s] . Wdown^T (8 k-slices)
//
// replacing resid_norm_kernel<4,2> + gemv_rx_kernel<12,..,GEGLU> + gemv_rx_kernel<12,..,F32>
// (PMDecoderLayer cross-attention residual + T5GemmaMLP, [tf] modeling_t5gemma.py:81-97,
// hf_export/modeling_t5gemma_voice.py:256-323). What the launch buys is overlap: every
// workgroup requests its whole gate/up weight stream BEFORE the normed rows exist, and its
// down weights before the act slice it multiplies is complete, so the two weight streams
// run back to back while the norm and the hand-offs happen underneath them. Two launch
// boundaries, the norm's launch and the fill / drain of two GEMV launches go away.
//
// Hand-offs (gfx950 recipe, cdna_hip_programming.md Guideline 16 R1): the handed-off
// bytes (xn rows, act) are stored write-through (sc1) by every storing wave, each storing
// wave drains (vmcnt(0)), the workgroup meets at a barrier, ONE lane adds to a relaxed
// agent-scope counter (one per 128-byte line); the consumer polls that counter relaxed from
// ONE wave (which has no weight loads queued ahead of the poll), the workgroup meets at a
// barrier, and every load of the handed-off bytes is an sc1 load. Counter sets start at
// zero (zeroed at engine creation and by the host after a timeout); each decoder layer has
// its own set, and each launch zeroes the NEXT layer's set as it starts (that set's last
// user has completed), so no arrival count is needed at the end. Every wait is bounded:
// a wait that gives up stores a
// timeout code that makes every later wait give up at once (outputs are then garbage and
// the host raises, t5g_read_tokens); no wave can spin forever.
//
// Numerics: every stage is the exact arithmetic of the kernels it replaces (the same
// per-wave k-step chains, the same fixed-order wave reductions, the same norm reductions),
// so the fused launch is bitwise equal to the three launches (tests/test_gpu_fused.py).
#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

T5G_TS_UNIT(fused)

constexpr int FM_NW = 12;         // waves per workgroup (the gate/up and down kernels' count)
constexpr int FM_NS = 4;          // cross-o split-K slabs read by the norm stage
constexpr int FM_DS = 8;          // down-projection k-slices
constexpr int FM_NORM_UNITS = 3;  // gate/up units of a norm workgroup (tools/diag_fused.py)
constexpr unsigned FM_SPIN_MAX = 1u << 18;   // ~0.3-0.5 s of polling before a wait gives up

// lines of a counter set (FusedMlpArgs::sync), one word per 128-byte line
constexpr int L_N1 = 0, L_Q0 = 1, L_A0 = 9, L_O0 = 17, L_N2 = 25, L_SL0 = 26, L_D0 = 34, L_N3 = 42, L_P0 = 43,
              L_S0 = 51, L_K0 = 59;
static_assert(L_K0 + 8 == FM_SET_LINES, "counter set layout");
__device__ __forceinline__ unsigned* cline(unsigned* set, int line) { return set + line * FM_LINE; }
constexpr int FS_NORM = L_N2 * FM_LINE;
__device__ __forceinline__ int fs_slice(int s) { return (L_SL0 + s) * FM_LINE; }

__device__ __forceinline__ unsigned ld_rlx(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one wave polls N counter lines of a set at once (lane i reads line line0 + i, lane 63 the
// timeout word): every round is ONE memory round trip whatever N is; true when every line
// has reached `target`, false on a timeout (this wait's or an earlier one's)
template <int N>
__device__ __forceinline__ bool fm_wait_n(unsigned* set, int line0, unsigned target, unsigned* tmo, unsigned code) {
    static_assert(N >= 1 && N < 64, "lines per poll");
    const int lane = threadIdx.x & 63;
    unsigned* p = lane == 63 ? tmo : set + (line0 + min(lane, N - 1)) * FM_LINE;
    for (unsigned spins = 0;; ++spins) {
        const unsigned v = ld_rlx(p);
        if (__all(lane == 63 || v >= target)) return true;
        if (__shfl(v, 63, 64) != 0) return false;
        if (spins > FM_SPIN_MAX) {
            if (lane == 0) __hip_atomic_store(tmo, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// the same over 8 lines that share `total` arrivals round-robin (arrival k goes to line
// k % 8): line i waits for (total - i + 7) / 8
template <int N>
__device__ __forceinline__ bool fm_wait_split(unsigned* set, int line0, unsigned total, unsigned* tmo, unsigned code) {
    static_assert(N >= 1 && N < 64, "lines per poll");
    const int lane = threadIdx.x & 63;
    const int li = min(lane, N - 1);
    unsigned* p = lane == 63 ? tmo : set + (line0 + li) * FM_LINE;
    const unsigned target = (total + (unsigned)(N - 1 - li)) / (unsigned)N;
    for (unsigned spins = 0;; ++spins) {
        const unsigned v = ld_rlx(p);
        if (__all(lane == 63 || v >= target)) return true;
        if (__shfl(v, 63, 64) != 0) return false;
        if (spins > FM_SPIN_MAX) {
            if (lane == 0) __hip_atomic_store(tmo, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// workgroup rendezvous with no memory semantics for the compiler to add waits for (the
// weight loads in flight must stay in flight across it); the "memory" clobber keeps the
// handed-off loads below it
__device__ __forceinline__ void wg_barrier() { asm volatile("s_barrier" ::: "memory"); }
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr int AUX_NT = 2, AUX_SC1 = 16;
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void unpack8f(u32x4 w, float (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[2 * j] = bf_lo(w[j]);
        v[2 * j + 1] = bf_hi(w[j]);
    }
}
__device__ __forceinline__ u32x4 pack8f(const float (&v)[8]) {
    u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = pack2(v[2 * j], v[2 * j + 1]);
    return w;
}
// norm.hip's block_sum_once over this launch's 12 waves: the waves past the 288 active
// threads add +0.0f after the 5 real wave sums, which leaves the (non-negative) total
// bitwise unchanged -- the same value as the 288-thread resid_norm launch
__device__ __forceinline__ float fm_block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
    for (int i = 0; i < FM_NW; ++i) s += red[i];
    return s;
}
__device__ __forceinline__ void fm_rms8(float (&v)[8], bool active, int d, u32x4 w8, float eps, float* red) {
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    const float tot = fm_block_sum(active ? ss : 0.f, red);
    const float r = 1.0f / sqrtf(tot / (float)d + eps);
    if (!active) return;
    float wf[8];
    unpack8f(w8, wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf((v[j] * r) * (1.0f + wf[j]));
}

// Stage N for row m (resid_norm_kernel<4, 2> with post, resid and pre): xn published sc1.
__device__ __forceinline__ void fm_norm_row(const FusedMlpArgs& a, int m, float* red) {
    const int d = a.d;
    const int c = threadIdx.x;
    const bool active = 8 * c < d;
    const int cc = active ? c : d / 8 - 1;
    const u32x4 w_post = *(const u32x4*)(a.post_w + 8 * cc);
    const u32x4 w_pre = *(const u32x4*)(a.pre_w + 8 * cc);
    const u32x4 rw = *(const u32x4*)(a.h + (long)m * d + 8 * cc);
    f32x4 p[FM_NS][2];
#pragma unroll
    for (int s = 0; s < FM_NS; ++s) {
        const f32x4* ps = (const f32x4*)(a.part_in + ((long)s * a.M + m) * d + 8 * cc);
        p[s][0] = ps[0];
        p[s][1] = ps[1];
    }
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < FM_NS; ++s) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] += p[s][0][j];
            v[4 + j] += p[s][1][j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf(v[j]);
    fm_rms8(v, active, d, w_post, a.eps, red);
    float r8[8];
    unpack8f(rw, r8);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf(r8[j] + v[j]);
    if (active) *(u32x4*)(a.h + (long)m * d + 8 * c) = pack8f(v);   // next launch reads it
    fm_rms8(v, active, d, w_pre, a.eps, red + 32);
    if (active) {
        const __amdgpu_buffer_rsrc_t xr = raw_rsrc(a.xn, (uint32_t)(a.M * d * 2));
        __builtin_amdgcn_raw_buffer_store_b128(pack8f(v), xr, (m * d + 8 * c) * 2, 0, AUX_SC1);
    }
}

// One register-resident-X GEMV stage (gemv_rx_kernel's arithmetic): the workgroup's nu
// units g = g0 + i * gs of W (KB k-steps of which [kb_lo, kb_lo + KBs) are summed), X rows from
// `X` (handed off in this launch: sc1 loads), partial sums to LDS `red`, then the
// epilogue. `wait` runs in wave 0 BEFORE its weight requests (the poll must not queue
// behind them); the other waves request their weights first.
template <int MT, int EPI, int SPU, int UMAX, typename Wait, typename Ts>
__device__ __forceinline__ bool fm_gemv(const bf16_t* W, int NG, int KB, int kb_lo, int KBs, int g0, int gs, int nu,
                                        const bf16_t* X, int ldx, int xbytes, int M, void* Y, int ldy, int ybytes,
                                        int N, f32x4* red, Wait wait, Ts ts, int ts0) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int xr = lane & 15;
    const __amdgpu_buffer_rsrc_t wr = frag_rsrc(W, (uint32_t)NG * (uint32_t)KB * 1024u);
    auto wbatch = [&](int i, bf16x8_s(&w)[SPU]) __attribute__((always_inline)) {
        const int g = g0 + i * gs;
#pragma unroll
        for (int j = 0; j < SPU; ++j) {
            const int kb = wave + j * FM_NW;
            const int off = (i < nu && kb < KBs) ? ((g * KB + kb_lo + kb) * 64 + lane) * 16 : (int)0xfffffff0u;
            w[j] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, AUX_NT));
        }
    };
    bool ok = true;
    if (wave == 0) ok = wait();
    ts(ts0);
    bf16x8_s wa[SPU], wb[SPU];
    bf16x8_s wall[UMAX > 0 ? UMAX : 1][SPU];
    if constexpr (UMAX > 0) {
#pragma unroll
        for (int i = 0; i < UMAX; ++i) wbatch(i, wall[i]);
    } else {
        wbatch(0, wa);
    }
    wg_barrier();   // the hand-off is complete (or abandoned) for every wave past here
    // this wave's X fragments: sc1 loads of bytes other workgroups stored sc1
    const __amdgpu_buffer_rsrc_t xrs = raw_rsrc(X, (uint32_t)xbytes);
    bf16x8_s xf[MT][SPU];
    const bf16x8_s z8 = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < MT; ++t) {
        const int row = 16 * t + xr;
        const int xo = (min(row, M - 1) * ldx + kb_lo * 32 + 8 * (lane >> 4)) * 2;
#pragma unroll
        for (int j = 0; j < SPU; ++j) {
            const int kb = min(wave + j * FM_NW, KBs - 1);
            const bf16x8_s v =
                __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo + kb * 64, 0, AUX_SC1));
            xf[t][j] = (row < M && wave + j * FM_NW < KBs) ? v : z8;
        }
    }
    auto mul = [&](int i, bf16x8_s(&w)[SPU]) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < SPU; ++j) acc = mfma16(w[j], xf[t][j], acc);
            if (i < nu) red[((i * MT + t) * FM_NW + wave) * 64 + lane] = acc;
        }
    };
    if constexpr (UMAX > 0) {
#pragma unroll
        for (int i = 0; i < UMAX; ++i) mul(i, wall[i]);
    } else {
        for (int i = 0; i < nu; i += 2) {
            wbatch(i + 1, wb);
            mul(i, wa);
            wbatch(i + 2, wa);
            mul(i + 1, wb);
        }
    }
    __syncthreads();
    ts(ts0 + 1);

    constexpr bool GLU = EPI == EPI_GEGLU;
    const int n_out = GLU ? N / 2 : N;
    const __amdgpu_buffer_rsrc_t yr = raw_rsrc(Y, (uint32_t)ybytes);
    if (!(GLU && lane >= 32)) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const int m = 16 * t + xr;
            if (m >= M) continue;
            for (int i = wave; i < nu; i += FM_NW) {
                const f32x4* ri = red + (size_t)(i * MT + t) * FM_NW * 64 + lane;
                const int n0 = (g0 + i * gs) * (GLU ? 8 : 16) + 4 * (lane >> 4);
                if constexpr (GLU) {
                    f32x4 gs = {0.f, 0.f, 0.f, 0.f}, us = gs;
#pragma unroll
                    for (int s2 = 0; s2 < FM_NW; ++s2) {
                        gs += ri[s2 * 64];
                        us += ri[s2 * 64 + 32];
                    }
                    float v[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = rbf(gelu_tanh(rbf(gs[r]))) * rbf(us[r]);
                    // act is handed to other workgroups: one 8-byte write-through store
                    // (n_out is a multiple of 8 here: fused_mlp checks f % 64)
                    const uint2 o2 = {pack2(v[0], v[1]), pack2(v[2], v[3])};
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, o2), yr, (m * ldy + n0) * 2, 0,
                                                          AUX_SC1);
                } else {
                    f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int s2 = 0; s2 < FM_NW; ++s2) s4 += ri[s2 * 64];
                    float* y = (float*)Y + (long)m * ldy;   // slabs: read by the next launch
                    if (n0 + 3 < n_out) *(f32x4*)(y + n0) = s4;
                    else
                        for (int r = 0; r < 4; ++r)
                            if (n0 + r < n_out) y[n0 + r] = s4[r];
                }
            }
        }
    }
    return ok;
}

template <int MT>
__global__ __launch_bounds__(FM_NW * 64) void fused_mlp_kernel(FusedMlpArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f32x4* red = (f32x4*)smem;                             // GEMV partial sums
    float* nred = (float*)smem;                            // norm stage: 2 x 32 floats (before the GEMVs)
    unsigned* tmo = a.timeout;
    const int bu = (int)blockIdx.x, nb = (int)gridDim.x;
    const int d = a.d, f = a.f;
    auto ts = [&](int k) __attribute__((always_inline)) { T5G_TS(k); };
    (void)ts;
    T5G_TS(0);
    // the next launch's counters: their last user (the previous step's launch of that
    // layer) has completed, their next user starts after this launch
    if (bu == 0 && threadIdx.x < FM_SET_LINES)
        __hip_atomic_store(a.sync_next + threadIdx.x * FM_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // ---- stage N: the norm workgroups publish xn rows
    const int nrow = bu - a.norm_b0;
    if (nrow >= 0 && nrow < a.M) {
        fm_norm_row(a, nrow, nred);
        drain_vm();            // every storing wave (R1)
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(a.sync + FS_NORM, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        T5G_TS(1);
    }

    // ---- stage G: a contiguous run of gate/up units (8 act features each). The norm
    // workgroups (the last M) start streaming ~5 us late and take FM_NORM_UNITS units;
    // the others share the rest, the first `uextra` of them one unit more. A run meets at
    // most two down slices.
    const int KBg = d / 32, NGg = a.NGgu;
    const unsigned Mu = (unsigned)a.M;
    constexpr int SPUg = 72 / FM_NW;
    const int nr = nb - a.M, rest = NGg - a.M * FM_NORM_UNITS;
    const int ubase = rest / nr, uextra = rest - ubase * nr;
    const int nu_g = bu < nr ? ubase + (bu < uextra ? 1 : 0) : FM_NORM_UNITS;
    const int g_lo = bu < nr ? bu * ubase + min(bu, uextra) : rest + (bu - nr) * FM_NORM_UNITS;
    bool ok = fm_gemv<MT, EPI_GEGLU, SPUg, MT == 1 ? 5 : 0>(
        a.Wgu, NGg, KBg, 0, KBg, g_lo, 1, nu_g, a.xn, d, a.M * d * 2, a.M, a.act, f, a.M * f * 2, 2 * f, red,
        [&]() { return fm_wait_n<1>(a.sync, L_N2, Mu, tmo, 1u); }, ts, 2);
    drain_vm();                // act stores of every wave (R1)
    __syncthreads();
    const int units_per_slice = f / FM_DS / 8;   // gate/up units (8 act features each) per down k-slice
    if (threadIdx.x == 0 && nu_g > 0) {   // one arrival per slice the run meets, counting its units
        const int s0 = g_lo / units_per_slice, s1 = (g_lo + nu_g - 1) / units_per_slice;
        for (int sl = s0; sl <= s1; ++sl) {
            const int n = min(g_lo + nu_g, (sl + 1) * units_per_slice) - max(g_lo, sl * units_per_slice);
            __hip_atomic_fetch_add(a.sync + fs_slice(sl), (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // ---- stage D: down slice s = bu / dg, units j, j + dg, ... (workgroups past 8 * dg idle)
    const int dg = nb / FM_DS;
    const int s = bu / dg, j = bu - s * dg;
    if (s < FM_DS) {
        const int KBd = f / 32, per = KBd / FM_DS;
        constexpr int SPUd = 36 / FM_NW;
        ok &= fm_gemv<MT, EPI_F32, SPUd, 5>(
            a.Wd, a.NGd, KBd, s * per, per, j, dg, (a.NGd - j + dg - 1) / dg, a.act, f, a.M * f * 2, a.M, a.part_out + (long)s * a.M * d, d,
            0, d, red, [&]() { return fm_wait_n<1>(a.sync, L_SL0 + s, (unsigned)units_per_slice, tmo, 2u + s); }, ts,
            4);
    }
    (void)ok;

    T5G_TS(6);
}

// ===========================================================================
// fused_block_kernel: the cross-attention chain in front of the MLP half (xattn = 1).
//
//   N1 (M norm workgroups)   h1 = h + RMSNorm_post1(o-proj slabs) (kept in registers),
//                            xn1 = RMSNorm_pre1(h1)                       -> L_N1
//   Q  (every workgroup)     one cross-q unit-slice: 16 q columns x 36 k-steps -> L_Q[head]
//   A  (8M workgroups)       PMCrossAttention of (row, q head): q from the 2 slabs, PM-RoPE,
//                            scores / aten softmax / P.V over <= 64 text keys -> L_A[head]
//   O  (every workgroup)     cross-o unit-slices (4 k-slices of 16 k-steps)     -> L_O[wg % 8]
//   N2 (norm workgroups)     h = h1 + RMSNorm_post2(cross-o slabs), xn = RMSNorm_pre2(h) -> L_N2
//   G, D                     as fused_mlp_kernel
//
// replacing resid_norm + cross-q (register-X GEMV, 12 waves, 2 k-slices) + cross attention
// (attn_decode_kernel<256, 1, true>) + cross-o (register-X GEMV, 8 waves, 4 k-slices) in
// front of the three MLP-half launches, with the same arithmetic in every stage (bitwise
// equal to the seven launches: tests/test_gpu_fused.py). Every wave requests the weights
// of a stage as early as its registers allow: Q's before N1 completes, O's during the
// attention, gate/up's right after O (norm workgroups: after N2), down's after gate/up;
// the cross K / V of the attention workgroups and their RoPE table at launch start.
// Round 5 adds the layer's decode self attention as stage S (fb_self_attn, the flash launch's
// arithmetic): fused_block_kernel<1> runs it in front of O1; fused_block_kernel<2> runs the
// NEXT layer's at the end, after the q|k|v stage (its K / V requested before the N3 wait),
// followed by that layer's O1 into the slabs the next launch's N1 reads
// (tests/test_gpu_attn_in_block.py: bitwise equal to the separate flash launch).

// Split form of fm_gemv: the weight requests (waves < NWG) ...
template <int NWG, int SPU, int UMAX>
__device__ __forceinline__ void fb_issue(bf16x8_s (&w)[UMAX][SPU], const bf16_t* W, int NG, int KB, int kb_lo, int KBs,
                                         int g0, int gs, int nu) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave >= NWG) return;
    const __amdgpu_buffer_rsrc_t wr = frag_rsrc(W, (uint32_t)NG * (uint32_t)KB * 1024u);
#pragma unroll
    for (int i = 0; i < UMAX; ++i) {
        const int g = g0 + i * gs;
#pragma unroll
        for (int j = 0; j < SPU; ++j) {
            const int kb = wave + j * NWG;
            const int off = (i < nu && kb < KBs) ? ((g * KB + kb_lo + kb) * 64 + lane) * 16 : (int)0xfffffff0u;
            w[i][j] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, AUX_NT));
        }
    }
}
// ... and the rest: rendezvous, X fragments (sc1), MFMAs, fixed-order wave reduction,
// epilogue. OUT: 0 = GeGLU bf16 (sc1, 8 B), 1 = fp32 plain, 2 = fp32 sc1 (16 B).
// LDSU: units i < nu_reg come from w, unit nu_reg (if < nu) from the LDS image lw (k-steps
// 0 .. NWG * SPU - 1 of one unit, 1 KiB each, fragment layout) -- the same MFMAs in the
// same order as from registers.
template <int NWG, int EPI, int SPU, int UMAX, int OUT, bool LDSU = false>
__device__ __forceinline__ void fb_finish(bf16x8_s (&w)[UMAX][SPU], int g0, int gs, int nu, int kb_lo, int KBs,
                                          const bf16_t* X, int ldx, int xbytes, int M, void* Y, int ldy, int ybytes,
                                          int N, f32x4* red, const char* lw = nullptr, int nu_reg = 0) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int xr = lane & 15;
    wg_barrier();   // the hand-off is complete (or abandoned) for every wave past here
    if (wave < NWG) {
        const __amdgpu_buffer_rsrc_t xrs = raw_rsrc(X, (uint32_t)xbytes);
        bf16x8_s xf[SPU];
        const bf16x8_s z8 = {0, 0, 0, 0, 0, 0, 0, 0};
        const int xo = (min(xr, M - 1) * ldx + kb_lo * 32 + 8 * (lane >> 4)) * 2;
#pragma unroll
        for (int j = 0; j < SPU; ++j) {
            const int kb = min(wave + j * NWG, KBs - 1);
            const bf16x8_s v =
                __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(xrs, xo + kb * 64, 0, AUX_SC1));
            xf[j] = (xr < M && wave + j * NWG < KBs) ? v : z8;
        }
        const int nr = LDSU ? nu_reg : nu;
#pragma unroll
        for (int i = 0; i < UMAX; ++i) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < SPU; ++j) acc = mfma16(w[i][j], xf[j], acc);
            if (i < nr) red[(i * NWG + wave) * 64 + lane] = acc;
        }
        if constexpr (LDSU) {
            if (nu_reg < nu) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < SPU; ++j)
                    acc = mfma16(*(const bf16x8_s*)(lw + ((wave + j * NWG) * 64 + lane) * 16), xf[j], acc);
                red[(nu_reg * NWG + wave) * 64 + lane] = acc;
            }
        }
    }
    __syncthreads();
    constexpr bool GLU = EPI == EPI_GEGLU;
    const int n_out = GLU ? N / 2 : N;
    const int m = xr;
    if (wave >= NWG || m >= M || (GLU && lane >= 32)) return;
    const __amdgpu_buffer_rsrc_t yr = raw_rsrc(Y, (uint32_t)ybytes);
    for (int i = wave; i < nu; i += NWG) {
        const f32x4* ri = red + (size_t)i * NWG * 64 + lane;
        const int n0 = (g0 + i * gs) * (GLU ? 8 : 16) + 4 * (lane >> 4);
        if constexpr (GLU) {
            f32x4 gsum = {0.f, 0.f, 0.f, 0.f}, usum = gsum;
#pragma unroll
            for (int s2 = 0; s2 < NWG; ++s2) {
                gsum += ri[s2 * 64];
                usum += ri[s2 * 64 + 32];
            }
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = rbf(gelu_tanh(rbf(gsum[r]))) * rbf(usum[r]);
            const uint2 o2 = {pack2(v[0], v[1]), pack2(v[2], v[3])};
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, o2), yr, (m * ldy + n0) * 2, 0, AUX_SC1);
        } else {
            f32x4 s4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s2 = 0; s2 < NWG; ++s2) s4 += ri[s2 * 64];
            if constexpr (OUT == 2) {
                // n_out is a multiple of 16 here (the q / cross-o widths)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, s4), yr, (m * ldy + n0) * 4, 0,
                                                       AUX_SC1);
            } else {
                float* y = (float*)Y + (long)m * ldy;   // slabs read by the next launch
                if (n0 + 3 < n_out) *(f32x4*)(y + n0) = s4;
                else
                    for (int r = 0; r < 4; ++r)
                        if (n0 + r < n_out) y[n0 + r] = s4[r];
            }
        }
    }
}

// resid_norm_kernel<4, 2>'s arithmetic for row m: v = bf16(sum of the 4 slabs),
// post-norm, h = bf16(r + v) (r8: the residual in, the new residual out, in registers),
// xn = pre-norm(h) stored write-through. Slabs read plain (previous launch) or sc1.
template <int NS, bool SC1>
__device__ __forceinline__ void fb_norm(const float* part, int M, int m, int d, const bf16_t* post_w,
                                        const bf16_t* pre_w, float eps, float (&r8)[8], bf16_t* xn, float* red) {
    const int c = threadIdx.x;
    const bool active = 8 * c < d;
    const int cc = active ? c : d / 8 - 1;
    const u32x4 w_post = *(const u32x4*)(post_w + 8 * cc);
    const u32x4 w_pre = *(const u32x4*)(pre_w + 8 * cc);
    f32x4 p[NS][2];
    const __amdgpu_buffer_rsrc_t pr = raw_rsrc(part, (uint32_t)(NS * M * d * 4));
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int o = ((s * M + m) * d + 8 * cc) * 4;
        if constexpr (SC1) {
            p[s][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, o, 0, AUX_SC1));
            p[s][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, o + 16, 0, AUX_SC1));
        } else {
            const f32x4* ps = (const f32x4*)(part + ((long)s * M + m) * d + 8 * cc);
            p[s][0] = ps[0];
            p[s][1] = ps[1];
        }
    }
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[j] += p[s][0][j];
            v[4 + j] += p[s][1][j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf(v[j]);
    fm_rms8(v, active, d, w_post, eps, red);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf(r8[j] + v[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) r8[j] = v[j];
    fm_rms8(v, active, d, w_pre, eps, red + 32);
    if (active) {
        const __amdgpu_buffer_rsrc_t xr = raw_rsrc(xn, (uint32_t)(M * d * 2));
        __builtin_amdgcn_raw_buffer_store_b128(pack8f(v), xr, (m * d + 8 * c) * 2, 0, AUX_SC1);
    }
}

// every storing wave drains, the workgroup meets, one lane adds `n` to `ctr`
__device__ __forceinline__ void fb_publish(unsigned* ctr, unsigned n) {
    drain_vm();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(ctr, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS of the attention stage (after the GEMV partial sums)
struct FbAttnLds {
    f32x4 ored[4][32][2];
    float sm[64];
    float pl[64 + 16];
    float qs[256];
    float stat_l;
};
constexpr int FB_D = 2304;                                    // the block kernel's model width
constexpr int FB_GU_KB = FB_D / 32;                           // gate/up k-steps (= FM_NW x 6)
constexpr size_t FB_GU_OFF = (5 * FM_NW * 1024 + sizeof(FbAttnLds) + 16 + 64 * sizeof(float) + FB_D * 2 + 1023) / 1024 * 1024;
constexpr size_t FB_LDS = FB_GU_OFF + (size_t)FB_GU_KB * 1024;

// ---- stage S: the layer's decode self-attention (a.self_attn), attn.hip
// attn_decode_kernel<256, 2, true, true> + attn_flash_finish restated on this launch's 12
// waves as three 4-wave groups, each one 64-key chunk in that kernel's lane map: the same
// loads, q / new-key PM-RoPE, cache append, sums and roundings, so the launch stays bitwise
// equal to the flash launch + the per-op chain. Chunk slots (chunk-major: chunk x rows x kv
// heads) run on workgroup c % nwg, group c / nwg, so the K / V stream is spread over every CU. A chunk's partial goes out write-through with one ticket add per
// chunk; the workgroup holding the last chunk of a (row, kv head) combines them in the flash
// kernel's order (its whole workgroup, after every group's ticket) and publishes att_self on
// line L_S0 + kv head, which O1's k-slice of that head pair waits for. Rows of <= 64 keys take
// the kernel's one-block (aten-order) path in their group. Nothing in S waits, so every chunk
// finishes and every (row, kv head) publishes exactly once.
constexpr int FS_G = 2, FS_D = 256, FS_CH = 64, FS_LPK = FS_D / 8, FS_KPW = 64 / FS_LPK, FS_KPB = FS_KPW * 4,
              FS_NIT = FS_CH / FS_KPB, FS_GRP = FM_NW / 4, FS_MAXROWS = 32,
              FS_MAXPASS = 2;   // front: passes of 3 chunk slots per workgroup (8 rows: <= 48 chunks)
static_assert(FS_LPK == 32, "the P.V lanes of a key fold in one xor-32 step");
struct FbSelfGrp {
    f32x4 ored[4][FS_G][FS_LPK][2];
    float sm[FS_G][FS_CH];
    float pl[FS_G][FS_CH + 16];
    float qs[FS_G][FS_D];
    float kvnew[2][FS_D];
    float stat_l[FS_G];
    float cstat[FS_G][2];
    float wts[FS_G][DEC_MAX_CHUNKS];   // the combine's chunk weights and sums
    float lsum[FS_G];
    int last;
};
struct FbSelfLds {
    FbSelfGrp g[FS_GRP];
};
static_assert(sizeof(FbSelfLds) <= 5 * FM_NW * 1024, "stage S lives in the GEMV partial-sum LDS");

// diagnostic timeline of stage S and O1 (T5G_DBG_TS library variant only,
// tools/diag_fused_s.py): thread 0 (or `tid`) of every workgroup stores the 100 MHz clock at
// numbered points, 32 slots per workgroup
#ifdef T5G_DBG_TS
__device__ unsigned long long* fs_ts_buf;
extern "C" int t5g_dbg_set_fused_s(void* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(fs_ts_buf), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
// timing variants of stage S (never in the product): 1 no K / V loads, 2 one q|k|v slab
// address for every lane, 3 every (row, kv head) reads row 0 / kv head 0's cache (L2 hits),
// 4 the stage run twice (the second one warm: instruction cache, TLB, L2), 5 no K / V load
// instructions at all
__device__ int fs_dbg_var;
extern "C" int t5g_dbg_set_fused_s_var(int v) {
    return hipMemcpyToSymbol(HIP_SYMBOL(fs_dbg_var), &v, sizeof(v)) == hipSuccess ? 0 : -1;
}
#define FS_DBG_VAR fs_dbg_var
#define FS_TS_BY(k, tid)                                                                           \
    do {                                                                                           \
        if (threadIdx.x == (tid) && fs_ts_buf) fs_ts_buf[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define FS_DBG_VAR 0
#define FS_TS_BY(k, tid) do { } while (0)
#endif
#define FS_TS(k) FS_TS_BY(k, 0)

// barrier that waits for this wave's LDS traffic only (no vmcnt: loads stay in flight)
__device__ __forceinline__ void fb_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// TAIL (a.self_tail): the stage runs at the END of the previous layer's launch for this
// layer -- the K / V requests go out before `mid` (the N3 wait, the q|k|v stage and its
// hand-off, run by the caller), the q|k|v slabs are read (sc1) after it; slots live on the
// first `nwg` workgroups' groups 0-1 only (group 2's waves poll), and `len_in` is the row
// length the caller requested at launch start. Front: `mid` is empty, len_in < 0.
template <bool TAIL, typename Mid>
__device__ __forceinline__ void fb_self_attn(const FusedMlpArgs& a, FbSelfLds& sl, Mid&& mid, int nwg, int len_in,
                                             int pass = 0) {
    constexpr int G = FS_G, D = FS_D, LPK = FS_LPK, KPW = FS_KPW, KPB = FS_KPB, NIT = FS_NIT;
    const int tq = (int)threadIdx.x, wave = tq >> 6, lane = tq & 63;
    const int grp = wave >> 2, gw = wave & 3, gt = tq & 255;
    const int kg = lane / LPK, dl = lane % LPK;
    const int M = a.M, Hkv = a.Hkv;
    FbSelfGrp& L = sl.g[grp];
    // this group's chunk slot (row m, kv head, chunk sp): slot c = sp x (M Hkv) + row x Hkv +
    // kv head on workgroup c % nb, group c / nb -- known before the row lengths, so the q|k|v
    // slabs and the RoPE row are requested with the row length; chunk-major, so the live
    // chunks (sp < the row's count) fill group 0 of every workgroup before any group 1
    // (in front, a call with more slots than 3 nb runs several passes: slots 3 nb p ..)
    const int cidx = (int)blockIdx.x + (grp + FS_GRP * pass) * nwg;
    const bool has_s = (int)blockIdx.x < nwg && cidx < M * Hkv * a.s_nsplit;
    const int sp = has_s ? cidx / (M * Hkv) : 0, rk = has_s ? cidx - sp * (M * Hkv) : 0;
    const int m = rk / Hkv, kvh = rk - m * Hkv;
    const int dvar = FS_DBG_VAR;
    const int len = TAIL ? len_in : a.kv_len[m];
    int role = 0, c4 = 0, g_own = 0, col;
    if (gt < G * D / 4) {
        g_own = gt / (D / 4);
        c4 = gt % (D / 4);
        col = (kvh * G + g_own) * D + 4 * c4;
    } else {   // the appended key / value (used by the slot holding key t)
        const int idx = gt - G * D / 4;
        role = 1 + idx / (D / 4);   // 1: key, 2: value
        c4 = idx % (D / 4);
        col = (role == 1 ? a.q_dim : a.q_dim + Hkv * D) + kvh * D + 4 * c4;
    }
    const long uo = dvar == 2 ? 0 : col;
    // unconditional (slots past the grid read row 0's): a load under a branch makes the
    // compiler wait for everything in flight at the join, the row length included. In the
    // tail the slabs are this launch's (after `mid`).
    f32x4 u0, u1;
    if constexpr (!TAIL) {
        u0 = *(const f32x4*)(a.qkv_in + (long)m * a.qkv_dim + uo);
        u1 = *(const f32x4*)(a.qkv_in + ((long)M + m) * a.qkv_dim + uo);
    }
    const float* tr = a.rope_tab + (long)m * D + (8 * dl) % (D / 2);
    f32x4 ca = *(const f32x4*)tr, cb = *(const f32x4*)(tr + 4);
    f32x4 sa = *(const f32x4*)(tr + D / 2), sb = *(const f32x4*)(tr + D / 2 + 4);
    // row geometry (attn_decode_kernel's rules: causal, the sliding window); a row of <= 64
    // keys is one chunk (the one-block path; a row with no key still publishes)
    const int t = len - 1;
    const int hi = min(t + 1, len), lo = a.window > 0 ? max(0, t - a.window + 1) : 0;
    const int span = max(hi - lo, 0);
    const bool single = span <= FS_CH;
    const int nch = single ? 1 : (span + FS_CH - 1) / FS_CH;
    const bool has_c = has_s && sp < nch;
    if (has_s && sp == 0 && gt == 0 && nch > a.s_nsplit)   // past the host's key bound: give every wait up
        __hip_atomic_store(a.timeout, 18u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int c0 = lo + sp * FS_CH, c1 = min(hi, c0 + FS_CH), n = c1 - c0;
    const bool gv = has_c && n > 0;
    const bool has_t = gv && t >= c0 && t < c1;
    if (!TAIL && gt == 0) L.last = 0;
    const __amdgpu_buffer_rsrc_t ors = raw_rsrc(a.att_self, (uint32_t)(M * a.q_dim * 2));
    const long nrec = (long)M * Hkv * a.s_nsplit;
    const __amdgpu_buffer_rsrc_t prs = frag_rsrc(a.fpart, (uint32_t)(nrec * G * D * 4));
    const __amdgpu_buffer_rsrc_t srs = frag_rsrc(a.fstat, (uint32_t)(nrec * G * 2 * 4));
    const long hs = (long)a.s_cap * D, bs = hs * Hkv;
    bf16_t* Kb = a.sk + (dvar == 3 ? 0 : m * bs + kvh * hs);
    bf16_t* Vb = a.sv + (dvar == 3 ? 0 : m * bs + kvh * hs);
    float c8[8], s8[8];
    const __amdgpu_buffer_rsrc_t krs = frag_rsrc(Kb, (uint32_t)a.s_cap * D * 2u);
    const __amdgpu_buffer_rsrc_t vrs = frag_rsrc(Vb, (uint32_t)a.s_cap * D * 2u);
    // groups without a chunk request nothing (a wave-uniform branch): their loads would queue
    // in the CU's memory pipeline ahead of the working groups' data
    u32x4 kr[NIT], vr[NIT];
    if (gv && dvar != 5) {
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int j = c0 + i * KPB + gw * KPW + kg;
            const int off = (j < c1 && dvar != 1) ? (j * D + 8 * dl) * 2 : (int)0x7ffffff0;
            kr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
            vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0));
        }
        // q (and the appended key / value) staged in the same block as the K / V requests, so
        // the wait for the slabs counts exactly the requests behind them
        if constexpr (!TAIL) {
            f32x4 acc = u0;
            acc += u1;
            if (role == 0) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) L.qs[g_own][4 * c4 + jj] = rbf(acc[jj]);
            } else if (has_t) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) L.kvnew[role - 1][4 * c4 + jj] = rbf(acc[jj]);
            }
        }
        // the RoPE row consumed here too (an empty asm use): past the branch join the compiler
        // would otherwise wait for nearly every K / V request before the q rotation
        asm volatile("" : "+v"(ca), "+v"(cb), "+v"(sa), "+v"(sb));
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            c8[jj] = ca[jj];
            c8[4 + jj] = cb[jj];
            s8[jj] = sa[jj];
            s8[4 + jj] = sb[jj];
        }
    } else {
#pragma unroll
        for (int i = 0; i < NIT; ++i) kr[i] = vr[i] = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) c8[jj] = s8[jj] = 0.f;
    }
    if constexpr (TAIL) {
        mid();   // N3, the q|k|v stage and its hand-off (workgroup-uniform, with barriers)
        const __amdgpu_buffer_rsrc_t qrs = raw_rsrc(a.qkv_in, (uint32_t)(2 * M * a.qkv_dim * 4));
        u0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qrs, (int)((m * a.qkv_dim + uo) * 4), 0, AUX_SC1));
        u1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(qrs, (int)(((M + m) * a.qkv_dim + uo) * 4), 0,
                                                                              AUX_SC1));
        if (gt == 0) L.last = 0;
        if (gv) {
            f32x4 acc = u0;
            acc += u1;
            if (role == 0) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) L.qs[g_own][4 * c4 + jj] = rbf(acc[jj]);
            } else if (has_t) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) L.kvnew[role - 1][4 * c4 + jj] = rbf(acc[jj]);
            }
        }
    }
    fb_lds_barrier();
    FS_TS(2);
    // groups without a chunk skip the arithmetic too (wave-uniform): their waves would take
    // VALU issue slots from the working groups on the same SIMDs
    if (gv) {
        float q[G][8];
        {
            const float sg = dl < LPK / 2 ? -1.0f : 1.0f;
            const int pbase = (8 * dl + D / 2) % D;
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int jj = 0; jj < 8; ++jj) {
                    const float x = L.qs[g][8 * dl + jj];
                    const float pr = L.qs[g][pbase + jj];
                    q[g][jj] = rbf(rbf(x * c8[jj]) + rbf((sg * pr) * s8[jj]));
                }
        }
        FS_TS(14);
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            // (keys past c1 were requested out of the descriptor's range: already zero)
            const int j = c0 + i * KPB + gw * KPW + kg;
            if (has_t && j == t) {
                // key t: PM-RoPE of the new key, then append it and its value
                const float sg = dl < LPK / 2 ? -1.0f : 1.0f;
                const int pbase = (8 * dl + D / 2) % D;
                u32x4 kw, vw;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    float ko[2], vo[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int dd = 8 * dl + 2 * jj + e;
                        const float c = c8[2 * jj + e], sn = s8[2 * jj + e];
                        const float x = L.kvnew[0][dd], pr = L.kvnew[0][pbase + 2 * jj + e];
                        ko[e] = rbf(rbf(x * c) + rbf((sg * pr) * sn));
                        vo[e] = L.kvnew[1][dd];
                    }
                    kw[jj] = pack2(ko[0], ko[1]);
                    vw[jj] = pack2(vo[0], vo[1]);
                }
                kr[i] = kw;
                vr[i] = vw;
                *(u32x4*)(Kb + (long)t * D + 8 * dl) = kw;
                *(u32x4*)(Vb + (long)t * D + 8 * dl) = vw;
            }
        }
        // the scores stay in registers until every key's reduction is done (no store between
        // them), so the 16 butterfly reductions of a wave overlap instead of running one by one
        // the two q heads side by side in packed fp32 (v_pk_mul / v_pk_add: the same IEEE
        // operations per head, half the instructions)
        static_assert(G == 2, "packed head pair");
        f32x2 qq[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) qq[jj] = (f32x2){q[0][jj], q[1][jj]};
        float sc[NIT][G];
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            f32x2 s2 = {0.f, 0.f};
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const float k0 = bf_lo(kr[i][jj]), k1 = bf_hi(kr[i][jj]);
                s2 += qq[2 * jj] * k0 + qq[2 * jj + 1] * k1;
            }
#pragma unroll
            for (int g = 0; g < G; ++g) sc[i][g] = xsum_v<LPK>(s2[g]);   // xsum<LPK>'s adds, VALU exchanges
        }
        FS_TS(16);
        if (dl == 0) {
#pragma unroll
            for (int i = 0; i < NIT; ++i)
#pragma unroll
                for (int g = 0; g < G; ++g) L.sm[g][i * KPB + gw * KPW + kg] = fast_score(sc[i][g], a.scale, a.softcap);
        }
    }
    fb_lds_barrier();
    FS_TS(3);
    // softmax of the chunk: one aten block (one-block row) or the flash chunk statistics
    if (gv && gw < G) {
        const int g = gw;
        const float s = lane < n ? L.sm[g][lane] : -INFINITY;
        const float mx = wave_max(s);
        if (single) {
            const float p = lane < n ? sdpa_p(__fsub_rn(s, mx), lane, span) : 0.f;
            L.pl[g][lane] = p;
            if (lane < 16) L.pl[g][FS_CH + lane] = 0.f;
            L.sm[g][lane] = rbf(p);
            __builtin_amdgcn_wave_barrier();
            const float l = sdpa_block_sum_lds<FS_CH>(L.pl[g], span, lane);
            if (lane == 0) L.stat_l[g] = l;
        } else {
            const float p = lane < n ? __expf(s - mx) : 0.f;
            L.sm[g][lane] = rbf(p);
            const float l = xsum<64>(p);
            if (lane == 0) {
                L.cstat[g][0] = mx;
                L.cstat[g][1] = l;
            }
        }
    }
    fb_lds_barrier();
    if (gv) {
        // both heads' accumulators packed (o2[d] = {head 0, head 1}): the same per-head chain
        f32x2 o2[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) o2[jj] = (f32x2){0.f, 0.f};
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int jl = i * KPB + gw * KPW + kg;
            const f32x2 pp = {L.sm[0][jl], L.sm[1][jl]};
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                o2[2 * jj] += pp * bf_lo(vr[i][jj]);
                o2[2 * jj + 1] += pp * bf_hi(vr[i][jj]);
            }
        }
        float o[G][8];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) o[g][jj] = o2[jj][g] + xlane32_v(o2[jj][g]);   // LPK = 32: one xor-32 step
        if (kg == 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                L.ored[gw][g][dl][0] = (f32x4){o[g][0], o[g][1], o[g][2], o[g][3]};
                L.ored[gw][g][dl][1] = (f32x4){o[g][4], o[g][5], o[g][6], o[g][7]};
            }
        }
    }
    fb_lds_barrier();
    FS_TS(4);
    if (gv && gt < G * LPK) {
        const int g = gt / LPK, d8 = gt % LPK;
        const f32x4 lo4 = L.ored[0][g][d8][0] + L.ored[1][g][d8][0] + L.ored[2][g][d8][0] + L.ored[3][g][d8][0];
        const f32x4 hi4 = L.ored[0][g][d8][1] + L.ored[1][g][d8][1] + L.ored[2][g][d8][1] + L.ored[3][g][d8][1];
        if (single) {   // the row's output
            const float inv = __fdiv_rn(1.0f, L.stat_l[g]);
            u32x4 w;
            w[0] = pack2(__fmul_rn(lo4[0], inv), __fmul_rn(lo4[1], inv));
            w[1] = pack2(__fmul_rn(lo4[2], inv), __fmul_rn(lo4[3], inv));
            w[2] = pack2(__fmul_rn(hi4[0], inv), __fmul_rn(hi4[1], inv));
            w[3] = pack2(__fmul_rn(hi4[2], inv), __fmul_rn(hi4[3], inv));
            __builtin_amdgcn_raw_buffer_store_b128(w, ors, (m * a.q_dim + (kvh * G + g) * D + 8 * d8) * 2, 0, AUX_SC1);
        } else {        // the chunk's partial
            const int off = (int)(((((long)m * Hkv + kvh) * a.s_nsplit + sp) * G + g) * D + 8 * d8) * 4;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo4), prs, off, 0, AUX_SC1);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi4), prs, off + 16, 0, AUX_SC1);
        }
    }
    if (gv && !single && gt < G) {
        const u32x2_t st = {__float_as_uint(L.cstat[gt][0]), __float_as_uint(L.cstat[gt][1])};
        __builtin_amdgcn_raw_buffer_store_b64(
            st, srs, (int)(((((long)m * Hkv + kvh) * a.s_nsplit + sp) * G + gt) * 2) * 4, 0, AUX_SC1);
    }
    drain_vm();
    fb_lds_barrier();
    FS_TS(5);
    unsigned* tk = a.fticket + (long)m * Hkv + kvh;
    if (has_c && !single && gt == 0)
        L.last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nch - 1);
    fb_lds_barrier();
    FS_TS(6);
    // the group holding the last chunk of its (row, kv head) combines the chunk records
    // (attn_flash_finish's combine on the group's 4 waves: waves 0..G-1 the chunk weights
    // exp(m_c - M) and the sum, waves G.. the output quads, their first batch of partials
    // requested before the weights are known); every group that completed a (row, kv head)
    // then publishes it. The groups of a workgroup combine side by side.
    const bool comb = has_c && !single && L.last != 0;
    const bool pub = has_c && (single || comb);
    {
        constexpr int FB = 16, NOUT = G * D / 4;   // attn_flash_finish's combine batch
        const long rec = ((long)m * Hkv + kvh) * a.s_nsplit;   // chunk records of this (row, kv head)
        const int ot = gt - 64 * G;
        const bool outer = comb && ot >= 0 && ot < NOUT;
        const int og = outer ? ot / (D / 4) : 0, o4 = outer ? ot % (D / 4) : 0;
        auto pload = [&](f32x4 (&pv)[FB], int cb) {
#pragma unroll
            for (int k = 0; k < FB; ++k) {
                int off = cb + k < nch ? (int)((((rec + cb + k) * G + og) * D + 4 * o4) * 4) : (int)0x7ffffff0;
                asm volatile("" : "+v"(off));
                pv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(prs, off, 0, AUX_SC1));
            }
        };
        if (comb && gt == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        f32x4 pv[FB];
        if (outer) pload(pv, 0);
        if (comb && gw < G) {
            constexpr int CPL = DEC_MAX_CHUNKS / 64;   // lane owns chunks lane + 64 i (attn_flash_finish)
            const int g = gw;
            float mc[CPL], lc[CPL];
#pragma unroll
            for (int i = 0; i < CPL; ++i) {
                const int c = lane + 64 * i;
                int off = c < nch ? (int)((((rec + c) * G + g) * 2) * 4) : (int)0x7ffffff0;
                asm volatile("" : "+v"(off));
                const u32x2_t st = __builtin_amdgcn_raw_buffer_load_b64(srs, off, 0, AUX_SC1);
                mc[i] = c < nch ? __uint_as_float(st[0]) : -INFINITY;
                lc[i] = c < nch ? __uint_as_float(st[1]) : 0.f;
            }
            float mm = mc[0];
#pragma unroll
            for (int i = 1; i < CPL; ++i) mm = fmaxf(mm, mc[i]);
            const float Mx = wave_max(mm);
            float wl = 0.f;
#pragma unroll
            for (int i = 0; i < CPL; ++i) {
                const float w = lane + 64 * i < nch ? __expf(mc[i] - Mx) : 0.f;
                L.wts[g][lane + 64 * i] = w;
                wl += w * lc[i];
            }
            const float Ls = xsum<64>(wl);
            if (lane == 0) L.lsum[g] = Ls;
        }
        fb_lds_barrier();
        if (outer) {   // attn_flash_finish's batches of 16 records, in order
            f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
            for (int cb = 0; cb < nch; cb += FB) {
                if (cb > 0) pload(pv, cb);
#pragma unroll
                for (int k = 0; k < FB; ++k) {
                    const float w = cb + k < nch ? L.wts[og][cb + k] : 0.f;
                    acc += w * pv[k];
                }
            }
            const float inv = 1.0f / L.lsum[og];
            const u32x2_t ow = {pack2(acc[0] * inv, acc[1] * inv), pack2(acc[2] * inv, acc[3] * inv)};
            __builtin_amdgcn_raw_buffer_store_b64(ow, ors, (m * a.q_dim + (kvh * G + og) * D + 4 * o4) * 2, 0,
                                                  AUX_SC1);
        }
    }
    drain_vm();
    fb_lds_barrier();
    if (pub && gt == 0) __hip_atomic_fetch_add(cline(a.sync, L_S0 + kvh), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    FS_TS(7);
}

// SM: the self-attention stage S -- 0 none, 1 in front of O1 (a.self_attn), 2 at the end for
// the next layer, followed by the next layer's O1 (a.self_tail; N1 then reads the previous
// launch's o-projection slabs). Separate instantiations, so a launch carries only its own
// stages' code and registers.
template <int SM>
__global__ __launch_bounds__(FM_NW * 64) void fused_block_kernel(FusedMlpArgs a) {
    constexpr bool SELF = SM == 1;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    f32x4* red = (f32x4*)smem;                                   // GEMV partial sums, <= 60 KB
    FbAttnLds& al = *(FbAttnLds*)(smem + 5 * FM_NW * 1024);      // attention scratch
    float* nred = (float*)(smem + 5 * FM_NW * 1024 + sizeof(FbAttnLds) + 16);   // norm: 2 x 32 floats
    // a norm workgroup's residual row between N1, N2 and N3 (bf16, exact: every h is rounded)
    u32x4* hrow = (u32x4*)(smem + 5 * FM_NW * 1024 + sizeof(FbAttnLds) + 16 + 64 * sizeof(float));
    // a worker's last gate/up unit (72 KiB), fetched by LDS-DMA while the chain runs O1 -> O
    char* gul = smem + FB_GU_OFF;
    unsigned* tmo = a.timeout;
    const int bu = (int)blockIdx.x, nb = (int)gridDim.x;
    const int tq = (int)threadIdx.x, wave = tq >> 6, lane = tq & 63;
    const int d = a.d, f = a.f, M = a.M, D = 256;
    T5G_TS(0);
    if (bu == 0 && tq < FM_SET_LINES)
        __hip_atomic_store(a.sync_next + tq * FM_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int nrow = bu - a.norm_b0;
    const bool normwg = nrow >= 0 && nrow < M;
    const bool attnwg = bu < M * a.Hq;
    const int am = bu / a.Hq, ah = bu - am * a.Hq;   // attention task (row, q head)
    bool ok = true;
    // ---- S: the layer's self-attention on every workgroup (O1 waits for its heads)
    if constexpr (SELF) {
        FS_TS(0);
        // a call with more chunk slots than 3 per workgroup: a second pass of 3 nb slots
        // (uniform; two inlined copies -- a loop keeps the stage's registers live across it)
        fb_self_attn<false>(a, *(FbSelfLds*)smem, [] {}, nb, -1, 0);
        if (M * a.Hkv * a.s_nsplit > FS_GRP * nb) fb_self_attn<false>(a, *(FbSelfLds*)smem, [] {}, nb, -1, 1);
        if (FS_DBG_VAR == 4) {   // timing variant: the stage again, warm (points overwritten)
            FS_TS(13);
            fb_self_attn<false>(a, *(FbSelfLds*)smem, [] {}, nb, -1);
        }
        FS_TS(8);
    }
    // the tail's row length, requested first (the oldest load: waiting for it later waits for
    // nothing else); the same slot map as fb_self_attn<true> over the nb - M workers
    int len_tail = 0;
    if constexpr (SM == 2) {
        if (a.Wqkv) FS_TS(0);   // (the last layer's launch has no tail: its start would overwrite)
        const int nwk = nb - M, cidx = bu + (wave >> 2) * nwk;
        const int rk = cidx % (M * a.Hkv);
        len_tail = a.kv_len[bu < nwk ? rk / a.Hkv : 0];
    }

    // ---- the attention workers request their row's cross K / V chunk and RoPE row
    // (attn_decode_kernel<256, 1, true>'s VFIRST loads, waves 0-3) right after O1
    constexpr int LPK = 32, KPW = 2, KPB = 8, NIT = 8;
    const int kg = lane / LPK, dl = lane % LPK;
    u32x4 kr[NIT], vr[NIT];
    float c8[8], s8[8];
    int alen = 0;
    auto kv_prefetch = [&]() __attribute__((always_inline)) {
    if (attnwg && wave < 4) {
        alen = a.enc_len[am];
        const int kvc = ah / (a.Hq / a.Hkv);
        const long hs = (long)a.kv_cap * D, bs = hs * a.Hkv;
        const __amdgpu_buffer_rsrc_t krs = frag_rsrc(a.ck + am * bs + kvc * hs, (uint32_t)a.kv_cap * D * 2u);
        const __amdgpu_buffer_rsrc_t vrs = frag_rsrc(a.cv + am * bs + kvc * hs, (uint32_t)a.kv_cap * D * 2u);
#pragma unroll
        for (int i = 0; i < NIT; ++i) {
            const int j = i * KPB + wave * KPW + kg;
            const int off = j < alen ? (j * D + 8 * dl) * 2 : (int)0x7ffffff0;
            kr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
            vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, off, 0, 0));
        }
        const float* tr = a.rope_tab + (long)am * D + (8 * dl) % (D / 2);
        const f32x4 ca = *(const f32x4*)tr, cb = *(const f32x4*)(tr + 4);
        const f32x4 sa = *(const f32x4*)(tr + D / 2), sb = *(const f32x4*)(tr + D / 2 + 4);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            c8[jj] = ca[jj];
            c8[4 + jj] = cb[jj];
            s8[jj] = sa[jj];
            s8[4 + jj] = sb[jj];
        }
    }
    };

    // ---- the norm workgroups (the last M): N1, N2, N3 for their row and nothing else, so no
    // weight stream of their own ever queues ahead of a norm on the critical path
    const int nw = nb - M;   // GEMV / attention workers
    if (normwg) {
        {
            float hreg[8];
            const int cc = min(tq, d / 8 - 1);
            unpack8f(*(const u32x4*)(a.h + (long)nrow * d + 8 * cc), hreg);
            if (a.Wo1) {   // the o-projection slabs come from this launch's O1 stage
                if (wave == 0) ok &= fm_wait_split<8>(a.sync, L_P0, (unsigned)(4 * (nw / 4)), tmo, 16u);
                wg_barrier();
                fb_norm<FM_NS, true>(a.o1slab, M, nrow, d, a.post1_w, a.pre1_w, a.eps, hreg, a.xn1, nred);
            } else {
                fb_norm<FM_NS, false>(a.o_slabs, M, nrow, d, a.post1_w, a.pre1_w, a.eps, hreg, a.xn1, nred);
            }
            if (tq < d / 8) hrow[tq] = pack8f(hreg);
            fb_publish(cline(a.sync, L_N1), 1u);
            if constexpr (SELF) FS_TS(12);
        }
        {
            if (wave == 0) ok &= fm_wait_split<8>(a.sync, L_O0, (unsigned)(4 * (nw / 4)), tmo, 4u);
            wg_barrier();
            float r2[8];
            unpack8f(hrow[min(tq, d / 8 - 1)], r2);
            fb_norm<FM_NS, true>(a.oslab, M, nrow, d, a.post_w, a.pre_w, a.eps, r2, a.xn, nred);
            if (tq < d / 8) hrow[tq] = pack8f(r2);
            fb_publish(cline(a.sync, L_N2), 1u);
        }
        {
            if (wave == 0) ok &= fm_wait_split<8>(a.sync, L_D0, (unsigned)(FM_DS * (nw / FM_DS)), tmo, 14u);
            wg_barrier();
            float r3[8];
            unpack8f(hrow[min(tq, d / 8 - 1)], r3);
            fb_norm<FM_DS, true>(a.dslab, M, nrow, d, a.post3_w, a.pre3_w, a.eps, r3, a.xn, nred);
            if (tq < d / 8) *(u32x4*)(a.h + (long)nrow * d + 8 * tq) = pack8f(r3);   // read by the next launch
            fb_publish(cline(a.sync, L_N3), 1u);
        }
        T5G_TS(6);
        return;
    }
    const int w = bu;   // worker index
    // gate/up: contiguous unit runs over the workers (<= 5 units, the last one from LDS)
    const int KBg = d / 32, NGg = a.NGgu;
    const int ubase = NGg / nw, uextra = NGg - ubase * nw;
    const int nu_g = ubase + (w < uextra ? 1 : 0);
    const int g_lo = w * ubase + min(w, uextra);
    const bool gu_lds = nu_g > 0 && !attnwg;
    const int oper = nw / 4, so = w / oper, jo = w - so * oper;   // o-projection mapping (O1 and O)
    const bool owork = so < 4;
    const int nu_o = owork ? (a.NGo - jo + oper - 1) / oper : 0;

    // ---- O1: the self-attention o-projection, 4 k-slices of 16 k-steps over nw / 4 workers
    // each (<= 3 units, 8 waves); its input is the previous launch's (no wait), or stage S's:
    // k-slice so is the q-head pair of kv head so, complete when its M rows have published
    if (a.Wo1 && owork) {
        bf16x8_s w1[3][2];
        fb_issue<8, 2, 3>(w1, a.Wo1, a.NGo, a.q_dim / 32, so * 16, 16, jo, oper, nu_o);
        if (SELF && wave == FM_NW - 1) ok &= fm_wait_n<1>(a.sync, L_S0 + so, (unsigned)M, tmo, 17u);
        if constexpr (SELF) FS_TS_BY(9, (FM_NW - 1) * 64);
        fb_finish<8, EPI_F32, 2, 3, 2>(w1, jo, oper, nu_o, so * 16, 16, a.att_self, a.q_dim, M * a.q_dim * 2, M,
                                       a.o1slab + (long)so * M * d, d, M * d * 4, d, red);
        fb_publish(cline(a.sync, L_P0 + (w & 7)), 1u);
        if constexpr (SELF) FS_TS(10);
    }
    kv_prefetch();

    // ---- Q: cross-q, 2 k-slices of 36 k-steps over nw / 2 workers each (<= 2 units)
    {
        const int qper = nw / 2, sq = w / qper, jq = w - sq * qper;
        if (sq < 2) {
            const int nu_q = (a.NGq - jq + qper - 1) / qper;
            bf16x8_s wq[2][3];
            // every wave's weights first, the poller's too: they were requested ~5 us before
            // N1 completes, so its poll is not held back by them, and wave 0's share no
            // longer starts only when the hand-off is seen
            fb_issue<FM_NW, 3, 2>(wq, a.Wq, a.NGq, d / 32, sq * 36, 36, jq, qper, nu_q);
            if (wave == 0) ok &= fm_wait_n<1>(a.sync, L_N1, (unsigned)M, tmo, 1u);
            T5G_TS(1);
            if constexpr (SELF) FS_TS(11);
            fb_finish<FM_NW, EPI_F32, 3, 2, 2>(wq, jq, qper, nu_q, sq * 36, 36, a.xn1, d, M * d * 2, M,
                                               a.qslab + (long)sq * M * a.q_dim, a.q_dim, M * a.q_dim * 4, a.q_dim,
                                               red);
            drain_vm();
            __syncthreads();
            if (tq == 0)
                for (int i = 0; i < nu_q; ++i)
                    __hip_atomic_fetch_add(cline(a.sync, L_Q0 + (jq + i * qper) / (D / 16)), 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // waves 8-10 of the workers that run no attention request the run's last gate/up unit
    // into LDS: 24 x 1 KiB each, no registers, while the attention workers run A (on an
    // attention worker the copies would queue ahead of its q loads). O's publish drains
    // them (vmcnt); its barrier makes them visible to the other waves.
    if (gu_lds && wave >= 8 && wave < 11) {
        const int wv = __builtin_amdgcn_readfirstlane(wave - 8);
        const __amdgpu_buffer_rsrc_t gr = frag_rsrc(a.Wgu, (uint32_t)NGg * (uint32_t)KBg * 1024u);
        const int gb = ((g_lo + nu_g - 1) * KBg + wv * (FB_GU_KB / 3)) * 1024 + lane * 16;
        __attribute__((address_space(3))) char* dst =
            (__attribute__((address_space(3))) char*)gul + wv * (FB_GU_KB / 3) * 1024;
#pragma unroll
        for (int q = 0; q < FB_GU_KB / 3; ++q)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(gr, dst + q * 1024, 16, gb + q * 1024, 0, 0, AUX_NT);
    }

    // ---- A (attention workers) with O's weight requests around it
    bf16x8_s wo[3][2];
    if (attnwg && wave >= 4 && owork) fb_issue<8, 2, 3>(wo, a.Wo, a.NGo, a.q_dim / 32, so * 16, 16, jo, oper, nu_o);
    if (attnwg) {
        const int qcnt = 2 * (D / 16);   // 16 q units per head x 2 k-slices
        if (wave == 0) ok &= fm_wait_n<1>(a.sync, L_Q0 + ah, (unsigned)qcnt, tmo, 2u);
        wg_barrier();
        const int n = alen;
        const int span = alen;
        if (tq < 256) {
            const int c4 = tq < D / 4 ? tq : 0;
            const int col = ah * D + 4 * c4;
            const __amdgpu_buffer_rsrc_t qr = raw_rsrc(a.qslab, (uint32_t)(2 * M * a.q_dim * 4));
            const f32x4 u0 = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(qr, (am * a.q_dim + col) * 4, 0, AUX_SC1));
            const f32x4 u1 = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(qr, ((M + am) * a.q_dim + col) * 4, 0, AUX_SC1));
            const f32x4 acc = u0 + u1;
            if (tq < D / 4) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) al.qs[4 * c4 + jj] = rbf(acc[jj]);
            }
        }
        fb_lds_barrier();   // LDS only: waves 4-7 keep their O weights in flight
        if (tq < 256) {
            float q[8];
            const float sg = dl < LPK / 2 ? -1.0f : 1.0f;
            const int pbase = (8 * dl + D / 2) % D;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const float x = al.qs[8 * dl + jj];
                const float pr = al.qs[pbase + jj];
                q[jj] = rbf(rbf(x * c8[jj]) + rbf((sg * pr) * s8[jj]));
            }
#pragma unroll
            for (int i = 0; i < NIT; ++i) {
                const int j = i * KPB + wave * KPW + kg;
                if (j >= n) {
                    kr[i] = (u32x4){0u, 0u, 0u, 0u};
                    vr[i] = (u32x4){0u, 0u, 0u, 0u};
                }
            }
            // every key's reduction before any store (they overlap), exchanges on the VALU
            float scs[NIT];
#pragma unroll
            for (int i = 0; i < NIT; ++i) {
                float sc = 0.f;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const float k0 = bf_lo(kr[i][jj]), k1 = bf_hi(kr[i][jj]);
                    sc += q[2 * jj] * k0 + q[2 * jj + 1] * k1;
                }
                scs[i] = xsum_v<LPK>(sc);   // xsum<LPK>'s adds
            }
            if (dl == 0) {
#pragma unroll
                for (int i = 0; i < NIT; ++i) al.sm[i * KPB + wave * KPW + kg] = fast_score(scs[i], a.scale, a.softcap);
            }
        }
        fb_lds_barrier();   // LDS only: waves 4-7 keep their O weights in flight
        if (wave == 0) {
            const float sc = lane < n ? al.sm[lane] : -INFINITY;
            const float mx = wave_max(sc);
            const float p = lane < n ? sdpa_p(__fsub_rn(sc, mx), lane, span) : 0.f;
            al.pl[lane] = p;
            if (lane < 16) al.pl[64 + lane] = 0.f;
            al.sm[lane] = rbf(p);
            __builtin_amdgcn_wave_barrier();
            const float l = sdpa_block_sum_lds<64>(al.pl, span, lane);
            if (lane == 0) al.stat_l = l;
        }
        fb_lds_barrier();   // LDS only: waves 4-7 keep their O weights in flight
        if (tq < 256) {
            float o[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) o[jj] = 0.f;
#pragma unroll
            for (int i = 0; i < NIT; ++i) {
                const int jl = i * KPB + wave * KPW + kg;
                const float p = al.sm[jl];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    o[2 * jj] += p * bf_lo(vr[i][jj]);
                    o[2 * jj + 1] += p * bf_hi(vr[i][jj]);
                }
            }
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) o[jj] += xlane32_v(o[jj]);   // LPK = 32: one xor-32 step
            if (kg == 0) {
                al.ored[wave][dl][0] = (f32x4){o[0], o[1], o[2], o[3]};
                al.ored[wave][dl][1] = (f32x4){o[4], o[5], o[6], o[7]};
            }
        }
        fb_lds_barrier();   // LDS only: waves 4-7 keep their O weights in flight
        if (tq < LPK && n > 0) {
            const int d8 = tq;
            const f32x4 lo4 = al.ored[0][d8][0] + al.ored[1][d8][0] + al.ored[2][d8][0] + al.ored[3][d8][0];
            const f32x4 hi4 = al.ored[0][d8][1] + al.ored[1][d8][1] + al.ored[2][d8][1] + al.ored[3][d8][1];
            const float inv = __fdiv_rn(1.0f, al.stat_l);
            u32x4 w;
            w[0] = pack2(__fmul_rn(lo4[0], inv), __fmul_rn(lo4[1], inv));
            w[1] = pack2(__fmul_rn(lo4[2], inv), __fmul_rn(lo4[3], inv));
            w[2] = pack2(__fmul_rn(hi4[0], inv), __fmul_rn(hi4[1], inv));
            w[3] = pack2(__fmul_rn(hi4[2], inv), __fmul_rn(hi4[3], inv));
            const __amdgpu_buffer_rsrc_t orr = raw_rsrc(a.att, (uint32_t)(M * a.q_dim * 2));
            __builtin_amdgcn_raw_buffer_store_b128(w, orr, (am * a.q_dim + ah * D + 8 * d8) * 2, 0, AUX_SC1);
        }
        // only wave 0 stored: it drains and publishes (the other waves' O weight requests
        // stay in flight)
        if (wave == 0) {
            drain_vm();
            if (lane == 0) __hip_atomic_fetch_add(cline(a.sync, L_A0 + ah), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // ---- O: cross-o, 4 k-slices of 16 k-steps over nw / 4 workers each (<= 3 units, 8 waves)
    if (owork) {
        // waves 0-7 (the GEMV) request their weights first; wave 11, idle in this stage and
        // with nothing queued, polls the 8 q heads
        if (!(attnwg && wave >= 4)) fb_issue<8, 2, 3>(wo, a.Wo, a.NGo, a.q_dim / 32, so * 16, 16, jo, oper, nu_o);
        if (wave == FM_NW - 1) ok &= fm_wait_n<8>(a.sync, L_A0, (unsigned)M, tmo, 3u);
        T5G_TS_BY(2, (FM_NW - 1) * 64);
        fb_finish<8, EPI_F32, 2, 3, 2>(wo, jo, oper, nu_o, so * 16, 16, a.att, a.q_dim, M * a.q_dim * 2, M,
                                       a.oslab + (long)so * M * d, d, M * d * 4, d, red);
        fb_publish(cline(a.sync, L_O0 + (w & 7)), 1u);
    }

    // ---- G: gate/up, contiguous unit runs over the workers (<= 5 units; the last from LDS
    // on the workers that fetched it)
    {
        bf16x8_s wg[5][6];
        const int nu_r = gu_lds ? nu_g - 1 : nu_g;
        fb_issue<FM_NW, 6, 5>(wg, a.Wgu, NGg, KBg, 0, KBg, g_lo, 1, nu_r);
        if (wave == 0) ok &= fm_wait_n<1>(a.sync, L_N2, (unsigned)M, tmo, 5u);
        T5G_TS(3);
        fb_finish<FM_NW, EPI_GEGLU, 6, 5, 0, true>(wg, g_lo, 1, nu_g, 0, KBg, a.xn, d, M * d * 2, M, a.act, f,
                                                   M * f * 2, 2 * f, red, gul, nu_r);
    }
    T5G_TS(4);
    const int units_per_slice = f / FM_DS / 8;
    drain_vm();
    __syncthreads();
    if (tq == 0 && nu_g > 0) {
        const int s0 = g_lo / units_per_slice, s1 = (g_lo + nu_g - 1) / units_per_slice;
        for (int sl = s0; sl <= s1; ++sl) {
            const int n = min(g_lo + nu_g, (sl + 1) * units_per_slice) - max(g_lo, sl * units_per_slice);
            __hip_atomic_fetch_add(a.sync + fs_slice(sl), (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // ---- D: down, 8 k-slices of 36 k-steps over nw / 8 workers each (<= 5 units)
    const int dper = nw / FM_DS, s = w / dper, j = w - s * dper;
    if (s < FM_DS) {
        const int KBd = f / 32, per = KBd / FM_DS;
        const int nu_d = (a.NGd - j + dper - 1) / dper;
        bf16x8_s wd[5][3];
        fb_issue<FM_NW, 3, 5>(wd, a.Wd, a.NGd, KBd, s * per, per, j, dper, nu_d);
        if (wave == 0) ok &= fm_wait_n<1>(a.sync, L_SL0 + s, (unsigned)units_per_slice, tmo, 6u + s);
        T5G_TS(5);
        fb_finish<FM_NW, EPI_F32, 3, 5, 2>(wd, j, dper, nu_d, s * per, per, a.act, f, M * f * 2, M,
                                           a.dslab + (long)s * M * d, d, M * d * 4, d, red);
        fb_publish(cline(a.sync, L_D0 + (w & 7)), 1u);
    }

    // ---- QKV: the next layer's q|k|v, 2 k-slices of 36 k-steps over nw / 2 workers each
    // (<= 3 units), weights requested while N3 runs
    if (a.Wqkv) {
        const int kper = nw / 2, sk = w / kper, jk = w - sk * kper;
        if constexpr (SM == 2) {
            // the tail: q|k|v written through and handed off in-launch, the next layer's self
            // attention (its K / V requested before the N3 wait), then the next layer's O1
            const int nu_k = sk < 2 ? (a.NGqkv - jk + kper - 1) / kper : 0;
            bf16x8_s wk[3][3];
            fb_issue<FM_NW, 3, 3>(wk, a.Wqkv, a.NGqkv, d / 32, sk * 36, 36, jk, kper, nu_k);
            auto mid = [&]() __attribute__((always_inline)) {
                // wave 11 (group 2: never a chunk slot in the tail, so no K / V queued ahead of
                // its polls) waits for N3, then for every q|k|v workgroup
                if (wave == FM_NW - 1) ok &= fm_wait_n<1>(a.sync, L_N3, (unsigned)M, tmo, 15u);
                FS_TS_BY(17, (FM_NW - 1) * 64);
                fb_finish<FM_NW, EPI_F32, 3, 3, 2>(wk, jk, kper, nu_k, sk * 36, 36, a.xn, d, M * d * 2, M,
                                                   a.qkv_out + (long)sk * M * a.qkv_dim, a.qkv_dim,
                                                   M * a.qkv_dim * 4, a.qkv_dim, red);
                fb_publish(cline(a.sync, L_K0 + (w & 7)), 1u);   // every worker (an odd one projects nothing)
                FS_TS(18);
                if (wave == FM_NW - 1) ok &= fm_wait_split<8>(a.sync, L_K0, (unsigned)nw, tmo, 19u);
                FS_TS_BY(19, (FM_NW - 1) * 64);
                wg_barrier();
            };
            fb_self_attn<true>(a, *(FbSelfLds*)gul, mid, nw, len_tail);
            // the next layer's O1: k-slice so waits for kv head so's rows
            if (owork) {
                bf16x8_s w1[3][2];
                fb_issue<8, 2, 3>(w1, a.Wo1n, a.NGo, a.q_dim / 32, so * 16, 16, jo, oper, nu_o);
                if (wave == FM_NW - 1) ok &= fm_wait_n<1>(a.sync, L_S0 + so, (unsigned)M, tmo, 20u);
                FS_TS_BY(20, (FM_NW - 1) * 64);
                fb_finish<8, EPI_F32, 2, 3, 2>(w1, jo, oper, nu_o, so * 16, 16, a.att_self, a.q_dim, M * a.q_dim * 2, M,
                                               a.o1n + (long)so * M * d, d, M * d * 4, d, red);
                FS_TS(21);
            }
        } else if (sk < 2) {
            const int nu_k = (a.NGqkv - jk + kper - 1) / kper;
            bf16x8_s wk[3][3];
            fb_issue<FM_NW, 3, 3>(wk, a.Wqkv, a.NGqkv, d / 32, sk * 36, 36, jk, kper, nu_k);
            if (wave == 0) ok &= fm_wait_n<1>(a.sync, L_N3, (unsigned)M, tmo, 15u);
            fb_finish<FM_NW, EPI_F32, 3, 3, 1>(wk, jk, kper, nu_k, sk * 36, 36, a.xn, d, M * d * 2, M,
                                               a.qkv_out + (long)sk * M * a.qkv_dim, a.qkv_dim, 0, a.qkv_dim, red);
        }
    }
    (void)ok;
    T5G_TS(6);
}

constexpr size_t FM_LDS_MAX = 160 * 1024;

static int fused_mlp_launch(const FusedMlpArgs& a_in, hipStream_t st, bool launch);
int fused_mlp(const FusedMlpArgs& a_in, hipStream_t st) { return fused_mlp_launch(a_in, st, true); }
int fused_mlp_check(const FusedMlpArgs& a_in) { return fused_mlp_launch(a_in, nullptr, false); }

static int fused_mlp_launch(const FusedMlpArgs& a_in, hipStream_t st, bool launch) {
    FusedMlpArgs a = a_in;
    if (a.M <= 0) return 0;
    // the shapes the stages are built for: K = 2304 gate/up (72 k-steps), f = 9216 down in
    // 8 slices of 36 k-steps, 4 cross-o slabs, <= 32 rows
    if (a.M > 32 || a.d != 2304 || a.f != 9216 || a.f % 64) return -1;
    if (!a.part_in || !a.post_w || !a.pre_w || !a.h || !a.xn || !a.Wgu || !a.act || !a.Wd || !a.part_out || !a.sync ||
        !a.sync_next || !a.timeout || a.sync_next == a.sync)
        return -1;
    if (a.NGgu * 8 != a.f || a.NGd * 16 != a.d) return -1;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev))
        return -2;
    const int nb = a.grid > 0 ? a.grid : cus;
    if (nb > cus || nb < FM_DS || nb < a.M) return -1;   // every workgroup must be resident at once
    const int nr = nb - a.M, rest = a.NGgu - a.M * FM_NORM_UNITS;
    if (nr <= 0 || rest < 0) return -1;
    const int nu_g = (rest + nr - 1) / nr;
    const int nu_d = (a.NGd + nb / FM_DS - 1) / (nb / FM_DS);
    if (nu_g > 5 || nu_d > 5) return -1;   // UMAX = 5 batches per wave (needs >= 231 workgroups)
    const int MT = a.M > 16 ? 2 : 1;
    if (a.xattn) {
        // the cross-attention chain: 2 k-slices x NGq cross-q units = one unit-slice per
        // workgroup, 4 x 64 cross-o workgroups, 8 x 32 down workgroups; one 64-key chunk of
        // text keys; attention and norm workgroups disjoint
        const int nw = nb - a.M;   // workers (the last M workgroups run the norms)
        auto most = [](int units, int per) { return per > 0 ? (units + per - 1) / per : 1 << 20; };
        if (MT != 1 || most(a.NGq, nw / 2) > 2 || most(a.NGo, nw / 4) > 3 || most(a.NGd, nw / FM_DS) > 5 ||
            most(a.NGgu, nw) > 5 || (a.Wqkv && most(a.NGqkv, nw / 2) > 3))
            return -1;
        if (a.D != 256 || a.Hq * a.D != a.q_dim || a.Hq % a.Hkv || a.Hq > 8 ||
            a.NGq * 16 != a.q_dim || a.NGo * 16 != a.d || a.text_max > 64 || a.text_max > a.kv_cap || a.M * a.Hq > nw || !a.o_slabs ||
            !a.post1_w || !a.pre1_w || !a.xn1 || !a.Wq || !a.qslab || !a.ck || !a.cv || !a.enc_len || !a.rope_tab ||
            !a.att || !a.Wo || !a.oslab)
            return -1;
        if (!a.dslab || !a.post3_w || !a.pre3_w) return -1;
        if (a.Wo1 && (!a.att_self || !a.o1slab)) return -1;
        // stage S: 8 q heads over 4 kv heads of 256 (O1's 4 k-slices = the 4 head pairs), the
        // flash kernel's chunk records (rows of <= s_nsplit x 64 keys, checked by the host)
        if (a.self_attn &&
            (!a.Wo1 || !a.qkv_in || !a.sk || !a.sv || !a.kv_len || !a.fpart || !a.fstat || !a.fticket || a.Hq != 8 ||
             a.Hkv != 4 || a.D != FS_D || a.M > FS_MAXROWS || a.qkv_dim != a.q_dim + 2 * a.Hkv * a.D || a.s_cap < 1 ||
             a.s_nsplit < 1 || a.s_nsplit > DEC_MAX_CHUNKS || a.s_nsplit > (a.s_cap + FS_CH - 1) / FS_CH ||
             a.window < 0 || (long)a.M * a.Hkv * a.s_nsplit * FS_G * FS_D * 4 > 0x7fff0000L ||
             a.M * a.Hkv * a.s_nsplit > FS_GRP * nb * FS_MAXPASS))   // <= 3 chunks per workgroup and pass
            return -1;
        if (a.Wqkv && (!a.qkv_out || a.NGqkv * 16 != a.qkv_dim)) return -1;
        a.norm_b0 = nb - a.M;
        static_assert(FB_GU_KB == FM_NW * 6 && FB_GU_KB % 3 == 0 && FB_LDS <= FM_LDS_MAX, "gate/up LDS unit");
        if (a.d != FB_D) return -1;
        const size_t shm = FB_LDS;
        // function attributes and the occupancy check are per device (an engine per GPU in
        // one process must not skip the second device's hipFuncSetAttribute)
        if (dev < 0 || dev >= 64) return -1;
        // the tail: the next layer's S after the q|k|v stage, then its O1 (front O1 off); slots
        // on groups 0-1 of the workers only (group 2 polls), the S scratch in the gate/up unit's LDS
        static_assert(sizeof(FbSelfLds) <= (size_t)FB_GU_KB * 1024, "tail S scratch in the gate/up unit LDS");
        if (a.self_tail &&
            (a.self_attn || a.Wo1 || !a.Wqkv || !a.Wo1n || !a.o1n || !a.att_self || a.qkv_in != a.qkv_out ||
             !a.sk || !a.sv || !a.kv_len || !a.fpart || !a.fstat || !a.fticket || a.Hq != 8 || a.Hkv != 4 ||
             a.D != FS_D || a.M > FS_MAXROWS || a.qkv_dim != a.q_dim + 2 * a.Hkv * a.D || a.s_cap < 1 ||
             a.s_nsplit < 1 || a.s_nsplit > DEC_MAX_CHUNKS || a.s_nsplit > (a.s_cap + FS_CH - 1) / FS_CH || a.window < 0 ||
             a.M * a.Hkv * a.s_nsplit > 2 * (nb - a.M) || (long)a.M * a.Hkv * a.s_nsplit * FS_G * FS_D * 4 > 0x7fff0000L))
            return -1;
        const int sv = a.self_tail ? 2 : a.self_attn ? 1 : 0;
        auto* fb = sv == 2 ? fused_block_kernel<2> : sv ? fused_block_kernel<1> : fused_block_kernel<0>;
        static bool attr_b[64][3] = {};
        if (!attr_b[dev][sv]) {
            (void)hipFuncSetAttribute((const void*)fb, hipFuncAttributeMaxDynamicSharedMemorySize, (int)FM_LDS_MAX);
            int occ = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fb, FM_NW * 64, shm) != hipSuccess || occ < 1)
                return -1;
            attr_b[dev][sv] = true;
        }
        if (!launch) return 0;
        hipLaunchKernelGGL(fb, dim3((unsigned)nb), dim3(FM_NW * 64), shm, st, a);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    const size_t shm = (size_t)5 * MT * FM_NW * 64 * 16;
    if (shm > FM_LDS_MAX) return -1;
    // norm rows on workgroups with one gate/up unit fewer (their weight stream starts after
    // the norm): the last ones
    a.norm_b0 = nb - a.M;
    auto* fn = MT == 1 ? fused_mlp_kernel<1> : fused_mlp_kernel<2>;
    if (dev < 0 || dev >= 64) return -1;
    static bool attr[64][2] = {};
    if (!attr[dev][MT - 1]) {
        (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)FM_LDS_MAX);
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, FM_NW * 64, shm) != hipSuccess || occ < 1) return -1;
        attr[dev][MT - 1] = true;
    }
    if (!launch) return 0;
    hipLaunchKernelGGL(fn, dim3((unsigned)nb), dim3(FM_NW * 64), shm, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

// Parity mode's decode layer after the self attention as ONE persistent launch (one
// 512-thread workgroup per CU), the exact-order counterpart of fused.hip:
//
//   O1  o-projection of the self-attention output              (144 groups of 16 outputs)
//   N1  h = h + RMSNorm_post(o); xn = RMSNorm_pre(h)          (one norm workgroup per row)
//   Q   cross-q projection                                     (128 groups)
//   A   PM cross attention over <= 64 text keys, q RoPE        (row x kv head x 32-dim slice)
//   O   cross-o projection                                     (144 groups)
//   N2  norm pair
//   G   gate/up + GeGLU                                        (1 152 groups, contiguous runs)
//   D   down projection in the reference's 2 K parts           (144 groups x 2 parts)
//   N3  norm pair from the parts (the next layer's input norm, or the final norm)
//   QKV the next layer's q|k|v                                 (256 groups)
//
// replacing ten launches of the per-op parity path (xmm.hip xmm_dec_kernel, norm.hip
// resid_norm_kernel EXACT, xattn.hip xattn_single_kernel; hf_export/modeling_t5gemma_voice.py
// :256-323, [tf] modeling_t5gemma.py:81-97). Every stage is the arithmetic of the launch it
// replaces, on the same shared device pieces (exact_dev.h: the E/O chunk MFMAs, the aten
// AVX2 sum-of-squares cascade and RMSNorm, RoPE), folded in the same order, so the launch is
// bitwise equal to the per-op launches and to the reference's CPU run (tests/test_gpu_exact.py
// golden tests run both).
//
// What it buys: nine launch boundaries per layer, and every stage's weights requested before
// the hand-off its activations wait for, so each weight stream is in flight while the previous
// stage finishes. Hand-offs follow fused.hip / cdna_hip_programming.md Guideline 16 R1: every
// handed-off byte is stored sc1 (write-through) by the wave that computed it, every storing
// wave drains (vmcnt(0)), the workgroup meets at a barrier, one lane adds to a relaxed
// agent-scope counter (arrivals spread over up to 8 lines of 128 bytes); the consumer's wave 0
// polls its lines in one round trip per poll, the workgroup meets it at a barrier, and every
// load of handed-off bytes is an sc1 load. Each layer has its own counter set; a launch zeroes
// the NEXT layer's set as it starts (its last user, the previous step's launch of that layer,
// has completed). Every wait is bounded (fused.hip's sticky timeout word: a wait that gives up
// makes every later one give up at once; t5g_read_tokens reports T5G_EHANDOFF and engine.py
// reruns the call on the per-op launches).
#include "common.h"
#include "exact_dev.h"
#include "exact_math.h"
#include "t5g_kernels.h"

// diagnostic stage timeline (T5G_DBG_TS library variant only, tools/xlayer_timeline.py):
// thread 0 of every workgroup stores the 100 MHz clock at numbered points of the launches
// that run a next layer's q|k|v, 32 slots per workgroup
#ifdef T5G_DBG_TS
__device__ unsigned long long* xl_ts_buf;
extern "C" int t5g_dbg_set_xlayer(void* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(xl_ts_buf), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
// timing variants of the GEMV stages (never in the product): 1 no MFMA, 2 no fold, 3 no
// weight loads
__device__ int xl_dbg_var;
extern "C" int t5g_dbg_set_xlayer_var(int v) {
    return hipMemcpyToSymbol(HIP_SYMBOL(xl_dbg_var), &v, sizeof(v)) == hipSuccess ? 0 : -1;
}
#define XL_DBG_VAR xl_dbg_var
#define XL_TS(k)                                                                                   \
    do {                                                                                           \
        if (threadIdx.x == 0 && xl_ts_buf && a.Wqkv)                                              \
            xl_ts_buf[blockIdx.x * 32 + (k)] = __builtin_amdgcn_s_memrealtime();                   \
    } while (0)
#else
#define XL_DBG_VAR 0
#define XL_TS(k) do { } while (0)
#endif

namespace t5g {

constexpr int XL_NW = 8;                    // waves per workgroup (xmm_dec_kernel's count)
constexpr int XL_CPW = 9;                   // chunks per wave per task
constexpr int XL_SC = XL_NW * XL_CPW;       // 72 chunks: the most any task has (K = 2304)
constexpr int XL_EL = 8 * 16;               // chunk-sum elements of a group: 8 rows x 16 outputs
constexpr int XL_D = 2304, XL_F = 9216, XL_QD = 2048, XL_KVD = 1024, XL_HD = 256, XL_G = 2, XL_HKV = 4;
constexpr int XL_DOWN_KBC = 144;            // the reference's K part of the down projection at M = 1 (chunks)
constexpr unsigned XL_SPIN_MAX = 1u << 18;
constexpr int XL_AUX_SC1 = 16;
constexpr int XL_XWIN = 144;                // X window chunks in LDS: the down projection's K part

// counter set lines (one word per 128-byte line)
constexpr int XC_O1 = 0, XC_N1 = 8, XC_Q = 9, XC_A = 13, XC_O = 21, XC_N2 = 29, XC_G0 = 30, XC_G1 = 38, XC_D = 46,
              XC_N3 = 54;
static_assert(XC_N3 + 1 <= XL_SET_LINES, "xlayer counter set layout");

__device__ __forceinline__ unsigned* xline(unsigned* set, int line) { return set + line * FM_LINE; }
__device__ __forceinline__ unsigned xl_ld_rlx(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void xl_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void xl_barrier() { asm volatile("s_barrier" ::: "memory"); }
// the workgroup meets after its LDS accesses completed -- and NOT after its outstanding global
// loads: __syncthreads() is a workgroup release fence + barrier, which waits vmcnt(0), i.e. for
// the next pass's weights requested ahead (that wait serialised every weight stream behind the
// MFMAs: G stage 25 us -> see DESIGN.md)
__device__ __forceinline__ void xl_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// one wave polls the N lines a stage's arrivals are spread over (any distribution) until
// their sum reaches `total`: one memory round trip per poll; lane 63 watches the timeout word
template <int N>
__device__ __forceinline__ bool xl_wait(unsigned* set, int line0, unsigned total, unsigned* tmo, unsigned code) {
    static_assert(N >= 1 && N <= 8, "lines per stage");
    const int lane = threadIdx.x & 63;
    unsigned* p = lane == 63 ? tmo : xline(set, line0 + min(lane, N - 1));
    for (unsigned spins = 0;; ++spins) {
        const unsigned v = xl_ld_rlx(p);
        unsigned sum = lane < N ? v : 0u;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) sum += __shfl_xor(sum, o, 64);   // lanes 0..7 hold the total
        if (__shfl(sum, 0, 64) >= total) return true;
        if (__shfl(v, 63, 64) != 0) return false;
        if (spins > XL_SPIN_MAX) {
            if (lane == 0) __hip_atomic_store(tmo, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}
// the whole workgroup waits: wave 0 polls, every wave meets it at the barrier
template <int N>
__device__ __forceinline__ void xl_wait_wg(unsigned* set, int line0, unsigned total, unsigned* tmo, unsigned code) {
    if (threadIdx.x < 64) (void)xl_wait<N>(set, line0, total, tmo, code);
    xl_barrier();
}
// every storing wave drains, the workgroup meets, one lane adds n arrivals to `line`
__device__ __forceinline__ void xl_publish(unsigned* set, int line, unsigned n) {
    xl_drain();
    __syncthreads();
    if (threadIdx.x == 0 && n) __hip_atomic_fetch_add(xline(set, line), n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xl_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                             (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// ---------------------------------------------------------------- exact decode GEMV tasks
// xmm_dec_kernel<1, true, EPI, PART> (rows M <= 8; R8: lanes j >= 8 read lane j - 8's X
// fragment) for one task = (16-output group g, chunk range): the 8 waves take the chunks
// round-robin, chunk sums go to LDS [chunk][row][col], thread t < 128 folds element (row
// t >> 4, col t & 15) over the chunks in order as one plain chain from 0 (the reference
// splits none of these Linears at M = 1 but the down projection, whose two K parts are two
// tasks, each folded from 0), then the epilogue stores sc1.
// one pass of <= 72 chunks of a task; a task of more chunks (the down projection's 144-chunk
// parts) is several passes whose fold continues one chain (first / last pass flags). xb: the
// first chunk of the X window the pass reads (the stage's whole K, or the down part's range)
struct XlTask {
    int g, kb_lo, kb_hi, part, xb;
    bool first, last;
};
struct XlGemv {
    const bf16_t* W;                     // E16 weights, NG groups x KB chunks
    int KB;                              // chunks of the full K (the weight row stride)
    __amdgpu_buffer_rsrc_t x;            // X16 of the operand rows (sc1 loads)
    int N, M;
    __amdgpu_buffer_rsrc_t y, part;      // outputs (sc1 stores): Y [M][N] bf16 or Y16 / parts
    bool y16;                            // EPI_BF16: Y is row-major [M][N]; GEGLU: Y is the X16 act (K = N / 2)
    int xwin;                            // chunks of the X window staged in LDS (<= XL_XWIN)
};
// the weights of one pass in registers: wave w holds chunks w, w + 8, ... (<= 9)
struct XlW {
    u32x4 w[XL_CPW];
};
__device__ __forceinline__ void xl_issue_w(XlW& o, const XlGemv& s, const XlTask& t, int wave, int lane) {
    if (XL_DBG_VAR == 3) {
#pragma unroll
        for (int c = 0; c < XL_CPW; ++c) o.w[c] = u32x4{(unsigned)t.g, 0u, 0u, (unsigned)lane};
        return;
    }
    const u32x4* wp = (const u32x4*)(s.W + (long)t.g * s.KB * 512) + lane;
#pragma unroll
    for (int c = 0; c < XL_CPW; ++c) {
        const int kb = min(t.kb_lo + wave + c * XL_NW, t.kb_hi - 1);
        o.w[c] = wp[(long)kb * 64];
    }
}
// the X window [xb, xb + xwin) of rows 0..7 into LDS once per stage (per down part): per chunk
// the 32 lanes (q, j < 8) of the X16 tile, 512 bytes (R8: lanes j >= 8 read lane j - 8's)
__device__ __forceinline__ void xl_fill_x(const XlGemv& s, int xb, u32x4* xs) {
    const int n = s.xwin * 32;
    u32x4 v[XL_XWIN * 32 / 512];
#pragma unroll
    for (int u = 0; u < XL_XWIN * 32 / 512; ++u) {
        const int i = min((int)threadIdx.x + u * 512, n - 1), kb = xb + (i >> 5), r = i & 31;
        int off = (kb * 64 + (r >> 3) * 16 + (r & 7)) * 16;
        asm volatile("" : "+v"(off));
        v[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(s.x, off, 0, XL_AUX_SC1));
    }
#pragma unroll
    for (int u = 0; u < XL_XWIN * 32 / 512; ++u) {
        const int i = (int)threadIdx.x + u * 512;
        if (i < n) xs[i] = v[u];
    }
}
// the chunk MFMAs of one pass into LDS cs[chunk][XL_EL], X from the LDS window
__device__ __forceinline__ void xl_mfma(const XlW& o, const XlTask& t, const u32x4* xs, float* cs, int wave,
                                        int lane) {
    const int n = t.kb_hi - t.kb_lo, j = lane & 15, q = lane >> 4;
    const u32x4* xl = xs + (t.kb_lo - t.xb) * 32 + q * 8 + (lane & 7);
    if (XL_DBG_VAR == 1) {
        if (j < 8) *(f32x4_t*)&cs[wave * XL_EL + j * 16 + 4 * q] = (f32x4_t){__uint_as_float(o.w[0][0]),
                                                                          __uint_as_float(o.w[8][1]), 0.f, 0.f};
        return;
    }
#pragma unroll
    for (int c = 0; c < XL_CPW; ++c) {
        const int cc = wave + c * XL_NW;
        if (cc < n) {
            const f32x4_t v = xmm_chunk(o.w[c], xl[cc * 32]);
            if (j < 8) *(f32x4_t*)&cs[cc * XL_EL + j * 16 + 4 * q] = v;
        }
    }
}
// folder thread tid < 128: ((part + c0) + c1) + ... over the pass's chunks, 16 per LDS round trip
__device__ __forceinline__ float xl_fold(const float* cs, int n, int tid, float part) {
    for (int c0 = 0; c0 < n; c0 += 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = cs[min(c0 + u, XL_SC - 1) * XL_EL + tid];
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
// epilogues (xmm.hip xdec_store, the decode calls' operands): EPI_BF16 -> Y [M][N] bf16;
// EPI_GEGLU -> the act in X16 (K = N / 2); PART -> fp32 part[part][M][N]; all sc1
template <int EPI, bool PART>
__device__ __forceinline__ void xl_store(const XlGemv& s, const XlTask& t, int m, int fcol, float y) {
    const int n = t.g * 16 + fcol;
    if constexpr (PART) {
        if (m < s.M && n < s.N)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), s.part, ((t.part * s.M + m) * s.N + n) * 4, 0,
                                                  XL_AUX_SC1);
        return;
    }
    if constexpr (EPI == EPI_GEGLU) {
        const float up = xlane<8>(y);   // col + 8 of the same row: the up row of this feature
        if (fcol >= 8 || m >= s.M) return;
        const int ft = t.g * 8 + fcol;
        if (ft >= s.N / 2) return;
        const bf16_t v = f2bf(rbf(__fmul_rn(rbf(t5g_exact::gelu_tanh(rbf(y))), rbf(up))));
        __builtin_amdgcn_raw_buffer_store_b16(v, s.y, (int)(x16_off(m, ft, s.N / 64) * 2), 0, XL_AUX_SC1);
        return;
    }
    if (m >= s.M || n >= s.N) return;
    __builtin_amdgcn_raw_buffer_store_b16(f2bf(rbf(y)), s.y, (m * s.N + n) * 2, 0, XL_AUX_SC1);
}

// LDS of a GEMV stage: the X window, two chunk-sum buffers (the fold of pass i reads one while
// the MFMAs of pass i + 1 fill the other)
struct XlGemvLds {
    u32x4* xs;
    float* cs0;
    float* cs1;
};

// the workgroup's passes [t0, t1) of one GEMV stage. The first pass's weights are requested
// before the stage's hand-off (wait()), then the X window is staged in LDS; each next pass's
// weights are requested before the current pass's MFMAs (two register buffers), and the
// folder threads fold pass i while the other waves run pass i + 1's MFMAs (one barrier per
// pass)
struct XlNoAfter {
    __device__ void operator()(int) const {}
};
template <int EPI, bool PART, typename TaskOf, typename Wait, typename After = XlNoAfter>
__device__ __forceinline__ void xl_gemv(const XlGemv& s, int t0, int t1, TaskOf task_of, const XlGemvLds& L,
                                        Wait wait, After after = After()) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (t0 >= t1) return;
    float acc = 0.f;   // folder threads: the chain across a task's passes
    int xb_cur = -1;
    XlW wa, wb;
    xl_issue_w(wa, s, task_of(t0), wave, lane);
    wait();
    auto pass = [&](XlW& cur, XlW& nxt, int i, float* cs) {
        const XlTask t = task_of(i);
        if (t.xb != xb_cur) {   // uniform: a new X window (the stage's first pass, a down part change)
            xl_lds_barrier();   // every earlier reader of the LDS window is done
            xl_fill_x(s, t.xb, L.xs);
            xl_lds_barrier();
            xb_cur = t.xb;
        }
        if (i + 1 < t1) xl_issue_w(nxt, s, task_of(i + 1), wave, lane);
        xl_mfma(cur, t, L.xs, cs, wave, lane);
        xl_lds_barrier();
        if (tid < XL_EL) {
            acc = XL_DBG_VAR == 2 ? cs[tid] : xl_fold(cs, t.kb_hi - t.kb_lo, tid, t.first ? 0.f : acc);
            if (t.last) xl_store<EPI, PART>(s, t, tid >> 4, tid & 15, acc);
        }
        if (t.last) after(i);   // uniform: the task's outputs are stored (by the folder threads)
    };
    for (int i = t0; i < t1; i += 2) {
        pass(wa, wb, i, L.cs0);
        if (i + 1 < t1) pass(wb, wa, i + 1, L.cs1);
    }
    xl_lds_barrier();   // the folds are done before the LDS is reused
}

struct XlNoTs {
    __device__ void operator()(int) const {}
};

// ---------------------------------------------------------------- exact norm (one row)
// resid_norm_kernel<NS, SRC, true> for one row with post, residual and pre (512 threads, the
// first d / 8 active): v = bf16(delta) (NS = 0) or bf16((0 + p0) + p1) (NS = 2, the down
// parts), post-norm, + h, pre-norm. The row's h stays in LDS between the launch's three
// norms (hrow) and goes back to HBM at N3; xn goes out row-major (plain) and in X16 (sc1).
template <int NS, typename Wait, typename Ts = XlNoTs>
__device__ __forceinline__ void xl_norm_row(const XLayerArgs& a, int m, const bf16_t* post_w, const bf16_t* pre_w,
                                            u32x4* hrow, bool first, bool last, float* sq, Wait wait, Ts ts = Ts()) {
    const int d = XL_D, c = threadIdx.x;
    const bool active = 8 * c < d;
    const int cc = active ? c : d / 8 - 1;
    // the norm weights and the launch's input h row are requested before the hand-off
    const u32x4 w_post = *(const u32x4*)(post_w + 8 * cc);
    const u32x4 w_pre = *(const u32x4*)(pre_w + 8 * cc);
    u32x4 rw = first ? *(const u32x4*)(a.h + (long)m * d + 8 * cc) : u32x4{0u, 0u, 0u, 0u};
    wait();
    if (!first) rw = hrow[cc];
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (NS == 0) {
        const __amdgpu_buffer_rsrc_t dr = xl_rsrc(a.tmp, (uint32_t)(a.M * d * 2));
        const u32x4 dw =
            __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(dr, (m * d + 8 * cc) * 2, 0, XL_AUX_SC1));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[2 * j] = bf_lo(dw[j]);
            v[2 * j + 1] = bf_hi(dw[j]);
        }
    } else {
        const __amdgpu_buffer_rsrc_t pr = xl_rsrc(a.dpart, (uint32_t)(NS * a.M * d * 4));
        f32x4 p[NS][2];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const int off = ((s * a.M + m) * d + 8 * cc) * 4;
            p[s][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, off, 0, XL_AUX_SC1));
            p[s][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, off + 16, 0, XL_AUX_SC1));
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
    }
    ts(0);
    rms8_exact(v, active, d, w_post, a.eps, sq);
    ts(1);
    {
        float r8[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            r8[2 * j] = bf_lo(rw[j]);
            r8[2 * j + 1] = bf_hi(rw[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rbf(r8[j] + v[j]);
    }
    __syncthreads();   // every thread has read hrow before it is rewritten
    if (active) {
        u32x4 hw;
#pragma unroll
        for (int j = 0; j < 4; ++j) hw[j] = pack2(v[2 * j], v[2 * j + 1]);
        hrow[c] = hw;
        if (last) *(u32x4*)(a.h + (long)m * d + 8 * c) = hw;   // read by the next launch
    }
    ts(2);
    rms8_exact(v, active, d, w_pre, a.eps, sq);
    ts(3);
    if (active) {
        u32x4 pk;
#pragma unroll
        for (int j = 0; j < 4; ++j) pk[j] = pack2(v[2 * j], v[2 * j + 1]);
        *(u32x4*)(a.xn + (long)m * d + 8 * c) = pk;   // row-major copy (not read in this launch)
        const __amdgpu_buffer_rsrc_t xr = xl_rsrc(a.xn16, (uint32_t)(16 * d * 2));
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
            __builtin_amdgcn_raw_buffer_store_b32(pk[jj], xr, (int)(x16_off(m, 8 * c + 2 * jj, d / 32) * 2), 0,
                                                  XL_AUX_SC1);
    }
}

// ---------------------------------------------------------------- PM cross attention task
// xattn_single_kernel<2, 256, true> for task (row qi, kv head, 32-dim slice z), on threads
// 0..255 of the workgroup (the others only meet the barriers): the row's <= 64 scores in the
// gemv order (four threads per key), exact p of the one block, aten's block sum, the 8-key
// group chains of the slice, output x 1/l. q arrives un-rotated from this launch's Q stage
// (sc1 loads) and is rotated while staged; the output goes out in X16 (sc1) and row-major.
struct XlAttnLds {
    float qs[XL_G][XL_HD];
    float wmax[4][XL_G];
    float ss[XL_G][64];
    float pex[XL_G][64 + 16];
    float pbf[XL_G][64];
    float tmp[8][XL_G][32];
    float l_s[XL_G];
};
template <typename Wait, typename Ts = XlNoTs>
__device__ __forceinline__ void xl_cross_attn(const XLayerArgs& a, int qi, int kvh, int z, XlAttnLds& S, Wait wait,
                                              Ts ts = Ts()) {
    constexpr int D = XL_HD, G = XL_G, NCB = D / 32, H2 = D / 2, DZ = 32, DP = DZ / 2, NG8 = 8, CH = 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kl = (tid & 255) >> 2, qa = tid & 3;
    const bool on = tid < 256;
    const int row = qi;
    const int lo = 0, hi = min(a.enc_len[row], CH);
    const int span = hi - lo;
    const int key = lo + kl;
    const bool valid = key < hi;
    const bf16_t* kr = a.ck + row * a.kv_bstride + kvh * a.kv_hstride + (long)(valid ? key : lo) * D + 8 * qa;
    u32x4 kv[NCB];
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) kv[cb] = *(const u32x4*)(kr + 32 * cb);
    const int dp = tid % DP, gl = (tid & 255) / DP;
    const bool vlane = on && gl < NG8;
    const bf16_t* Vb = a.cv + row * a.kv_bstride + kvh * a.kv_hstride + (long)lo * D + z * DZ;
    uint32_t vw[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        vw[j] = *(const uint32_t*)(Vb + (long)min(vlane ? gl * 8 + j : 0, max(span - 1, 0)) * D + 2 * dp);
    wait();   // K / V (written before the launch) in flight across the hand-off
    if (on) {
        const float* tab = a.rope_tab + (long)row * D;
        const __amdgpu_buffer_rsrc_t qr = xl_rsrc(a.q, (uint32_t)(a.M * XL_QD * 2));
        for (int i = tid; i < G * H2; i += 256) {
            const int g = i / H2, dd = i % H2;
            const int base = (qi * XL_QD + (kvh * G + g) * D) * 2;
            const float x1 = bf2f(__builtin_amdgcn_raw_buffer_load_b16(qr, base + dd * 2, 0, XL_AUX_SC1));
            const float x2 = bf2f(__builtin_amdgcn_raw_buffer_load_b16(qr, base + (dd + H2) * 2, 0, XL_AUX_SC1));
            float o1, o2;
            xd_rope(x1, x2, tab[dd], tab[H2 + dd], o1, o2);
            S.qs[g][dd] = o1;
            S.qs[g][dd + H2] = o2;
        }
    }
    __syncthreads();
    ts(0);
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
            const float* qc = &S.qs[g][cb * 32 + 8 * qa];
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
        const bool own = on && valid && qa == 0;
        const float sv = own ? sc : -INFINITY;
        if (own) S.ss[g][kl] = sv;
        const float mx = wave_max(sv);
        if (on && lane == 0) S.wmax[wave][g] = mx;
    }
    __syncthreads();
    ts(1);
    // exact p of the block, both q heads at once (threads g * 64 + key)
    if (tid < G * CH) {
        const int g = tid / CH, kk = tid % CH;
        const float mb = fmaxf(fmaxf(S.wmax[0][g], S.wmax[1][g]), fmaxf(S.wmax[2][g], S.wmax[3][g]));
        const float p = kk < span ? sdpa_p(__fsub_rn(S.ss[g][kk], mb), kk, span) : 0.f;
        S.pex[g][kk] = p;
        S.pbf[g][kk] = rbf(p);
    } else if (tid < G * CH + G * 16) {
        const int i = tid - G * CH;
        S.pex[i / 16][CH + i % 16] = 0.f;
    }
    __syncthreads();
    if (wave < G) {
        const int g = wave;
        const float mb = fmaxf(fmaxf(S.wmax[0][g], S.wmax[1][g]), fmaxf(S.wmax[2][g], S.wmax[3][g]));
        const float ts = sdpa_block_sum_lds<CH>(S.pex[g], span, lane);
        const float l = fmaf(sdpa_block_rescale(-INFINITY, mb), 0.f, ts);
        if (lane == 0) S.l_s[g] = l;
    }
    ts(2);
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
                        const float p1 = S.pbf[g][k0 + j + 1];
                        t0 = fmaf(p1, bf_lo(vw[j + 1]), t0);
                        t1 = fmaf(p1, bf_hi(vw[j + 1]), t1);
                    }
                    const float p0 = S.pbf[g][k0 + j];
                    t0 = fmaf(p0, bf_lo(vw[j]), t0);
                    t1 = fmaf(p0, bf_hi(vw[j]), t1);
                }
            }
            S.tmp[gl][g][2 * dp] = t0;
            S.tmp[gl][g][2 * dp + 1] = t1;
        }
    }
    __syncthreads();
    if (tid < G * DZ) {
        const int fg = tid / DZ, fd = tid % DZ;
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < NG8; ++u)
            if (u < ngrp) acc = __fadd_rn(acc, S.tmp[u][fg][fd]);
        const int col = (kvh * G + fg) * D + z * DZ + fd;
        const bf16_t o = f2bf(__fmul_rn(acc, __fdiv_rn(1.0f, S.l_s[fg])));
        a.att[(long)qi * XL_QD + col] = o;   // row-major copy (not read in this launch)
        const __amdgpu_buffer_rsrc_t orr = xl_rsrc(a.att16, (uint32_t)(16 * XL_QD * 2));
        __builtin_amdgcn_raw_buffer_store_b16(o, orr, (int)(x16_off(qi, col, XL_QD / 32) * 2), 0, XL_AUX_SC1);
    }
    __syncthreads();   // the LDS scratch is reused by the next task
    ts(3);
}

// contiguous run [lo, hi) of n items over `workers` workers (worker w)
__device__ __forceinline__ void xl_run(int n, int workers, int w, int& lo, int& hi) {
    const int base = n / workers, extra = n - base * workers;
    lo = w * base + min(w, extra);
    hi = lo + base + (w < extra ? 1 : 0);
}
// G and D tasks of worker w (a G task is one 72-chunk pass, a D task two), so that no worker
// runs more than 7 passes and the workers with two D tasks are off the critical path: the
// xd = nd - nw "light" workers run 3 G tasks of K part 0 and then 2 D tasks of part 0 (ready
// once every part-0 G task is done, which every worker runs first); the other "heavy" workers
// run 2-3 part-0 G tasks, then 2-3 part-1 G tasks, then one D task. Before: both runs put
// their extra tasks on the same low workers (9 passes; D end 90.7 us against 82.6 median).
// Requires nw <= nd <= 2 nw (checked by xlayer_launch through nb >= 144 + M).
struct XlGdRuns {
    int g0_lo, n0, g1_lo, n1, d_lo, nd;   // part-0 G run, part-1 G run (groups), D task run
};
__device__ __forceinline__ XlGdRuns xl_gd_runs(int ng, int ntd, int nw, int w) {
    const int half = ng / 2, xd = ntd - nw, H = nw - xd;
    XlGdRuns r;
    if (w < xd) {
        r = XlGdRuns{3 * w, 3, half, 0, 2 * w, 2};
    } else {
        const int h = w - xd;
        const int e0 = half - 3 * xd - 2 * H;             // heavy workers with 3 part-0 tasks
        const int b1 = half / H, e1 = half - b1 * H;      // part-1 base count, extras
        const int e1a = min(e1, H - e0), e1b = e1 - e1a;  // extras on the 2-part-0 workers, then on the first
        r.n0 = 2 + (h < e0 ? 1 : 0);
        r.g0_lo = 3 * xd + 2 * h + min(h, e0);
        r.n1 = b1 + ((h >= e0 && h - e0 < e1a) || h < e1b ? 1 : 0);
        r.g1_lo = half + b1 * h + min(h, e1b) + max(0, min(h - e0, e1a));
        r.d_lo = 2 * xd + h;
        r.nd = 1;
    }
    return r;
}

// ---------------------------------------------------------------- the launch
// LDS: the X window (aliased, outside the GEMV stages, by the norms' sum-of-squares scratch
// and the cross attention's), the two chunk-sum buffers, the norm workgroup's h row
constexpr size_t XL_LDS_XS = (size_t)XL_XWIN * 32 * 16;
constexpr size_t XL_LDS_CS = (size_t)XL_SC * XL_EL * 4;
constexpr size_t XL_LDS_SQ = (size_t)(XL_D + 64) * 4;
constexpr size_t XL_LDS_H = (size_t)XL_D * 2;
constexpr size_t XL_LDS = XL_LDS_XS + 2 * XL_LDS_CS + XL_LDS_H;
static_assert(XL_LDS_SQ <= XL_LDS_XS && sizeof(XlAttnLds) <= XL_LDS_XS, "aliases of the X window");
static_assert(XL_LDS <= 160 * 1024, "LDS of one CU");

template <bool HAS_QKV>
__global__ __launch_bounds__(XL_NW * 64) void xlayer_kernel(XLayerArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const XlGemvLds gl{(u32x4*)smem, (float*)(smem + XL_LDS_XS), (float*)(smem + XL_LDS_XS + XL_LDS_CS)};
    float* sq = (float*)smem;
    u32x4* hrow = (u32x4*)(smem + XL_LDS_XS + 2 * XL_LDS_CS);
    XlAttnLds& al = *(XlAttnLds*)smem;
    const int bu = (int)blockIdx.x, nb = (int)gridDim.x, tid = (int)threadIdx.x;
    const int M = a.M, d = XL_D;
    unsigned* set = a.sync;
    unsigned* tmo = a.timeout;
    if (bu == 0 && tid < XL_SET_LINES)
        __hip_atomic_store(a.sync_next + tid * FM_LINE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int nrow = bu - (nb - M);             // the last M workgroups run the norms
    const bool normwg = nrow >= 0;
    const int nw = nb - M;                      // workers of the G and D stages
    auto none = [] {};
    XL_TS(0);

    // ---- O1: o-projection of the self attention (K = q_dim: 64 chunks), groups 0..143
    if (bu < d / 16) {
        const XlGemv s{a.Wo, XL_QD / 32, xl_rsrc(a.att16_self, 16u * XL_QD * 2u), d, M,
                       xl_rsrc(a.tmp, (uint32_t)(M * d * 2)), xl_rsrc(nullptr, 0u), false, XL_QD / 32};
        xl_gemv<EPI_BF16, false>(s, bu, bu + 1, [&](int g) { return XlTask{g, 0, XL_QD / 32, 0, 0, true, true}; }, gl, none);
        xl_publish(set, XC_O1 + (bu & 7), 1u);
        XL_TS(1);
    }
    // ---- N1 (norm workgroups)
    if (normwg) {
        xl_norm_row<0>(
            a, nrow, a.n1_post, a.n1_pre, hrow, true, false, sq,
            [&] {
                xl_wait_wg<8>(set, XC_O1, (unsigned)(d / 16), tmo, 21u);
                XL_TS(19);
            },
            [&](int k) { XL_TS(20 + k); });
        xl_publish(set, XC_N1, 1u);
        XL_TS(2);
    }
    // ---- Q: cross-q (128 groups); published per kv head (32 groups: its two q heads)
    if (bu < XL_QD / 16) {
        static_assert(XL_DOWN_KBC % 2 == 0 && XL_DOWN_KBC / 2 <= XL_SC, "down passes");
        const XlGemv s{a.Wq, d / 32, xl_rsrc(a.xn16, 16u * d * 2u), XL_QD, M, xl_rsrc(a.q, (uint32_t)(M * XL_QD * 2)),
                       xl_rsrc(nullptr, 0u), false, d / 32};
        xl_gemv<EPI_BF16, false>(s, bu, bu + 1, [&](int g) { return XlTask{g, 0, d / 32, 0, 0, true, true}; }, gl,
                                 [&] {
                                     xl_wait_wg<1>(set, XC_N1, (unsigned)M, tmo, 22u);
                                     XL_TS(3);
                                 });
        xl_publish(set, XC_Q + bu / 32, 1u);
        XL_TS(4);
    }
    // ---- A: PM cross attention, task t = (row, kv head, 32-dim slice), row fastest
    {
        const int ntask = M * XL_HKV * (XL_HD / 32);
        int done = 0;
        for (int t = bu; t < ntask; t += nb) {
            const int qi = t % M, kvh = (t / M) % XL_HKV, z = t / (M * XL_HKV);
            xl_cross_attn(
                a, qi, kvh, z, al,
                [&] {
                    xl_wait_wg<1>(set, XC_Q + kvh, 32u, tmo, 23u);
                    XL_TS(5);
                },
                [&](int k) { XL_TS(24 + k); });
            ++done;
        }
        if (done) xl_publish(set, XC_A + (bu & 7), (unsigned)done);
        XL_TS(6);
    }
    // ---- O: cross-o (K = q_dim), groups 0..143
    if (bu < d / 16) {
        const XlGemv s{a.Wco, XL_QD / 32, xl_rsrc(a.att16, 16u * XL_QD * 2u), d, M,
                       xl_rsrc(a.tmp, (uint32_t)(M * d * 2)), xl_rsrc(nullptr, 0u), false, XL_QD / 32};
        const unsigned nA = (unsigned)(M * XL_HKV * (XL_HD / 32));
        xl_gemv<EPI_BF16, false>(s, bu, bu + 1, [&](int g) { return XlTask{g, 0, XL_QD / 32, 0, 0, true, true}; }, gl,
                                 [&] {
                                     xl_wait_wg<8>(set, XC_A, nA, tmo, 24u);
                                     XL_TS(7);
                                 });
        xl_publish(set, XC_O + (bu & 7), 1u);
        XL_TS(8);
    }
    // ---- N2
    if (normwg) {
        xl_norm_row<0>(a, nrow, a.n2_post, a.n2_pre, hrow, false, false, sq, [&] {
            xl_wait_wg<8>(set, XC_O, (unsigned)(d / 16), tmo, 25u);
            XL_TS(9);
        });
        xl_publish(set, XC_N2, 1u);
        XL_TS(10);
    }
    // ---- G: gate/up + GeGLU, contiguous runs of the 1 152 groups over the nw workers;
    // arrivals counted per down K part (groups [0, 576) hold the act features of part 0)
    const int ngu = 2 * XL_F / 16, half = ngu / 2;
    const int ngd = d / 16, ntd = 2 * ngd;
    const XlGdRuns gd = xl_gd_runs(ngu, ntd, nw, bu);
    if (!normwg) {
        const int ngt = gd.n0 + gd.n1;
        const XlGemv s{a.Wgu, d / 32, xl_rsrc(a.xn16, 16u * d * 2u), 2 * XL_F, M, xl_rsrc(a.act16, 16u * XL_F * 2u),
                       xl_rsrc(nullptr, 0u), true, d / 32};
        // part 0's arrivals are published as soon as the worker's part-0 tasks are stored (the
        // down tasks of part 0 wait on those only), part 1's at the end
        const bool early0 = gd.n1 > 0;
        xl_gemv<EPI_GEGLU, false>(
            s, 0, ngt,
            [&](int i) { return XlTask{i < gd.n0 ? gd.g0_lo + i : gd.g1_lo + (i - gd.n0), 0, d / 32, 0, 0, true, true}; },
            gl,
                                  [&] {
                                      xl_wait_wg<1>(set, XC_N2, (unsigned)M, tmo, 26u);
                                      XL_TS(11);
                                  },
                                  [&](int i) {
                                      if (early0 && i == gd.n0 - 1) {
                                          xl_drain();
                                          __syncthreads();
                                          if (tid == 0)
                                              __hip_atomic_fetch_add(xline(set, XC_G0 + (bu & 7)), (unsigned)gd.n0,
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                      }
                                  });
        const int n0 = early0 ? 0 : gd.n0, n1 = gd.n1;
        xl_drain();
        __syncthreads();
        if (tid == 0) {
            if (n0) __hip_atomic_fetch_add(xline(set, XC_G0 + (bu & 7)), (unsigned)n0, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
            if (n1) __hip_atomic_fetch_add(xline(set, XC_G1 + (bu & 7)), (unsigned)n1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        }
        XL_TS(12);
    }
    // ---- D: down in the reference's two K parts, task t = part * 144 + group
    if (!normwg) {
        const int lo = gd.d_lo, hi = gd.d_lo + gd.nd;   // tasks (part, group); two passes of 72 chunks each
        const XlGemv s{a.Wd, XL_F / 32, xl_rsrc(a.act16, 16u * XL_F * 2u), d, M, xl_rsrc(nullptr, 0u),
                       xl_rsrc(a.dpart, (uint32_t)(2 * M * d * 4)), false, XL_DOWN_KBC};
        const bool need0 = lo < ngd && hi > lo, need1 = hi > ngd;
        xl_gemv<EPI_F32, true>(
            s, 2 * lo, 2 * hi,
            [&](int i) {
                const int t = i >> 1, sub = i & 1, p = t / ngd;
                const int k0 = p * XL_DOWN_KBC + sub * (XL_DOWN_KBC / 2);
                return XlTask{t - p * ngd, k0, k0 + XL_DOWN_KBC / 2, p, p * XL_DOWN_KBC, sub == 0, sub == 1};
            },
            gl, [&] {
                if (threadIdx.x < 64) {
                    if (need0) (void)xl_wait<8>(set, XC_G0, (unsigned)half, tmo, 27u);
                    if (need1) (void)xl_wait<8>(set, XC_G1, (unsigned)(ngu - half), tmo, 28u);
                }
                xl_barrier();
                XL_TS(13);
            });
        if (hi > lo) xl_publish(set, XC_D + (bu & 7), (unsigned)(hi - lo));
        XL_TS(14);
    }
    // ---- N3: from the parts; h back to HBM
    if (normwg) {
        xl_norm_row<2>(a, nrow, a.n3_post, a.n3_pre, hrow, false, true, sq, [&] {
            xl_wait_wg<8>(set, XC_D, (unsigned)ntd, tmo, 29u);
            XL_TS(15);
        });
        xl_publish(set, XC_N3, 1u);
        XL_TS(16);
    }
    // ---- QKV: the next layer's q|k|v, 256 groups over all workgroups (read by the next launch)
    if constexpr (HAS_QKV) {
        int lo, hi;
        xl_run(a.qkv_dim / 16, nb, bu, lo, hi);
        const XlGemv s{a.Wqkv, d / 32, xl_rsrc(a.xn16, 16u * d * 2u), a.qkv_dim, M,
                       xl_rsrc(a.qkv, (uint32_t)(M * a.qkv_dim * 2)), xl_rsrc(nullptr, 0u), false, d / 32};
        xl_gemv<EPI_BF16, false>(s, lo, hi, [&](int g) { return XlTask{g, 0, d / 32, 0, 0, true, true}; }, gl,
                                 [&] {
                                     xl_wait_wg<1>(set, XC_N3, (unsigned)M, tmo, 30u);
                                     XL_TS(17);
                                 });
        XL_TS(18);
    }
}

int xlayer_launch(const XLayerArgs& a, hipStream_t st) {
    if (a.M < 1 || a.M > 8 || !a.sync || !a.sync_next || !a.timeout) return -1;
    const int dev = t5g_cur_device();
    if (dev < 0) return -1;
    static int ncu[T5G_MAX_DEVICES] = {};
    static bool ok[T5G_MAX_DEVICES][2] = {};
    if (!ncu[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return -1;
        ncu[dev] = v;
    }
    // one workgroup per CU, every one resident at once (the hand-offs wait on each other)
    const int nb = ncu[dev] < 256 ? ncu[dev] : 256;
    if (nb < XL_D / 16 + a.M || nb < XL_QD / 16) return -1;
    auto k = a.Wqkv ? xlayer_kernel<true> : xlayer_kernel<false>;
    if (!ok[dev][a.Wqkv ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)XL_LDS);
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, XL_NW * 64, XL_LDS) != hipSuccess || occ < 1)
            return -1;
        ok[dev][a.Wqkv ? 1 : 0] = true;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)nb), dim3(XL_NW * 64), XL_LDS, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

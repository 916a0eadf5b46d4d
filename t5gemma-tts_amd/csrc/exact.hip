// Exact-order kernels: the engine's parity mode (t5g_engine_set_exact).
//
// The reference runs inference_tts on CPU in bf16 (inference_commandline_hf.py:102-106,
// hf_export/modeling_t5gemma_voice.py:565-862). Its logits depend on the ORDER in which
// torch 2.10's CPU kernels accumulate fp32 sums. Those orders were measured in the build
// container -- the machine the golden vectors were made on -- with absorption probes
// (a partial sum of 2^25 swallows small terms, so which terms vanish reveals the tree;
// tools/cpu_order/*) and then confirmed bit for bit on random data and on the reference's
// own full-model runs. The kernels here compute every sum in that order,
// in plain fp32 VALU arithmetic (products of two bf16 values are exact in fp32, so an
// fma and a separate multiply-add give the same bits):
//
// * Linear (F.linear -> oneDNN AMX matmul): per output, each 32-element chunk of K sums
//   its even-k and odd-k products in two sequential chains; chunk sum = E + O; chunk sums
//   fold sequentially into a part; K is cut into parts of Kb elements (Kb depends on the
//   call's row count M, N, K and the thread count: ref_ksplit.h), parts fold in order;
//   bias is added last.
// * SDPA (aten cpu_flash_attention, bf16): q.k and P.V per the GEMM kernel aten picks:
//   - a q block of one row without packing: oneDNN gemv. q.k = 16 lane accumulators,
//     lane l takes the pair (2l, 2l+1) of every 32-element chunk, odd product first
//     (VDPBF16PS), then lanes l + l^8, adjacent pairs, adjacent pairs, last pair (hadd
//     tree). P.V = groups of 8 keys: a fresh pair-ordered chain per group, added to the
//     output accumulator.
//   - otherwise the E/O chunk model of the Linear, q.k over 32-element chunks of the head
//     dim, P.V over chunks of 32 keys (+ tail) without packing, or over chunks of the
//     largest even divisor <= 32 of the (even-padded) block length when aten packs
//     (need_pack: kv and q lengths >= 64 and a per-thread work ratio >= 4).
//   - later kv blocks accumulate onto the rescaled output (beta = 1 GEMM).
//   The softmax pieces (fast exp, lane-ordered block sums, rescale) are common.h sdpa_*.
// * RMSNorm's mean (aten SumKernel.cpp, AVX2 kernel: no AVX-512 variant is registered):
//   norm.hip resid_norm_kernel<..., EXACT>.
// * GELU: exact_math.h (tanh form) and a 65,536-entry bf16 table for the erf form (the
//   reference host computes it with oneDNN's eltwise kernel).
#include "common.h"
#include "exact_math.h"
#include "t5g_kernels.h"

namespace t5g {

#ifdef T5G_DBG_TS
// diagnostic build only: per (query, head) the scaled scores and bf16 p of every key
__device__ float* t5g_dbg_exact_buf;
extern "C" int t5g_dbg_set_exact(void* p) {
    return hipMemcpyToSymbol(HIP_SYMBOL(t5g_dbg_exact_buf), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#define XA_DBG(slot, key, val)                                                                           \
    do {                                                                                                 \
        if (t5g_dbg_exact_buf) t5g_dbg_exact_buf[(((long)qi * a.Hq + h) * 4 + (slot)) * 4096 + (key)] = (val); \
    } while (0)
#else
#define XA_DBG(slot, key, val) do { } while (0)
#endif

// ---------------------------------------------------------------------------------
// Linear. Workgroup = 64 output rows (4 P16 row groups, one per lane) x RT rows of X,
// NW waves. Stage s: wave w computes chunk s*NW + w for all RT rows (X read through
// the scalar cache: its address is wave-uniform) and stores the chunk sums in LDS; after
// the barrier wave r folds row r's chunk sums of the stage, in chunk order. Two LDS
// buffers let stage s+1's chunks be computed while stage s is folded.
// Epilogue of output (row m, packed column n = g*16 + r16); y = the folded fp32 sum.
// Called by whole waves (GEGLU pairs lanes r16 and r16 + 8).
template <int EPI>
__device__ __forceinline__ void exact_lin_store(const ExactLinArgs& a, int m, int g, int r16, int n, float y) {
    if constexpr (EPI == EPI_GEGLU) {
        // rows g*16 + 0..7 gate, + 8..15 up of features g*8 + 0..7 (engine.py interleave)
        const float other = xlane<8>(y);
        if (m < a.M && r16 < 8) {
            const int f = g * 8 + r16;
            if (f < a.N / 2) {
                const float gate = rbf(t5g_exact::gelu_tanh(rbf(y)));
                ((bf16_t*)a.Y)[(long)m * a.ldy + f] = f2bf(__fmul_rn(gate, rbf(other)));
            }
        }
        return;
    }
    if (m >= a.M || n >= a.N) return;
    if constexpr (EPI == EPI_F32) {
        ((float*)a.Y)[(long)m * a.ldy + n] = y;
    } else if constexpr (EPI == EPI_BF16) {
        ((bf16_t*)a.Y)[(long)m * a.ldy + n] = f2bf(y);
    } else if constexpr (EPI == EPI_BIAS_BF16) {
        ((bf16_t*)a.Y)[(long)m * a.ldy + n] = f2bf(__fadd_rn(y, bf2f(a.bias[n])));
    } else {   // EPI_BIAS_GELU: nn.GELU() (erf) on the bf16 Linear output
        const bf16_t h = f2bf(__fadd_rn(y, bf2f(a.bias[n])));
        ((bf16_t*)a.Y)[(long)m * a.ldy + n] = a.gelu_lut ? a.gelu_lut[h] : f2bf(t5g_exact::gelu_erf(bf2f(h)));
    }
}

// The K-split chunk size (32-element chunks per part) of row m for packed column n.
__device__ __forceinline__ int exact_lin_kbc(const ExactLinArgs& a, int m, int n) {
    if (a.kb_fixed > 0) return a.kb_fixed;
    const int mu = a.row_len ? a.row_len[a.tok_row ? a.tok_row[m] : m] : 1;
    const uint16_t* tab = (a.kb_b && n >= a.nsplit_col) ? a.kb_b : a.kb_a;
    int kbc = tab ? tab[min(max(mu, 1), a.kb_len) - 1] : a.KB;
    return kbc <= 0 ? a.KB : kbc;
}

// One 32-element chunk sum (even chain + odd chain) of X row xr against the lane's
// unpacked weight chunk wf.
__device__ __forceinline__ float exact_chunk(const uint32_t* xr, const float* wf) {
    float e = 0.f, o = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t xw = xr[i];
        e = fmaf(bf_lo(xw), wf[2 * i], e);
        o = fmaf(bf_hi(xw), wf[2 * i + 1], o);
    }
    return __fadd_rn(e, o);
}

// exact_chunk with X's chunk read through vector loads (lanes of a wave on different chunks)
__device__ __forceinline__ float exact_chunk_v(const u32x4* xr4, const float* wf) {
    u32x4 xv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) xv[j] = xr4[j];
    float e = 0.f, o = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t xw = xv[i >> 2][i & 3];
        e = fmaf(bf_lo(xw), wf[2 * i], e);
        o = fmaf(bf_hi(xw), wf[2 * i + 1], o);
    }
    return __fadd_rn(e, o);
}

// exact_chunk_v on X words already in registers
__device__ __forceinline__ float exact_chunk_x(const u32x4 (&xv)[4], const float* wf) {
    float e = 0.f, o = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t xw = xv[i >> 2][i & 3];
        e = fmaf(bf_lo(xw), wf[2 * i], e);
        o = fmaf(bf_hi(xw), wf[2 * i + 1], o);
    }
    return __fadd_rn(e, o);
}

__device__ __forceinline__ void exact_load_chunk(const bf16_t* wg, int kb, int r16, float* wf) {
    u32x4 wv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wv[j] = *(const u32x4*)(wg + ((long)kb * 64 + j * 16 + r16) * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            wf[8 * j + 2 * q] = bf_lo(wv[j][q]);
            wf[8 * j + 2 * q + 1] = bf_hi(wv[j][q]);
        }
}

template <int RT, int NW, int EPI>
__global__ __launch_bounds__(NW * 64) void exact_linear_kernel(ExactLinArgs a) {
    static_assert(RT <= NW, "every folded row needs a wave");
    __shared__ float cs[2][RT][NW][64];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = blockIdx.x * 4 + (lane >> 4);
    const int r16 = lane & 15;
    const int n = blockIdx.x * 64 + lane;       // packed output row
    const int m0 = blockIdx.y * RT;
    const int KB = a.KB;
    const bf16_t* wg = a.W + (long)g * KB * 512;
    // fold state of row m0 + w (waves < RT)
    float tot = 0.f, part = 0.f;
    int kbc = KB;
    if (w < RT) kbc = exact_lin_kbc(a, min(m0 + w, a.M - 1), n);
    const int nst = (KB + NW - 1) / NW;
    for (int s = 0; s < nst; ++s) {
        const int kb = s * NW + w;
        if (kb < KB) {
            float wf[32];
            exact_load_chunk(wg, kb, r16, wf);
#pragma unroll
            for (int r = 0; r < RT; ++r) {
                const int m = min(m0 + r, a.M - 1);
                cs[s & 1][r][w][lane] = exact_chunk((const uint32_t*)(a.X + (long)m * a.ldx + kb * 32), wf);
            }
        }
        __syncthreads();
        if (w < RT) {
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int kb2 = s * NW + i;
                if (kb2 < KB) {
                    const float c = cs[s & 1][w][i][lane];
                    if (kb2 % kbc == 0) {
                        if (kb2 > 0) tot = __fadd_rn(tot, part);
                        part = __fadd_rn(0.f, c);
                    } else {
                        part = __fadd_rn(part, c);
                    }
                }
            }
        }
    }
    if (w >= RT) return;
    exact_lin_store<EPI>(a, m0 + w, g, r16, n, KB > kbc ? __fadd_rn(tot, part) : part);
}

template <int RT>
static int launch_exact_linear(const ExactLinArgs& a, int epi, hipStream_t st) {
    constexpr int NW = 8;
    const dim3 grid((unsigned)(a.NG / 4), (unsigned)((a.M + RT - 1) / RT)), blk(NW * 64);
    switch (epi) {
        case EPI_F32: hipLaunchKernelGGL((exact_linear_kernel<RT, NW, EPI_F32>), grid, blk, 0, st, a); break;
        case EPI_BF16: hipLaunchKernelGGL((exact_linear_kernel<RT, NW, EPI_BF16>), grid, blk, 0, st, a); break;
        case EPI_BIAS_BF16: hipLaunchKernelGGL((exact_linear_kernel<RT, NW, EPI_BIAS_BF16>), grid, blk, 0, st, a); break;
        case EPI_BIAS_GELU: hipLaunchKernelGGL((exact_linear_kernel<RT, NW, EPI_BIAS_GELU>), grid, blk, 0, st, a); break;
        case EPI_GEGLU: hipLaunchKernelGGL((exact_linear_kernel<RT, NW, EPI_GEGLU>), grid, blk, 0, st, a); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}


// Decode-size launches (M <= 8 rows): one workgroup per 16-row group g of W (16 output
// columns; 64-column tiles would leave most of the chip idle), 16 waves. A stage covers
// 64 chunks: wave w computes chunks 4w + (lane >> 4) for column lane & 15 and RT rows of
// X; after the barrier thread (row tid >> 4, column tid & 15) folds the stage's chunk sums
// of its row in chunk order -- the same order and arithmetic as exact_linear_kernel.
template <int RT, int EPI>
__global__ __launch_bounds__(1024) void exact_linear_g16_kernel(ExactLinArgs a) {
    constexpr int SC = 64, SP = SC + 4;   // chunks per stage; padded LDS row (16-byte aligned)
    __shared__ __attribute__((aligned(16))) float cs[2][RT][16][SP];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = blockIdx.x, r16 = lane & 15, q = lane >> 4;
    const int KB = a.KB;
    const bf16_t* wg = a.W + (long)g * KB * 512;
    const int fr = tid >> 4, fc = tid & 15;   // fold row / column (threads < RT * 16)
    const bool folder = tid < RT * 16;
    float tot = 0.f, part = 0.f;
    int kbc = KB;
    if (folder) kbc = exact_lin_kbc(a, min(fr, a.M - 1), g * 16 + fc);
    int nb = 0;   // next K part boundary (chunk index)
    const int nst = (KB + SC - 1) / SC;
    // this lane's weight chunk of the current stage, loaded one stage ahead; at 1-2 rows
    // (batch-1 / batch-2 decode) the X chunks too, so a stage never waits for a load
    constexpr bool XPRE = RT <= 2;
    u32x4 wv[4];
    u32x4 xq[XPRE ? RT : 1][4];
    auto load = [&](int kb) {
        if (kb < KB) {
#pragma unroll
            for (int j = 0; j < 4; ++j) wv[j] = *(const u32x4*)(wg + ((long)kb * 64 + j * 16 + r16) * 8);
            if constexpr (XPRE) {
#pragma unroll
                for (int r = 0; r < RT; ++r) {
                    const u32x4* xr4 = (const u32x4*)(a.X + (long)min(r, a.M - 1) * a.ldx + kb * 32);
#pragma unroll
                    for (int j = 0; j < 4; ++j) xq[r][j] = xr4[j];
                }
            }
        }
    };
    load(w * 4 + q);
    for (int s = 0; s < nst; ++s) {
        const int kb = s * SC + w * 4 + q;
        if (kb < KB) {
            float wf[32];
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    wf[8 * j + 2 * i] = bf_lo(wv[j][i]);
                    wf[8 * j + 2 * i + 1] = bf_hi(wv[j][i]);
                }
#pragma unroll
            for (int r = 0; r < RT; ++r) {
                const int m = min(r, a.M - 1);
                if constexpr (XPRE) cs[s & 1][r][r16][w * 4 + q] = exact_chunk_x(xq[r], wf);
                else cs[s & 1][r][r16][w * 4 + q] = exact_chunk_v((const u32x4*)(a.X + (long)m * a.ldx + kb * 32), wf);
            }
        }
        load(kb + SC);
        __syncthreads();
        if (folder) {
            const int kn = min(SC, KB - s * SC);
            float c[SC];
#pragma unroll
            for (int i = 0; i < SC; i += 4) *(float4*)&c[i] = *(const float4*)&cs[s & 1][fr][fc][i];
#pragma unroll
            for (int i = 0; i < SC; ++i) {
                const int kb2 = s * SC + i;
                if (i < kn) {
                    if (kb2 == nb) {   // a K part starts (multiples of kbc)
                        if (kb2 > 0) tot = __fadd_rn(tot, part);
                        part = __fadd_rn(0.f, c[i]);
                        nb += kbc;
                    } else {
                        part = __fadd_rn(part, c[i]);
                    }
                }
            }
        }
    }
    if (w * 64 >= RT * 16) return;   // whole waves: GEGLU pairs lanes fc and fc ^ 8
    exact_lin_store<EPI>(a, fr, g, fc, g * 16 + fc, KB > kbc ? __fadd_rn(tot, part) : part);
}

template <int RT>
static int launch_exact_linear_g16(const ExactLinArgs& a, int epi, hipStream_t st) {
    const dim3 grid((unsigned)a.NG), blk(1024);
    switch (epi) {
        case EPI_F32: hipLaunchKernelGGL((exact_linear_g16_kernel<RT, EPI_F32>), grid, blk, 0, st, a); break;
        case EPI_BF16: hipLaunchKernelGGL((exact_linear_g16_kernel<RT, EPI_BF16>), grid, blk, 0, st, a); break;
        case EPI_BIAS_BF16: hipLaunchKernelGGL((exact_linear_g16_kernel<RT, EPI_BIAS_BF16>), grid, blk, 0, st, a); break;
        case EPI_BIAS_GELU: hipLaunchKernelGGL((exact_linear_g16_kernel<RT, EPI_BIAS_GELU>), grid, blk, 0, st, a); break;
        case EPI_GEGLU: hipLaunchKernelGGL((exact_linear_g16_kernel<RT, EPI_GEGLU>), grid, blk, 0, st, a); break;
        default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

int exact_linear(const ExactLinArgs& a, int epi, hipStream_t st) {
    if (a.M <= 0) return 0;
    if (!a.X || !a.W || !a.Y || a.N <= 0 || a.KB <= 0 || a.NG % 4) return -1;
    if ((epi == EPI_BIAS_BF16 || epi == EPI_BIAS_GELU) && !a.bias) return -1;
    if (epi == EPI_GEGLU && a.N % 16) return -1;
    // rows per tile: the batch of a decode step (1..8 rows) without idle rows; 8 beyond
    // decode rows whose 64-column tiles cannot fill the chip: 16-column workgroups
    if (a.M <= 8 && a.NG / 4 < 256) switch (a.M) {
        case 1: return launch_exact_linear_g16<1>(a, epi, st);
        case 2: return launch_exact_linear_g16<2>(a, epi, st);
        case 3: case 4: return launch_exact_linear_g16<4>(a, epi, st);
        case 5: case 6: case 7: case 8: return launch_exact_linear_g16<8>(a, epi, st);
        default: break;
    }
    if (a.M <= 1) return launch_exact_linear<1>(a, epi, st);
    if (a.M <= 2) return launch_exact_linear<2>(a, epi, st);
    if (a.M <= 4) return launch_exact_linear<4>(a, epi, st);
    return launch_exact_linear<8>(a, epi, st);
}

// ---------------------------------------------------------------------------------
// SDPA. One workgroup per (query token, query head, 32-dim output slice), 256 threads.
// Keys of one 512-key block at a time: scores (thread per key, repeated by every slice),
// softmax pieces (wave 0), P.V (8 threads per output dim on chunk sums, one folds).
constexpr int XA_BLOCK = 512;
constexpr int XA_MAXD = 256;

__device__ __forceinline__ int xa_even_div_chunk(int K) {
    const int Ke = K + (K & 1);
    for (int c = 32; c > 2; c -= 2)
        if (Ke % c == 0) return c;
    return 2;
}

// aten cpu_flash_attention's `need_pack` (reduced floating types): pack the V / K blocks
// for the AMX brgemm when both lengths are >= 64 and the per-thread GEMM work is at least
// 4x the packing work (batch 1, num_head = query heads).
__device__ __forceinline__ bool xa_need_pack(int Tq, int Tk, int Hq, int D, int threads, bool causal) {
    if (!(Tk >= 64 && Tq >= 64)) return false;
    const int qs = sdpa_qsplit(Tq);
    const long q_slice = (Tq + qs - 1) / qs;
    const double pack_size = (double)Hq * Tk * D;
    const long qs_per_thread = ((long)Hq * q_slice + threads - 1) / threads;
    const double gemm = (double)qs_per_thread * qs * (causal ? Tq : Tk) * D;
    return gemm / pack_size >= 4.0;
}

constexpr int XA_DS = 32;               // output dims per workgroup (blockIdx.z slices)
constexpr int XA_PARTS = 256 / XA_DS;   // threads per dim in P.V

__global__ __launch_bounds__(256) void exact_attn_kernel(ExactAttnArgs a) {
    __shared__ float qs_[XA_MAXD];
    __shared__ float sp[XA_BLOCK + 16];   // scores, then bf16-rounded p of the block
    __shared__ float csum[XA_BLOCK / 2 * XA_DS];   // P.V chunk sums [chunk][dim] (chunks >= 2 keys)
    __shared__ float bsum;
    const int qi = blockIdx.x, h = blockIdx.y;
    const int d0 = blockIdx.z * XA_DS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int D = a.D;
    const int row = a.q_row ? a.q_row[qi] : qi;
    const int Tk_all = a.kv_len[row];
    const int Tq = a.q_len ? a.q_len[row] : 1;
    const int tq = a.q_pos ? a.q_pos[qi] : Tq - 1;
    const int abs_t = tq + (Tk_all - Tq);          // the query's own key position
    // explicit mask (sliding-window layer long enough for it) vs is_causal
    const bool has_mask = a.window > 0 && Tk_all >= a.window;
    int lo = 0;
    if (has_mask && Tq == 1 && a.causal) lo = Tk_all - a.window;   // DynamicSlidingWindowLayer
    const int Tk = Tk_all - lo;                    // keys of the call
    const bool sdpa_causal = a.causal && !has_mask && Tq > 1;
    const int qsz = sdpa_qsplit(Tq);
    const int qb0 = tq - tq % qsz;
    const int mblk = min(qsz, Tq - qb0);
    const int nk = sdpa_causal ? min(qb0 + mblk + (Tk_all - Tq), Tk) : Tk;
    const bool pack = xa_need_pack(Tq, Tk, a.Hq, D, a.threads, sdpa_causal);
    const bool gemv = mblk == 1 && !pack;
    const int kvh = h / (a.Hq / a.Hkv);
    const bf16_t* Kb = a.K + row * a.kv_bstride + kvh * a.kv_hstride + (long)lo * D;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride + (long)lo * D;
    for (int d = tid; d < D; d += 256) qs_[d] = bf2f(a.Q[(long)qi * a.ldq + h * D + d]);
    __syncthreads();

    float m = -INFINITY, l = 0.f, dst = 0.f;
    for (int bs = 0; bs < nk; bs += XA_BLOCK) {
        const int blen = min(XA_BLOCK, Tk - bs);
        // ---- scores of the block (masked keys -inf)
        if (gemv && !has_mask && !sdpa_causal) {
            // decode rows (one query, no mask): both of this thread's keys' rows requested
            // before either dot product (the loop below would wait for each in turn)
            u32x4 kv2[2][XA_MAXD / 8];
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const int kk = tid + 256 * r2;
                const bf16_t* kr = Kb + (long)(bs + (kk < blen && bs + kk < nk ? kk : 0)) * D;
#pragma unroll
                for (int j = 0; j < XA_MAXD / 8; ++j)
                    kv2[r2][j] = j * 8 < D ? *(const u32x4*)(kr + 8 * j) : (u32x4){0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int r2 = 0; r2 < 2; ++r2) {
                const int kk = tid + 256 * r2;
                if (kk < blen) {
                    float s = -INFINITY;
                    if (bs + kk < nk) {
                        float acc[16];
#pragma unroll
                        for (int l2 = 0; l2 < 16; ++l2) acc[l2] = 0.f;
#pragma unroll
                        for (int cb = 0; cb < XA_MAXD / 32; ++cb) {
                            if (cb * 32 < D) {
                                const int c = cb * 32;
#pragma unroll
                                for (int l2 = 0; l2 < 16; ++l2) {
                                    const uint32_t kw = kv2[r2][cb * 4 + (l2 >> 2)][l2 & 3];
                                    acc[l2] = fmaf(qs_[c + 2 * l2 + 1], bf_hi(kw), acc[l2]);
                                    acc[l2] = fmaf(qs_[c + 2 * l2], bf_lo(kw), acc[l2]);
                                }
                            }
                        }
                        float v8[8], v4[4];
#pragma unroll
                        for (int l2 = 0; l2 < 8; ++l2) v8[l2] = __fadd_rn(acc[l2], acc[l2 + 8]);
#pragma unroll
                        for (int l2 = 0; l2 < 4; ++l2) v4[l2] = __fadd_rn(v8[2 * l2], v8[2 * l2 + 1]);
                        s = __fmul_rn(__fadd_rn(__fadd_rn(v4[0], v4[1]), __fadd_rn(v4[2], v4[3])), a.scale);
                    }
                    sp[kk] = s;
                    XA_DBG(0, bs + kk, s);
                }
            }
        }
        for (int kk = tid; !(gemv && !has_mask && !sdpa_causal) && kk < blen; kk += 256) {
            const int key = bs + kk;               // index into the call's keys
            const int kabs = key + lo;
            bool vis;
            if (has_mask) {
                if (Tq == 1 && a.causal) vis = true;
                else if (a.causal) vis = kabs <= abs_t && kabs > abs_t - a.window;
                else vis = abs(abs_t - kabs) <= a.window;
            } else {
                vis = !sdpa_causal || kabs <= abs_t;
            }
            float s = -INFINITY;
            if (vis && key < nk) {
                const bf16_t* kr = Kb + (long)key * D;
                float tot;
                if (gemv) {
                    float acc[16];
#pragma unroll
                    for (int l2 = 0; l2 < 16; ++l2) acc[l2] = 0.f;
                    for (int c = 0; c < D; c += 32) {
                        u32x4 kv[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) kv[j] = *(const u32x4*)(kr + c + 8 * j);
#pragma unroll
                        for (int l2 = 0; l2 < 16; ++l2) {
                            const uint32_t kw = kv[l2 >> 2][l2 & 3];
                            acc[l2] = fmaf(qs_[c + 2 * l2 + 1], bf_hi(kw), acc[l2]);
                            acc[l2] = fmaf(qs_[c + 2 * l2], bf_lo(kw), acc[l2]);
                        }
                    }
                    float v8[8], v4[4];
#pragma unroll
                    for (int l2 = 0; l2 < 8; ++l2) v8[l2] = __fadd_rn(acc[l2], acc[l2 + 8]);
#pragma unroll
                    for (int l2 = 0; l2 < 4; ++l2) v4[l2] = __fadd_rn(v8[2 * l2], v8[2 * l2 + 1]);
                    tot = __fadd_rn(__fadd_rn(v4[0], v4[1]), __fadd_rn(v4[2], v4[3]));
                } else {
                    tot = 0.f;
                    for (int c = 0; c < D; c += 32) {
                        u32x4 kv[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) kv[j] = *(const u32x4*)(kr + c + 8 * j);
                        float e = 0.f, o = 0.f;
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const uint32_t kw = kv[i >> 2][i & 3];
                            e = fmaf(qs_[c + 2 * i], bf_lo(kw), e);
                            o = fmaf(qs_[c + 2 * i + 1], bf_hi(kw), o);
                        }
                        tot = __fadd_rn(tot, __fadd_rn(e, o));
                    }
                }
                s = __fmul_rn(tot, a.scale);
            }
            sp[kk] = s;
            XA_DBG(0, bs + kk, s);
        }
        __syncthreads();
        // ---- running max, exp, lane-ordered block sum (wave 0); p rounded to bf16
        float lm = -INFINITY;
        for (int kk = tid; kk < blen; kk += 256) lm = fmaxf(lm, sp[kk]);
        __shared__ float red[4];
        lm = wave_max(lm);
        if (lane == 0) red[wave] = lm;
        __syncthreads();
        const float mn = fmaxf(m, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
        __syncthreads();
        for (int kk = tid; kk < blen; kk += 256) {
            XA_DBG(2, bs + kk, __fsub_rn(sp[kk], mn));
            sp[kk] = sdpa_p(__fsub_rn(sp[kk], mn), kk, blen);
            XA_DBG(3, bs + kk, sp[kk]);
        }
        if (tid < 16) sp[blen + tid] = 0.f;
        __syncthreads();
        if (wave == 0) {
            const float ts = sdpa_block_sum_lds<XA_BLOCK>(sp, blen, lane);
            if (lane == 0) bsum = ts;
        }
        __syncthreads();
        const float et = sdpa_block_rescale(m, mn);
        l = fmaf(et, l, bsum);
        for (int kk = tid; kk < blen; kk += 256) {
            sp[kk] = rbf(sp[kk]);
            XA_DBG(1, bs + kk, sp[kk]);
        }
        __syncthreads();
        // ---- P.V onto the rescaled output. This workgroup owns XA_DS output dims; each
        // dim's keys are cut into the GEMM's chunks (gemv: groups of 8 keys; else E/O
        // chunks of ch keys), XA_PARTS threads per dim compute chunk sums in parallel, then
        // the dim's owner folds them in chunk order onto the rescaled output.
        {
            const int dl = tid % XA_DS, part = tid / XA_DS;
            const int d = d0 + dl;
            const int ch = gemv ? 8 : (pack ? xa_even_div_chunk(blen) : 32);
            const int nch = (blen + ch - 1) / ch;
            const bf16_t* vc = Vb + (long)bs * D + d;
            if (gemv) {
                // pairs (odd key first), one chain per 8-key group. Every V value of this
                // thread's groups (<= 8 groups x 8 keys) is requested before the first
                // chain: one memory round trip instead of one per group. Keys past the block
                // read key 0 and count as 0 (clamped address, no branch around the load).
                constexpr int MAXG = XA_BLOCK / 8 / XA_PARTS;
                const int dd = min(d, D - 1);
                float vv[MAXG][8];
#pragma unroll
                for (int i = 0; i < MAXG; ++i) {
                    const int c0 = (part + i * XA_PARTS) * 8;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int key = c0 + j;
                        const float v = bf2f(Vb[(long)(bs + (key < blen ? key : 0)) * D + dd]);
                        vv[i][j] = key < blen ? v : 0.f;
                    }
                }
#pragma unroll
                for (int i = 0; i < MAXG; ++i) {
                    const int c = part + i * XA_PARTS;
                    if (d < D && c < nch) {
                        const int c0 = c * 8, cn = min(8, blen - c0);
                        float tmp = 0.f;
#pragma unroll
                        for (int j = 0; j < 8; j += 2) {
                            if (j < cn) {
                                if (j + 1 < cn) tmp = fmaf(sp[c0 + j + 1], vv[i][j + 1], tmp);
                                tmp = fmaf(sp[c0 + j], vv[i][j], tmp);
                            }
                        }
                        csum[c * XA_DS + dl] = tmp;
                    }
                }
            }
            for (int c = part; !gemv && d < D && c < nch; c += XA_PARTS) {
                const int c0 = c * ch, cn = min(ch, blen - c0);
                float cs;
                {             // E/O chains of the chunk
                    float e = 0.f, o = 0.f;
                    for (int j0 = 0; j0 < cn; j0 += 8) {
                        float vv[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) vv[j] = j0 + j < cn ? bf2f(vc[(long)(c0 + j0 + j) * D]) : 0.f;
#pragma unroll
                        for (int j = 0; j < 8; j += 2) {
                            if (j0 + j < cn) e = fmaf(sp[c0 + j0 + j], vv[j], e);
                            if (j0 + j + 1 < cn) o = fmaf(sp[c0 + j0 + j + 1], vv[j + 1], o);
                        }
                    }
                    cs = __fadd_rn(e, o);
                }
                csum[c * XA_DS + dl] = cs;
            }
            __syncthreads();
            if (part == 0 && d < D) {
                float acc = bs == 0 ? 0.f : __fmul_rn(dst, et);
                for (int c = 0; c < nch; ++c) {
                    const float cs = csum[c * XA_DS + dl];
                    acc = (!gemv && bs == 0 && c == 0) ? cs : __fadd_rn(acc, cs);
                }
                dst = acc;
            }
        }
        m = mn;
        __syncthreads();
    }
    if (tid < XA_DS && d0 + tid < D) {
        const bf16_t o = f2bf(__fmul_rn(dst, __fdiv_rn(1.0f, l)));
        a.O[(long)qi * a.ldo + h * D + d0 + tid] = o;
        if (a.O16) a.O16[x16_off(qi, h * D + d0 + tid, a.ldo / 32)] = o;
    }
}

// The same SDPA with one workgroup per (query token, query head) for a compile-time head
// dim (the engine's prefill / encoder calls): the scores are computed once (not once per
// output slice), every key's row is requested in one go, and thread d < D owns output
// dimension d, its chunk sums chained in registers from V values requested 32 keys at a
// time. Same arithmetic, in the same order, as exact_attn_kernel.
template <int D>
__global__ __launch_bounds__(256) void exact_attn_hd_kernel(ExactAttnArgs a) {
    static_assert(D % 32 == 0 && D <= 256, "head dim");
    __shared__ float qs_[D];
    __shared__ float sp[XA_BLOCK + 16];
    __shared__ float bsum;
    __shared__ float red[4];
    const int qi = blockIdx.x, h = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row = a.q_row ? a.q_row[qi] : qi;
    const int Tk_all = a.kv_len[row];
    const int Tq = a.q_len ? a.q_len[row] : 1;
    const int tq = a.q_pos ? a.q_pos[qi] : Tq - 1;
    const int abs_t = tq + (Tk_all - Tq);
    const bool has_mask = a.window > 0 && Tk_all >= a.window;
    int lo = 0;
    if (has_mask && Tq == 1 && a.causal) lo = Tk_all - a.window;
    const int Tk = Tk_all - lo;
    const bool sdpa_causal = a.causal && !has_mask && Tq > 1;
    const int qsz = sdpa_qsplit(Tq);
    const int qb0 = tq - tq % qsz;
    const int mblk = min(qsz, Tq - qb0);
    const int nk = sdpa_causal ? min(qb0 + mblk + (Tk_all - Tq), Tk) : Tk;
    const bool pack = xa_need_pack(Tq, Tk, a.Hq, D, a.threads, sdpa_causal);
    const bool gemv = mblk == 1 && !pack;
    const int kvh = h / (a.Hq / a.Hkv);
    const bf16_t* Kb = a.K + row * a.kv_bstride + kvh * a.kv_hstride + (long)lo * D;
    const bf16_t* Vb = a.V + row * a.kv_bstride + kvh * a.kv_hstride + (long)lo * D;
    for (int d = tid; d < D; d += 256) qs_[d] = bf2f(a.Q[(long)qi * a.ldq + h * D + d]);
    __syncthreads();
    const int d = min(tid, D - 1);   // this thread's output dimension (threads >= D idle in P.V)
    float m = -INFINITY, l = 0.f, dst = 0.f;
    for (int bs = 0; bs < nk; bs += XA_BLOCK) {
        const int blen = min(XA_BLOCK, Tk - bs);
        // ---- scores: thread per key, the key's row requested whole before the dot product
#pragma unroll 1
        for (int kk = tid; kk < blen; kk += 256) {
            const int key = bs + kk, kabs = key + lo;
            bool vis;
            if (has_mask) {
                if (Tq == 1 && a.causal) vis = true;
                else if (a.causal) vis = kabs <= abs_t && kabs > abs_t - a.window;
                else vis = abs(abs_t - kabs) <= a.window;
            } else {
                vis = !sdpa_causal || kabs <= abs_t;
            }
            const bf16_t* kr = Kb + (long)(key < nk ? key : 0) * D;
            // q is read from LDS inside the loop: hoisted out it would take D registers
            int z = 0;
            asm volatile("" : "+v"(z));
            const float* qv = qs_ + z;
            u32x4 kv[D / 8];
#pragma unroll
            for (int j = 0; j < D / 8; ++j) kv[j] = *(const u32x4*)(kr + 8 * j);
            float s = -INFINITY;
            if (vis && key < nk) {
                float tot;
                if (gemv) {
                    float acc[16];
#pragma unroll
                    for (int l2 = 0; l2 < 16; ++l2) acc[l2] = 0.f;
#pragma unroll
                    for (int cb = 0; cb < D / 32; ++cb) {
#pragma unroll
                        for (int l2 = 0; l2 < 16; ++l2) {
                            const uint32_t kw = kv[cb * 4 + (l2 >> 2)][l2 & 3];
                            acc[l2] = fmaf(qv[cb * 32 + 2 * l2 + 1], bf_hi(kw), acc[l2]);
                            acc[l2] = fmaf(qv[cb * 32 + 2 * l2], bf_lo(kw), acc[l2]);
                        }
                    }
                    float v8[8], v4[4];
#pragma unroll
                    for (int l2 = 0; l2 < 8; ++l2) v8[l2] = __fadd_rn(acc[l2], acc[l2 + 8]);
#pragma unroll
                    for (int l2 = 0; l2 < 4; ++l2) v4[l2] = __fadd_rn(v8[2 * l2], v8[2 * l2 + 1]);
                    tot = __fadd_rn(__fadd_rn(v4[0], v4[1]), __fadd_rn(v4[2], v4[3]));
                } else {
                    tot = 0.f;
#pragma unroll
                    for (int cb = 0; cb < D / 32; ++cb) {
                        float e = 0.f, o = 0.f;
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const uint32_t kw = kv[cb * 4 + (i >> 2)][i & 3];
                            e = fmaf(qv[cb * 32 + 2 * i], bf_lo(kw), e);
                            o = fmaf(qv[cb * 32 + 2 * i + 1], bf_hi(kw), o);
                        }
                        tot = __fadd_rn(tot, __fadd_rn(e, o));
                    }
                }
                s = __fmul_rn(tot, a.scale);
            }
            sp[kk] = s;
        }
        __syncthreads();
        // ---- running max, exp, lane-ordered block sum (wave 0); p rounded to bf16
        float lm = -INFINITY;
        for (int kk = tid; kk < blen; kk += 256) lm = fmaxf(lm, sp[kk]);
        lm = wave_max(lm);
        if (lane == 0) red[wave] = lm;
        __syncthreads();
        const float mn = fmaxf(m, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
        __syncthreads();
        for (int kk = tid; kk < blen; kk += 256) sp[kk] = sdpa_p(__fsub_rn(sp[kk], mn), kk, blen);
        if (tid < 16) sp[blen + tid] = 0.f;
        __syncthreads();
        if (wave == 0) {
            const float ts = sdpa_block_sum_lds<XA_BLOCK>(sp, blen, lane);
            if (lane == 0) bsum = ts;
        }
        __syncthreads();
        const float et = sdpa_block_rescale(m, mn);
        l = fmaf(et, l, bsum);
        for (int kk = tid; kk < blen; kk += 256) sp[kk] = rbf(sp[kk]);
        __syncthreads();
        // ---- P.V of dimension d onto the rescaled output, in the GEMM's chunk order
        const int ch = gemv ? 8 : (pack ? xa_even_div_chunk(blen) : 32);
        const int nch = (blen + ch - 1) / ch;
        const bf16_t* vc = Vb + (long)bs * D + d;
        float acc = bs == 0 ? 0.f : __fmul_rn(dst, et);
        // gemv: 32 keys' values (4 groups) per round trip; E/O: one chunk's (<= 32) per
        // round trip -- a packed chunk length (an even divisor of the block) need not divide
        // 32. Keys past the chunk / block read key 0 and are not used.
        const int step = gemv ? 32 : ch;
#pragma unroll 1
        for (int k0 = 0; k0 < blen; k0 += step) {
            const int kend = min(k0 + step, blen);
            float vv[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) vv[j] = bf2f(vc[(long)(k0 + j < kend ? k0 + j : 0) * D]);
            if (gemv) {
                // groups of 8 keys: pairs, odd key first, a fresh chain each, added in order
#pragma unroll
                for (int g8 = 0; g8 < 4; ++g8) {
                    const int c0 = k0 + 8 * g8;
                    if (c0 >= blen) break;
                    const int cn = min(8, blen - c0);
                    float tmp = 0.f;
#pragma unroll
                    for (int j = 0; j < 8; j += 2) {
                        if (j < cn) {
                            if (j + 1 < cn) tmp = fmaf(sp[c0 + j + 1], vv[8 * g8 + j + 1], tmp);
                            tmp = fmaf(sp[c0 + j], vv[8 * g8 + j], tmp);
                        }
                    }
                    acc = __fadd_rn(acc, tmp);
                }
            } else {
                // the E/O chains of the chunk [k0, kend)
                const int cn = kend - k0;
                float e = 0.f, o = 0.f;
#pragma unroll
                for (int j = 0; j < 32; j += 2) {
                    if (j < cn) e = fmaf(sp[k0 + j], vv[j], e);
                    if (j + 1 < cn) o = fmaf(sp[k0 + j + 1], vv[j + 1], o);
                }
                const float cs = __fadd_rn(e, o);
                acc = (bs == 0 && k0 == 0) ? cs : __fadd_rn(acc, cs);
            }
        }
        dst = acc;
        m = mn;
        __syncthreads();
    }
    if (tid < D) {
        const bf16_t o = f2bf(__fmul_rn(dst, __fdiv_rn(1.0f, l)));
        a.O[(long)qi * a.ldo + h * D + tid] = o;
        if (a.O16) a.O16[x16_off(qi, h * D + tid, a.ldo / 32)] = o;
    }
}

int exact_attention(const ExactAttnArgs& a, hipStream_t st) {
    if (a.Mq <= 0) return 0;
    if (!a.Q || !a.K || !a.V || !a.kv_len || !a.O || a.D > XA_MAXD || a.D % 32 || a.Hq % a.Hkv || a.threads <= 0)
        return -1;
    const dim3 g2((unsigned)a.Mq, (unsigned)a.Hq);
    if (a.D == 256) hipLaunchKernelGGL(exact_attn_hd_kernel<256>, g2, dim3(256), 0, st, a);
    else if (a.D == 128) hipLaunchKernelGGL(exact_attn_hd_kernel<128>, g2, dim3(256), 0, st, a);
    else if (a.D == 64) hipLaunchKernelGGL(exact_attn_hd_kernel<64>, g2, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(exact_attn_kernel, dim3((unsigned)a.Mq, (unsigned)a.Hq, (unsigned)((a.D + XA_DS - 1) / XA_DS)),
                            dim3(256), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

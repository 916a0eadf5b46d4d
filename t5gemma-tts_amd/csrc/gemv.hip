// Decode-step weight-streaming GEMM (M <= 16 rows) with the row prologue fused in.
//
// Y[M][N] = X[M][K] . W[N][K]^T on v_mfma_f32_16x16x32_bf16 over the P16 packed
// weights (gemm.hip). A block owns RG row groups (16 outputs each) for the WHOLE K
// range: its NW waves split each group's K stream (k-step kb belongs to wave
// kb % WPG) and reduce through LDS in fixed wave order, so every output is complete
// and deterministic (no split-K slabs, no batch dependence).
//
// Why the prologue lives here: at batch 8 a decode layer moves 87 MB
// of weights in ~11 us of HBM time, while each separate norm launch costs ~5 us of
// launch + dependent-load latency. Every block therefore rebuilds the X rows it needs
// from the previous sub-block's bf16 output v and the residual stream h (37 KB each
// at M = 8, L2-resident), in the reference's rounding order
// ([tf] T5GemmaRMSNorm :61-78; PMDecoderLayer wiring hf_export/modeling_t5gemma_voice.py:285-323):
//   a  = bf16((v * rsqrt(mean(v^2) + eps)) * (1 + post_w))
//   h' = bf16(h + a)                        -> h_out (block 0)
//   x  = bf16((h' * rsqrt(mean(h'^2) + eps)) * (1 + pre_w))  -> LDS
// while the block's first weight fragments are already in flight (the prologue's
// loads are issued first, so the weight stream never waits behind them).
// PRO_EMBED builds h' = bf16(table[id] * normalizer) instead (layer 0, [tf] :789-790).
// Row sums are lane-ordered partials + a fixed butterfly: batch-invariant.
#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

__device__ __forceinline__ f32x2 unpack2(uint32_t w) {
    return (f32x2){__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
__device__ __forceinline__ uint32_t pack2v(f32x2 x) { return pack2(x[0], x[1]); }

// Rows of the prologue: wave w handles rows w, w + NW, ... (RPW of them, all loads
// issued up front), lane l the 16-byte chunks l, l + 64, ... (CIM of them).
template <int NW, int PRO, int RPW, int CIM, typename Issue>
__device__ __forceinline__ void prologue_rows(const DecGemmArgs& a, bf16_t* xs, int ldsx, int wave, int lane,
                                              Issue&& issue) {
    const int CH = a.K >> 3;
    const bool writer = blockIdx.x == 0;
    u32x4 pw[CIM], qw[CIM];
    u32x4 sv[RPW][CIM], sh[RPW][CIM];
    int mrow[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) mrow[r] = min(wave + r * NW, a.M - 1);
    if constexpr (PRO == PRO_EMBED) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) mrow[r] = a.ids[mrow[r]];
    }
#pragma unroll
    for (int i = 0; i < CIM; ++i) {
        const int c = min(lane + 64 * i, CH - 1);
        if constexpr (PRO == PRO_NORM) pw[i] = *(const u32x4*)(a.post_w + 8 * c);
        if constexpr (PRO != PRO_LOAD) qw[i] = *(const u32x4*)(a.pre_w + 8 * c);
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if constexpr (PRO == PRO_NORM) {
                sv[r][i] = *(const u32x4*)(a.v + (long)mrow[r] * a.K + 8 * c);
                sh[r][i] = *(const u32x4*)(a.h_in + (long)mrow[r] * a.K + 8 * c);
            } else if constexpr (PRO == PRO_EMBED) {
                sv[r][i] = *(const u32x4*)(a.table + (long)mrow[r] * a.K + 8 * c);
            } else {
                sv[r][i] = *(const u32x4*)(a.X + (long)mrow[r] * a.ldx + 8 * c);
            }
        }
    }
    issue();   // the weight stream queues behind the prologue's loads, not in front of them
    // Row math on packed pairs (v_pk_mul/fma_f32, one v_cvt_pk_bf16_f32 per pair).
    const float inv_k = 1.0f / (float)a.K;
    const f32x2 one = {1.0f, 1.0f};
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int m = wave + r * NW;
        u32x4 hw[CIM];   // h' (bf16 pairs)
        if constexpr (PRO == PRO_NORM) {
            f32x2 ss = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < CIM; ++i)
                if (lane + 64 * i < CH)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const f32x2 x = unpack2(sv[r][i][j]);
                        ss += x * x;
                    }
            const float r1 = 1.0f / sqrtf(wave_sum_dpp(ss[0] + ss[1]) * inv_k + a.eps);
            const f32x2 r1v = {r1, r1};
#pragma unroll
            for (int i = 0; i < CIM; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f32x2 av = rbf2((unpack2(sv[r][i][j]) * r1v) * (one + unpack2(pw[i][j])));
                    hw[i][j] = pack2v(unpack2(sh[r][i][j]) + av);
                }
        } else if constexpr (PRO == PRO_EMBED) {
            const f32x2 sc = {a.scale, a.scale};
#pragma unroll
            for (int i = 0; i < CIM; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) hw[i][j] = pack2v(unpack2(sv[r][i][j]) * sc);
        } else {
#pragma unroll
            for (int i = 0; i < CIM; ++i) hw[i] = sv[r][i];
        }
        u32x4 xw[CIM];
        if constexpr (PRO != PRO_LOAD) {
            if (writer && a.h_out && m < a.M) {
#pragma unroll
                for (int i = 0; i < CIM; ++i)
                    if (lane + 64 * i < CH) *(u32x4*)(a.h_out + (long)m * a.K + 8 * (lane + 64 * i)) = hw[i];
            }
            f32x2 ss = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < CIM; ++i)
                if (lane + 64 * i < CH)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const f32x2 x = unpack2(hw[i][j]);
                        ss += x * x;
                    }
            const float r2 = 1.0f / sqrtf(wave_sum_dpp(ss[0] + ss[1]) * inv_k + a.eps);
            const f32x2 r2v = {r2, r2};
#pragma unroll
            for (int i = 0; i < CIM; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) xw[i][j] = pack2v((unpack2(hw[i][j]) * r2v) * (one + unpack2(qw[i][j])));
        } else {
#pragma unroll
            for (int i = 0; i < CIM; ++i) xw[i] = hw[i];
        }
        if (m < a.M) {
#pragma unroll
            for (int i = 0; i < CIM; ++i) {
                const int c = lane + 64 * i;
                if (c < CH) {
                    *(u32x4*)(xs + m * ldsx + 8 * c) = xw[i];
                    if (writer && a.x_out) *(u32x4*)(a.x_out + (long)m * a.K + 8 * c) = xw[i];
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// PRO_LEAD row producer: block m (< M) finishes row m of the previous sub-block and
// publishes the normed row; every block polls the M row flags before staging X.
// Bit-identical to resid_norm_kernel<NS, 2> with post, resid and pre (norm.hip): the
// 8-element chunk c is virtual thread c of that kernel's ceil(d/8/64)*64-thread block,
// held here by thread c % P in slot c / P; both block sums reduce every virtual wave
// with the same xor butterfly and add the virtual waves in order.
// Hand-off (CDNA guide G16, MI355X_MICROARCH "Valid forms" table row 1: one block per
// CU, one lane signals for the whole workgroup): every byte of the normed row is
// stored sc1 (16 B), every storing wave drains (vmcnt(0)), a barrier, one lane's
// relaxed agent-scope flag store; consumers poll with relaxed agent-scope (sc1)
// loads from ONE wave, barrier, then read the rows with sc1 loads only.
constexpr int LEAD_NS_MAX = 8;

template <int NW>
__device__ __forceinline__ void lead_row(const DecGemmArgs& a, int m, float* red) {
    constexpr int P = NW * 64;
    constexpr int S = (512 + P - 1) / P;   // slots per thread (d <= 4096)
    const int d = a.K, nch = d >> 3, nvw = (nch + 63) >> 6;
    const int tid = (int)threadIdx.x, wave = tid >> 6, lane = tid & 63;
    u32x4 wpost[S], wpre[S], rw[S];
    f32x4 pp[S][LEAD_NS_MAX][2];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        const int cc = min(tid + s * P, nch - 1);   // idle slots re-read the last chunk
#pragma unroll
        for (int k = 0; k < LEAD_NS_MAX; ++k) {
            const f32x4* ps = (const f32x4*)(a.part + ((long)min(k, a.nsplit_p - 1) * a.M + m) * a.ldp + 8 * cc);
            pp[s][k][0] = ps[0];
            pp[s][k][1] = ps[1];
        }
        wpost[s] = *(const u32x4*)(a.post_w + 8 * cc);
        wpre[s] = *(const u32x4*)(a.pre_w + 8 * cc);
        rw[s] = *(const u32x4*)(a.h_in + (long)m * d + 8 * cc);
    }
    float v[S][8];
    float ss[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[s][j] = 0.f;
#pragma unroll
        for (int k = 0; k < LEAD_NS_MAX; ++k)
            if (k < a.nsplit_p) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[s][j] += pp[s][k][0][j];
                    v[s][4 + j] += pp[s][k][1][j];
                }
            }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[s][j] = rbf(v[s][j]);
    }
    // two RMSNorm(1+w) passes (post, then pre after the residual add)
    auto rms = [&](const u32x4 (&w8)[S]) __attribute__((always_inline)) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
            float x = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) x += v[s][j] * v[s][j];
            ss[s] = (tid + s * P < nch) ? x : 0.f;
        }
        __syncthreads();   // red is reused by the second pass
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const float t = wave_sum(ss[s]);
            const int vw = wave + s * NW;
            if (lane == 0 && vw < nvw) red[vw] = t;
        }
        __syncthreads();
        float tot = 0.f;
        for (int i = 0; i < nvw; ++i) tot += red[i];   // virtual-wave order
        const float r = 1.0f / sqrtf(tot / (float)d + a.eps);
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float wl = bf_lo(w8[s][j]), wh = bf_hi(w8[s][j]);
                v[s][2 * j] = rbf((v[s][2 * j] * r) * (1.0f + wl));
                v[s][2 * j + 1] = rbf((v[s][2 * j + 1] * r) * (1.0f + wh));
            }
    };
    rms(wpost);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        u32x4 hw;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v[s][2 * j] = rbf(bf_lo(rw[s][j]) + v[s][2 * j]);
            v[s][2 * j + 1] = rbf(bf_hi(rw[s][j]) + v[s][2 * j + 1]);
            hw[j] = pack2(v[s][2 * j], v[s][2 * j + 1]);
        }
        const int c = tid + s * P;
        if (c < nch) *(u32x4*)(a.h_out + (long)m * d + 8 * c) = hw;   // next launches only
    }
    rms(wpre);
    const __amdgpu_buffer_rsrc_t xr = frag_rsrc(a.X + (long)m * a.ldx, (uint32_t)d * 2u);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        u32x4 xw;
#pragma unroll
        for (int j = 0; j < 4; ++j) xw[j] = pack2(v[s][2 * j], v[s][2 * j + 1]);
        const int c = tid + s * P;
        if (c < nch) __builtin_amdgcn_raw_buffer_store_b128(xw, xr, 16 * c, 0, 16);   // sc1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
    __syncthreads();
    if (tid == 0) __hip_atomic_store(a.flags + m, *a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ONE wave polls the M row flags (relaxed, agent scope: sc1 loads), bounded: a give-up
// sets *tmo (checked by the host) instead of hanging the chip
__device__ __forceinline__ void lead_wait(const DecGemmArgs& a) {
    if (threadIdx.x < 64) {
        const int lane = (int)threadIdx.x;
        unsigned* f = a.flags + min(lane, a.M - 1);
        const unsigned ep = *a.epoch;   // written by an earlier launch of the step
        for (unsigned spins = 0;; ++spins) {
            const bool ok = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ep;
            if (__all(ok)) break;
            if (spins > (1u << 16)) {
                if (lane == 0) __hip_atomic_store(a.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: keeps loads below
    }
    __syncthreads();
}

// Work split: the NG/RG "units" (RG row groups each) are dealt round-robin to at most
// one block per CU (grid <= #CUs), so the prologue runs once per CU however many units
// a block streams; each wave's k-steps over its units form ONE register-double-buffered
// stream (UN fragments in flight, the next unit's fragments already requested while the
// current unit finishes). A unit's partial sums go to LDS when its last k-step is done.
template <int NW, int RG, int EPI, int PRO, int RPW, int CIM, int UN>
__global__ __launch_bounds__(NW * 64) void gemv_dec_kernel(DecGemmArgs a) {
    constexpr int WPG = NW / RG;   // waves sharing one row group's K stream
    extern __shared__ __attribute__((aligned(16))) char smem[];   // one LDS object (no extra waits)
    // PRO_LEAD: blocks 0..M-1 only produce rows (their weight stream would start after
    // the hand-off and finish last); the units are dealt over the other blocks
    const int lead_n = PRO == PRO_LEAD ? a.M : 0;
    const int nb = (int)gridDim.x - lead_n;
    const int bu = (int)blockIdx.x - lead_n;   // < 0: leader, no units
    const int nunits = a.NG / RG;
    const int nu = bu < 0 ? 0 : (nunits - bu + nb - 1) / nb;   // units of this block
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
    if constexpr (PRO == PRO_DIRECT) {
        // X fragments straight from L2 beside the weights (rows >= M fall outside the
        // descriptor: zeros, no traffic)
        const __amdgpu_buffer_rsrc_t xrs = frag_rsrc(a.X, (uint32_t)a.M * a.ldx * 2u);
        const int xoff = (xr * a.ldx + 8 * (lane >> 4)) * 2;
        bf16x8_s xa[UN], xb[UN];
        auto batch = [&](bf16x8_s(&w)[UN], bf16x8_s(&x)[UN]) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const int kb = ks + jp * WPG;
                w[u] = wload(woff(ip, jp));
                x[u] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(
                                                        xrs, (ip < nu && kb < KBs) ? xoff + (kb_lo + kb) * 64 : (int)0xfffffff0u,
                                                        0, 0));
                adv(ip, jp);
            }
        };
        auto mul = [&](bf16x8_s(&w)[UN], bf16x8_s(&x)[UN]) __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                acc = mfma16(w[u], x[u], acc);
                retire();
            }
        };
        batch(wa, xa);
        for (int q = 0; q < total; q += 2 * UN) {
            batch(wb, xb);
            mul(wa, xa);
            batch(wa, xa);
            mul(wb, xb);
        }
    } else {
        // prologue loads first (oldest in the in-order vmcnt queue), then the first
        // weight batch, so the row math runs while weights stream in
        auto issue = [&]() __attribute__((always_inline)) { wbatch(wa); };
        if constexpr (PRO == PRO_LOAD || PRO == PRO_LEAD) {
            // plain staging: every chunk of the block's rows, all requested at once.
            // PRO_LEAD: the weight batch goes first (it streams while the leaders finish
            // their rows; a leader issues it after publishing, so its drain does not wait
            // on it), then the poll, then the rows by sc1 loads.
            constexpr bool LEAD = PRO == PRO_LEAD;
            if constexpr (LEAD) {
                if (bu < 0) {
                    lead_row<NW>(a, (int)blockIdx.x, (float*)xs);
                    return;   // no units: nothing to stage or multiply
                }
                issue();
                lead_wait(a);
            }
            constexpr int XCH = 10;
            const int CH = KBs * 4, tot = a.M * CH;
            const bf16_t* X0 = a.X + kb_lo * 32;
            const __amdgpu_buffer_rsrc_t xsrc = frag_rsrc(a.X, (uint32_t)a.M * (uint32_t)a.ldx * 2u);
            u32x4 xv[XCH];
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                const int idx = max(0, min((int)threadIdx.x + NW * 64 * i, tot - 1));
                const int r = idx / max(CH, 1), c = idx - r * CH;
                if constexpr (LEAD)
                    xv[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                          xsrc, (r * a.ldx + kb_lo * 32 + 8 * c) * 2, 0, 16));   // sc1
                else
                    xv[i] = *(const u32x4*)(X0 + (long)r * a.ldx + 8 * c);
            }
            if constexpr (!LEAD) issue();
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                const int idx = (int)threadIdx.x + NW * 64 * i;
                if (idx < tot) {
                    const int r = idx / CH, c = idx - r * CH;
                    *(u32x4*)(xs + r * ldsx + 8 * c) = xv[i];
                }
            }
        } else {
            prologue_rows<NW, PRO, RPW, CIM>(a, xs, ldsx, wave, lane, issue);
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
// Instantiated combinations (what the decode step and its tests use).
template <int EPI, int PRO>
constexpr bool gd_allowed() {
    if (PRO == PRO_NORM) return EPI == EPI_F32 || EPI == EPI_GEGLU || EPI == EPI_BIAS_GELU || EPI == EPI_BF16;
    if (PRO == PRO_EMBED) return EPI == EPI_F32;
    if (PRO == PRO_LEAD) return EPI == EPI_F32 || EPI == EPI_GEGLU;
    if (PRO == PRO_LOAD) return EPI == EPI_BF16 || EPI == EPI_BIAS_BF16 || EPI == EPI_F32 || EPI == EPI_GEGLU;
    return EPI == EPI_BF16 || EPI == EPI_F32;   // PRO_DIRECT
}

constexpr size_t GD_LDS_MAX = 160 * 1024;   // gfx950: 160 KB LDS per workgroup

static int cu_count() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

// blocks of one launch: <= one per CU (the prologue runs once per block)
static int gd_grid(const DecGemmArgs& a, int rg) {
    const int units = a.NG / rg;
    if (a.splits > 1) return units;   // split-K: one unit per block
    const int cap = a.max_grid > 0 ? a.max_grid : cu_count();
    return units < cap ? units : cap;
}

// fragments in flight per wave, kept spill-free (VGPR budget 512 / waves per SIMD)
template <int NW, int PRO, int CIM>
constexpr int gd_un() {
    return (NW >= 16 || CIM > 5 || (PRO == PRO_DIRECT && NW >= 8)) ? 8 : 16;
}

template <int NW, int RG, int EPI, int PRO, int RPW, int CIM, int UN>
static void launch_gd_un(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    auto* fn = gemv_dec_kernel<NW, RG, EPI, PRO, RPW, CIM, UN>;
    static bool attr = false;   // one opt-in per instantiation (not a stream operation)
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GD_LDS_MAX);
        attr = true;
    }
    hipLaunchKernelGGL(fn, dim3((unsigned)gd_grid(a, RG), (unsigned)a.splits), dim3(NW * 64), shm, st, a);
}

template <int NW, int RG, int EPI, int PRO, int RPW, int CIM>
static void launch_gd(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    constexpr int UND = gd_un<NW, PRO, CIM>();
    if (UND == 16 && a.un == 8) launch_gd_un<NW, RG, EPI, PRO, RPW, CIM, 8>(a, shm, st);
    else launch_gd_un<NW, RG, EPI, PRO, RPW, CIM, UND>(a, shm, st);
}

template <int NW, int RG, int EPI, int PRO>
static int launch_rows(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    if constexpr (PRO == PRO_LOAD || PRO == PRO_DIRECT || PRO == PRO_LEAD) {
        launch_gd<NW, RG, EPI, PRO, 1, 1>(a, shm, st);
        return 0;
    } else {
        const int rpw = (a.M + NW - 1) / NW;
        const int cim = (a.K / 8 + 63) / 64;
        // (rows per wave, chunks per lane) kept spill-free: (1|2, <=5) and (1, <=8)
        if (cim > 8 || rpw > 2 || (cim > 5 && rpw > 1)) return -3;
        if (cim > 5) launch_gd<NW, RG, EPI, PRO, 1, 8>(a, shm, st);
        else if (rpw == 1) launch_gd<NW, RG, EPI, PRO, 1, 5>(a, shm, st);
        else launch_gd<NW, RG, EPI, PRO, 2, 5>(a, shm, st);
        return 0;
    }
}

template <int EPI, int PRO>
static int launch_nw(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    if constexpr (!gd_allowed<EPI, PRO>()) {
        return -3;
    } else if constexpr (EPI == EPI_GEGLU) {
        // one row group (8 gate + the same 8 up rows) per unit: 1152 units at 2b-2b
        // balance over the CUs (4.5 per block) far better than 576 two-group units
        if (a.nw == 4) return launch_rows<4, 1, EPI, PRO>(a, shm, st);
        if (a.nw == 8) return launch_rows<8, 1, EPI, PRO>(a, shm, st);
        return -1;
    } else {
        if (a.nw == 4) return launch_rows<4, 1, EPI, PRO>(a, shm, st);
        if (a.nw == 8) return launch_rows<8, 1, EPI, PRO>(a, shm, st);
        if constexpr (PRO == PRO_LOAD || PRO == PRO_DIRECT) {   // 1024 threads: 128 VGPRs, no room for row math
            if (a.nw == 16) return launch_rows<16, 1, EPI, PRO>(a, shm, st);
        }
        return -1;
    }
}

size_t gemv_dec_lds_bytes(const DecGemmArgs& a, int pro, int rg) {
    const int grid = gd_grid(a, rg) - (pro == PRO_LEAD ? a.M : 0);
    const int umax = (a.NG / rg + grid - 1) / grid;
    const int per = (a.KB + a.splits - 1) / a.splits;
    size_t shm = (size_t)umax * a.nw * 64 * 16;
    if (pro != PRO_DIRECT) shm += (size_t)a.M * (per * 32 + 8) * sizeof(bf16_t);
    return shm;
}

int gemv_dec(const DecGemmArgs& a, int epi, int pro, hipStream_t st) {
    if (a.M <= 0) return 0;
    if (a.M > 16 || a.K % 32 || a.KB * 32 != a.K || a.NG % 4 || a.NG * 16 < a.N) return -1;
    if (a.splits < 1 || a.splits > 64 || (a.splits > 1 && (epi != EPI_F32 || pro == PRO_NORM || pro == PRO_EMBED)))
        return -1;
    if (a.nw != 4 && a.nw != 8 && a.nw != 16) return -1;
    const int rg = 1;
    if (a.NG % rg) return -1;
    if ((pro == PRO_LOAD || pro == PRO_DIRECT) && (!a.X || a.ldx < a.K || a.ldx % 8)) return -1;
    if (pro == PRO_NORM && (!a.v || !a.h_in || !a.post_w || !a.pre_w)) return -1;
    if (pro == PRO_EMBED && (!a.ids || !a.table || !a.pre_w)) return -1;
    if ((epi == EPI_BIAS_BF16 || epi == EPI_BIAS_GELU) && !a.bias) return -1;
    if (pro == PRO_DIRECT && (long)a.M * a.ldx * 2 >= 0x7ffffff0L) return -1;
    const size_t shm = gemv_dec_lds_bytes(a, pro, rg);
    if (shm > GD_LDS_MAX) return -1;
    if ((pro == PRO_LOAD || pro == PRO_LEAD) && a.M * ((a.KB + a.splits - 1) / a.splits) * 4 > a.nw * 64 * 10)
        return -1;   // XCH chunks
    if (pro == PRO_LEAD) {
        // every row needs its leader block resident: grid (one block per CU) >= M
        if (a.splits != 1 || !a.X || a.ldx < a.K || a.ldx % 8 || !a.part || a.nsplit_p < 1 ||
            a.nsplit_p > LEAD_NS_MAX || a.ldp < a.K || a.ldp % 4 || !a.h_in || !a.h_out || !a.post_w || !a.pre_w ||
            !a.flags || !a.tmo || !a.epoch || a.K > 4096 || gd_grid(a, rg) < 2 * a.M)
            return -1;
    }
    int rc = -4;
#define T5G_GE(E_)                                                              \
    switch (pro) {                                                              \
        case PRO_LOAD: rc = launch_nw<E_, PRO_LOAD>(a, shm, st); break;         \
        case PRO_NORM: rc = launch_nw<E_, PRO_NORM>(a, shm, st); break;         \
        case PRO_EMBED: rc = launch_nw<E_, PRO_EMBED>(a, shm, st); break;       \
        case PRO_DIRECT: rc = launch_nw<E_, PRO_DIRECT>(a, shm, st); break;     \
        case PRO_LEAD: rc = launch_nw<E_, PRO_LEAD>(a, shm, st); break;         \
        default: rc = -1;                                                       \
    }
    switch (epi) {
        case EPI_BF16: T5G_GE(EPI_BF16); break;
        case EPI_BIAS_BF16: T5G_GE(EPI_BIAS_BF16); break;
        case EPI_BIAS_GELU: T5G_GE(EPI_BIAS_GELU); break;
        case EPI_GEGLU: T5G_GE(EPI_GEGLU); break;
        case EPI_F32: T5G_GE(EPI_F32); break;
        default: return -1;
    }
#undef T5G_GE
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// ===========================================================================
// Row-major VALU GEMV (decode, M <= 8): exact N/grid rows per block, no split-K.
//
// W is the plain nn.Linear weight [N][K] bf16 (GEGLU: gate rows [0, F) then up rows
// [F, 2F)). Block b owns R = NR*RW consecutive output rows (GEGLU: R/2 features, gate
// and up), so a 2304-row projection is 256 blocks of 9 rows -- every CU streams the
// same share and every output is complete in its block (no fp32 slabs, no combine).
// Wave w owns row set w / NK and K-slice w % NK; lane l the 16-byte chunks
// c_lo + l + 64 j. Per chunk one weight load per row and 8 X chunks (LDS, or L2 in
// PRO_DIRECT) feed 4 v_dot2c_f32_bf16 per (row, batch row): at batch 8 that is 16 % of
// the chip's VALU issue at the HBM rate, so the kernel stays a weight stream.
// Reduction: DPP in-row butterfly, then lanes 0/16/32/48 and the NK slices through LDS,
// summed in fixed order -> deterministic and batch-invariant.
constexpr int RM_MB = 8;   // batch rows of one launch (accumulators per weight row)

__device__ __forceinline__ float dot8(u32x4 w, u32x4 x, float c) {
    // words through memcpy: __builtin_bit_cast of a vector element here made hipcc
    // (ROCm 7.2) feed word 0 to all four dot2s
    const uint32_t wa[4] = {w.x, w.y, w.z, w.w};
    const uint32_t xa[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        bf16x2_b p, q;
        __builtin_memcpy(&p, &wa[j], 4);
        __builtin_memcpy(&q, &xa[j], 4);
        c = __builtin_amdgcn_fdot2_f32_bf16(p, q, c, false);
    }
    return c;
}

template <int NR, int NK, int RW, int EPI, int PRO, int RPW, int CIM>
__global__ __launch_bounds__(NR * NK * 64) void gemv_rm_kernel(DecGemmArgs a) {
    constexpr int NW = NR * NK;
    constexpr int R = NR * RW;
    constexpr bool GLU = EPI == EPI_GEGLU;
    static_assert(!GLU || RW % 2 == 0, "GeGLU row sets hold gate/up pairs");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* red = (float*)smem;                                      // [NW][4][RW][8]
    bf16_t* xs = (bf16_t*)(smem + NW * 4 * RW * RM_MB * sizeof(float));   // [M][K + 8]
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = wave / NK, wk = wave % NK;
    const int K = a.K, nck = K >> 3;
    const int per = (nck + NK - 1) / NK;
    const int c_lo = wk * per, c_hi = min(nck, c_lo + per);
    const int CJ = (per + 63) >> 6;   // chunk steps per lane
    const int ldsx = K + 8;
    // rows of this wave
    int row[RW];
    if constexpr (GLU) {
        const int F = a.N / 2;
        const int f0 = blockIdx.x * (R / 2) + wr * (RW / 2);
#pragma unroll
        for (int i = 0; i < RW / 2; ++i) {
            row[i] = f0 + i;
            row[RW / 2 + i] = F + f0 + i;
        }
    } else {
#pragma unroll
        for (int i = 0; i < RW; ++i) row[i] = blockIdx.x * R + wr * RW + i;
    }
    const __amdgpu_buffer_rsrc_t wrs = frag_rsrc(a.W, (uint32_t)a.N * (uint32_t)K * 2u);
    auto woff = [&](int i, int j) -> int __attribute__((always_inline)) {
        const int c = c_lo + lane + 64 * j;
        const bool ok = c < c_hi && j < CJ && (GLU ? row[i] - (i >= RW / 2 ? a.N / 2 : 0) < a.N / 2 : row[i] < a.N);
        return ok ? (row[i] * K + 8 * c) * 2 : (int)0xfffffff0u;
    };
    auto wload = [&](int off) __attribute__((always_inline)) {
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wrs, off, 0, 2));   // nt
    };
    float acc[RW][RM_MB];
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
        for (int m = 0; m < RM_MB; ++m) acc[i][m] = 0.f;
    u32x4 wa[RW], wb[RW];
    auto wbatch = [&](u32x4(&w)[RW], int j) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < RW; ++i) w[i] = wload(woff(i, j));
    };

    if constexpr (PRO == PRO_DIRECT) {
        // X chunks from L2 (the block reads its K-slices of X once); rows >= M read row
        // M-1 and are dropped in the epilogue
        const __amdgpu_buffer_rsrc_t xrs = frag_rsrc(a.X, (uint32_t)a.M * a.ldx * 2u);
        u32x4 xa[RM_MB], xb[RM_MB];
        auto xbatch = [&](u32x4(&x)[RM_MB], int j) __attribute__((always_inline)) {
            const int c = c_lo + lane + 64 * j;
            const bool ok = c < c_hi && j < CJ;
#pragma unroll
            for (int m = 0; m < RM_MB; ++m)
                x[m] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                     xrs, ok ? (min(m, a.M - 1) * a.ldx + 8 * c) * 2 : (int)0xfffffff0u,
                                                     0, 0));
        };
        auto mul = [&](u32x4(&w)[RW], u32x4(&x)[RM_MB]) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < RW; ++i)
#pragma unroll
                for (int m = 0; m < RM_MB; ++m) acc[i][m] = dot8(w[i], x[m], acc[i][m]);
        };
        // ping-pong with a peeled tail: no batch of loads is ever issued past the stream
        wbatch(wa, 0);
        xbatch(xa, 0);
        int j = 0;
        for (; j + 2 < CJ; j += 2) {
            wbatch(wb, j + 1);
            xbatch(xb, j + 1);
            mul(wa, xa);
            wbatch(wa, j + 2);
            xbatch(xa, j + 2);
            mul(wb, xb);
        }
        if (CJ - j == 2) {
            wbatch(wb, j + 1);
            xbatch(xb, j + 1);
            mul(wa, xa);
            mul(wb, xb);
        } else {
            mul(wa, xa);
        }
    } else {
        auto issue = [&]() __attribute__((always_inline)) { wbatch(wa, 0); };
        if constexpr (PRO == PRO_LOAD) {
            constexpr int XCH = 10;
            const int tot = a.M * nck;
            u32x4 xv[XCH];
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                const int idx = min((int)threadIdx.x + NW * 64 * i, tot - 1);
                const int r = idx / nck, c = idx - r * nck;
                xv[i] = *(const u32x4*)(a.X + (long)r * a.ldx + 8 * c);
            }
            issue();
#pragma unroll
            for (int i = 0; i < XCH; ++i) {
                const int idx = (int)threadIdx.x + NW * 64 * i;
                if (idx < tot) {
                    const int r = idx / nck, c = idx - r * nck;
                    *(u32x4*)(xs + r * ldsx + 8 * c) = xv[i];
                }
            }
        } else {
            prologue_rows<NW, PRO, RPW, CIM>(a, xs, ldsx, wave, lane, issue);
        }
        __syncthreads();
        auto mul = [&](u32x4(&w)[RW], int j) __attribute__((always_inline)) {
            const int c = min(c_lo + lane + 64 * j, nck - 1);   // out-of-slice lanes: zero weights
#pragma unroll
            for (int m = 0; m < RM_MB; ++m) {
                const u32x4 x = *(const u32x4*)(xs + min(m, a.M - 1) * ldsx + 8 * c);
#pragma unroll
                for (int i = 0; i < RW; ++i) acc[i][m] = dot8(w[i], x, acc[i][m]);
            }
        };
        int j = 0;
        for (; j + 2 < CJ; j += 2) {
            wbatch(wb, j + 1);
            mul(wa, j);
            wbatch(wa, j + 2);
            mul(wb, j + 1);
        }
        if (CJ - j == 2) {
            wbatch(wb, j + 1);
            mul(wa, j);
            mul(wb, j + 1);
        } else {
            mul(wa, j);
        }
    }

    // ---- reduce: in-row DPP butterfly, then 4 rows x NK slices through LDS
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
        for (int m = 0; m < RM_MB; ++m) acc[i][m] = row16_sum(acc[i][m]);
    if ((lane & 15) == 0) {
        float* rp = red + ((wave * 4 + (lane >> 4)) * RW) * RM_MB;
#pragma unroll
        for (int i = 0; i < RW; ++i)
#pragma unroll
            for (int m = 0; m < RM_MB; ++m) rp[i * RM_MB + m] = acc[i][m];
    }
    __syncthreads();
    // one thread per (row set, output row, batch row)
    constexpr int OUTW = GLU ? RW / 2 : RW;
    for (int t = threadIdx.x; t < NR * OUTW * RM_MB; t += NW * 64) {
        const int m = t % RM_MB, o = (t / RM_MB) % OUTW, rs = t / (RM_MB * OUTW);
        if (m >= a.M) continue;
        auto sum = [&](int i) __attribute__((always_inline)) {
            float s = 0.f;
            for (int k = 0; k < NK; ++k)
#pragma unroll
                for (int q = 0; q < 4; ++q) s += red[(((rs * NK + k) * 4 + q) * RW + i) * RM_MB + m];
            return s;
        };
        if constexpr (GLU) {
            const int f = blockIdx.x * (R / 2) + rs * (RW / 2) + o;
            if (f >= a.N / 2) continue;
            const float v = rbf(gelu_tanh(rbf(sum(o)))) * rbf(sum(RW / 2 + o));
            ((bf16_t*)a.Y)[(long)m * a.ldy + f] = f2bf(v);
        } else {
            const int n = blockIdx.x * R + rs * RW + o;
            if (n >= a.N) continue;
            float v = sum(o);
            if constexpr (EPI == EPI_F32) {
                ((float*)a.Y)[(long)m * a.ldy + n] = v;
            } else {
                if constexpr (EPI == EPI_BIAS_BF16 || EPI == EPI_BIAS_GELU) v = v + bf2f(a.bias[n]);
                if constexpr (EPI == EPI_BIAS_GELU) v = gelu_erf(rbf(v));
                ((bf16_t*)a.Y)[(long)m * a.ldy + n] = f2bf(v);
            }
        }
    }
}

// Instantiated row-major configurations: (NR, NK, RW) -> rows per block R = NR*RW.
template <int NR, int NK, int RW, int EPI, int PRO>
static int launch_rm(const DecGemmArgs& a, size_t shm, hipStream_t st) {
    constexpr int NW = NR * NK;
    const int rpw = (a.M + NW - 1) / NW;
    const int cim = (a.K / 8 + 63) / 64;
    const int R = NR * RW;
    const int rows = EPI == EPI_GEGLU ? a.N / 2 : a.N;
    const int grid = (rows + (EPI == EPI_GEGLU ? R / 2 : R) - 1) / (EPI == EPI_GEGLU ? R / 2 : R);
    auto go = [&](auto fn) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GD_LDS_MAX);
            attr = true;
        }
        hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(NW * 64), shm, st, a);
    };
    if constexpr (PRO == PRO_LOAD || PRO == PRO_DIRECT) {
        go(gemv_rm_kernel<NR, NK, RW, EPI, PRO, 1, 1>);
    } else {
        if (cim > 5 || rpw > 2) return -3;
        if (rpw == 1) go(gemv_rm_kernel<NR, NK, RW, EPI, PRO, 1, 5>);
        else go(gemv_rm_kernel<NR, NK, RW, EPI, PRO, 2, 5>);
    }
    return 0;
}

size_t gemv_rm_lds_bytes(const DecGemmArgs& a, int pro, int nw, int rw) {
    size_t shm = (size_t)nw * 4 * rw * RM_MB * sizeof(float);
    if (pro != PRO_DIRECT) shm += (size_t)a.M * (a.K + 8) * sizeof(bf16_t);
    return shm;
}

// Layout choice by output rows per CU: R = ceil(rows / CUs) picks the configuration.
template <int EPI, int PRO>
static int gemv_rm_pick(const DecGemmArgs& a, hipStream_t st) {
    const int rows = EPI == EPI_GEGLU ? a.N / 2 : a.N;     // GeGLU: features
    const int per_cu = (rows + cu_count() - 1) / cu_count();
#define T5G_RM(NR_, NK_, RW_)                                                              \
    do {                                                                                   \
        const size_t shm = gemv_rm_lds_bytes(a, PRO, NR_ * NK_, RW_);                      \
        if (shm > GD_LDS_MAX) return -1;                                                   \
        if (PRO == PRO_LOAD && a.M * (a.K / 8) > NR_ * NK_ * 64 * 10) return -1;           \
        return launch_rm<NR_, NK_, RW_, EPI, PRO>(a, shm, st);                             \
    } while (0)
    if constexpr (EPI == EPI_GEGLU) {
        if (per_cu <= 4) T5G_RM(4, 1, 2);          // 4 features per block (tests)
        if (per_cu <= 36) T5G_RM(12, 1, 6);        // 36 features: 2b-2b gate/up (9216 / 256)
        return -3;
    } else if constexpr (PRO == PRO_DIRECT) {
        if (per_cu <= 1) T5G_RM(1, 4, 1);
        if (a.K >= 4096) {
            if (per_cu <= 9) T5G_RM(1, 8, 9);      // down: 9 rows, K split over 8 waves
        } else {
            if (per_cu <= 9) T5G_RM(1, 4, 9);
        }
        if (per_cu <= 16) T5G_RM(2, 4, 8);
        return -3;
    } else {
        if (per_cu <= 1) T5G_RM(4, 1, 1);
        if (per_cu <= 8) T5G_RM(2, 2, 4);          // cross-q: 8 rows
        if (per_cu <= 9) T5G_RM(1, 4, 9);          // o / head1: 9 rows
        if (per_cu <= 16) T5G_RM(4, 1, 4);         // q|k|v: 16 rows
        return -3;
    }
#undef T5G_RM
}

int gemv_rm(const DecGemmArgs& a, int epi, int pro, hipStream_t st) {
    if (a.M <= 0) return 0;
    if (a.M > RM_MB || a.K % 32 || !a.W || !a.Y) return -1;
    if (epi == EPI_GEGLU && a.N % 2) return -1;
    if ((pro == PRO_LOAD || pro == PRO_DIRECT) && (!a.X || a.ldx < a.K || a.ldx % 8)) return -1;
    if (pro == PRO_NORM && (!a.v || !a.h_in || !a.post_w || !a.pre_w)) return -1;
    if (pro == PRO_EMBED && (!a.ids || !a.table || !a.pre_w)) return -1;
    if ((epi == EPI_BIAS_BF16 || epi == EPI_BIAS_GELU) && !a.bias) return -1;
    if ((long)a.N * a.K * 2 >= 0xfffffff0L || (long)a.M * a.ldx * 2 >= 0x7ffffff0L) return -1;
    int rc = -3;
    switch (epi) {
        case EPI_F32:
            if (pro == PRO_NORM) rc = gemv_rm_pick<EPI_F32, PRO_NORM>(a, st);
            else if (pro == PRO_EMBED) rc = gemv_rm_pick<EPI_F32, PRO_EMBED>(a, st);
            else if (pro == PRO_DIRECT) rc = gemv_rm_pick<EPI_F32, PRO_DIRECT>(a, st);
            else rc = gemv_rm_pick<EPI_F32, PRO_LOAD>(a, st);
            break;
        case EPI_BF16:
            if (pro == PRO_NORM) rc = gemv_rm_pick<EPI_BF16, PRO_NORM>(a, st);
            else if (pro == PRO_DIRECT) rc = gemv_rm_pick<EPI_BF16, PRO_DIRECT>(a, st);
            else if (pro == PRO_LOAD) rc = gemv_rm_pick<EPI_BF16, PRO_LOAD>(a, st);
            break;
        case EPI_BIAS_GELU:
            if (pro == PRO_NORM) rc = gemv_rm_pick<EPI_BIAS_GELU, PRO_NORM>(a, st);
            break;
        case EPI_GEGLU:
            if (pro == PRO_NORM) rc = gemv_rm_pick<EPI_GEGLU, PRO_NORM>(a, st);
            else if (pro == PRO_LOAD) rc = gemv_rm_pick<EPI_GEGLU, PRO_LOAD>(a, st);
            break;
        default: return -1;
    }
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

// On-device AR sampler + stop logic: one 1024-thread block per utterance row.
//
// Restates, step for step and in the reference's bf16 rounding order, the
// ``sample_helper`` / ``topk_sampling`` / ``top_k_top_p_filtering`` path of
// hf_export/modeling_t5gemma_voice.py:84-138 and :702-786 (SURVEY a14'):
//   1. EOS / silence edits on the bf16 logits (-1e9 -> -998244352, -10000 -> -9984)
//   2. argmax of the edited logits (force-stop check)
//   3. x = bf16(x / T)
//   4. min_p: p = bf16(softmax(x)); drop p < bf16(min_p) if anything survives;
//      disables top-k / top-p
//   5. top-k: threshold = k-th largest (ties kept) by a 2-pass 8-bit radix select
//      over the 16-bit ordered bf16 keys
//   6. top-p: the sorted cumsum is replaced by a walk over DISTINCT values in
//      descending order (2-level radix histogram): within a tie group every
//      member adds the same bf16 probability, so the fp32 running sum with a
//      bf16-rounded prefix (torch CPU cumsum on bf16) is reproduced exactly
//      without sorting. Only if the cut falls INSIDE a tie group does the member
//      order matter (torch.sort's libstdc++ std::sort order); the kernel keeps the
//      lowest indices and flags the step ``ambiguous`` (parity mode re-runs such
//      steps with t5g_host_sample).
//   7. token = first argmax of bf16(bf16(softmax(x)) / q), q = the exponential
//      draw torch.multinomial makes (parity: uploaded; production: Philox4x32-10)
//   8. force-stop / time budget / silence-run state; next PM position computed in
//      double like the reference's Python float math (:817-823).
// The row's logits live in LDS as packed bf16 pairs (133 KB of the CU's 160 KB):
// every transform above rounds to bf16, so nothing is lost; thread t owns pairs
// t + 1024 * jp, i.e. elements 2 * (t + 1024 * jp) + {0, 1}.
#include "common.h"
#include "sort_emu.h"
#include "t5g_kernels.h"

namespace t5g {

T5G_TS_UNIT(sampler)

constexpr int SN = 1024;
constexpr int NW = SN / 64;
constexpr int SPER = 66;                // V <= SN * SPER = 67584
constexpr int SP2 = (SPER + 1) / 2;     // packed pairs
constexpr int TIE_CAP = 256;

__device__ __forceinline__ uint32_t okey(float v) {
    uint32_t b = (uint32_t)f2bf(v);
    return (b & 0x8000u) ? (~b & 0xffffu) : (b | 0x8000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
    uint32_t b = (k & 0x8000u) ? (k & 0x7fffu) : (~k & 0xffffu);
    return bf2f(b);
}

// element j (0..SPER-1) of thread t: pair jp = j >> 1, half j & 1 -> index 2*(t + SN*jp) + (j&1)
struct Packed {
    uint32_t* w;  // LDS base of this thread's pairs, stride SN
    __device__ __forceinline__ float get(int j) const {
        const uint32_t p = w[(j >> 1) * SN];
        return (j & 1) ? bf_hi(p) : bf_lo(p);
    }
    __device__ __forceinline__ void set(int j, float v) {
        const uint32_t b = f2bf(v);
        uint32_t& p = w[(j >> 1) * SN];
        p = (j & 1) ? ((p & 0xffffu) | (b << 16)) : ((p & 0xffff0000u) | b);
    }
};
__device__ __forceinline__ int eidx(int tid, int j) { return 2 * (tid + SN * (j >> 1)) + (j & 1); }

__device__ __forceinline__ int block_argmax(float v, int idx, float* redv, int* redi) {
    wave_argmax(v, idx);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) { redv[w] = v; redi[w] = idx; }
    __syncthreads();
    float bv = redv[0];
    int bi = redi[0];
    const int nw = (int)(blockDim.x >> 6);
    for (int i = 1; i < nw; ++i)
        if (redv[i] > bv || (redv[i] == bv && redi[i] < bi)) { bv = redv[i]; bi = redi[i]; }
    return bi;
}

__device__ __forceinline__ int block_count(int c, int* redi) {
    c = wave_sum(c);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) redi[w] = c;
    __syncthreads();
    int s = 0;
    const int nw = (int)(blockDim.x >> 6);
    for (int i = 0; i < nw; ++i) s += redi[i];
    return s;
}

// Sum the per-wave histograms into hsum (all threads call).
__device__ __forceinline__ void hist_reduce(unsigned (*wh)[256], unsigned* hsum) {
    __syncthreads();
    if (threadIdx.x < 256) {
        unsigned s = 0;
        const int nw = (int)(blockDim.x >> 6);
        for (int w = 0; w < nw; ++w) s += wh[w][threadIdx.x];
        hsum[threadIdx.x] = s;
    }
    __syncthreads();
}
__device__ __forceinline__ void hist_clear(unsigned (*wh)[256]) {
    for (int i = threadIdx.x; i < (int)(blockDim.x >> 6) * 256; i += blockDim.x) (&wh[0][0])[i] = 0;
    __syncthreads();
}

// Wave 0: bin b (descending from 255) where the running count from the top first
// reaches k; writes sel = b and above = count strictly above b.
__device__ __forceinline__ void find_bin_wave0(const unsigned* h, int k, int* sel, int* above) {
    const int l = threadIdx.x;  // lane of wave 0; covers bins 255-4l .. 252-4l
    int c[4];
    int loc = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        c[r] = (int)h[255 - 4 * l - r];
        loc += c[r];
    }
    int inc = loc;  // inclusive scan over lanes (lane 0 = top bins)
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(inc, o, 64);
        if (l >= o) inc += t;
    }
    const int exc = inc - loc;
    const unsigned long long hit = __ballot(inc >= k);
    const int first = hit ? __ffsll((long long)hit) - 1 : 63;
    if (l == first) {
        int run = exc, b = 255 - 4 * l - 3;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (run + c[r] >= k) { b = 255 - 4 * l - r; break; }
            run += c[r];
        }
        *sel = b;
        *above = run;
    }
}

__device__ __forceinline__ uint32_t philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0, uint32_t k1) {
    uint32_t c3 = 0x9E3779B9u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c0;
}

// The exponential draw q of torch.multinomial for element i: parity mode reads the
// uploaded reference stream, production draws Philox4x32-10(i, step; seed): the
// counter holds no batch slot, so an utterance samples the same tokens whatever
// its slot in the batch or the rank it is sharded to (rows needing different
// streams get different seeds from the host).
__device__ __forceinline__ float draw_q(const SamplerArgs& a, const SamplerRow& pr, const SamplerState& st, int b,
                                        int i) {
    // parity mode: the step's reference draws (steps past the uploaded ones -- never reached
    // when the host sizes the stream to the row budget + 1 -- reuse the last, in bounds)
    if (a.noise_mt) {
        const uint32_t* r = a.noise_mt + ((long)b * a.noise_mt_steps + min(st.cur_num_gen, a.noise_mt_steps - 1)) * 2L * a.V;
        return mt_exp_q(r[2 * i], r[2 * i + 1]);
    }
    if (a.noise) return bf2f(a.noise[((long)b * a.noise_steps + min(st.cur_num_gen, a.noise_steps - 1)) * a.V + i]);
    (void)b;
    const uint32_t u = philox((uint32_t)i, (uint32_t)st.cur_num_gen, 0u, pr.seed_lo, pr.seed_hi);
    const float uf = ((float)(u >> 8) + 1.0f) * (1.0f / 16777216.0f);
    float q = rbf(-logf(uf));
    if (q <= 0.f) q = 5.9604645e-08f;
    return q;
}

// Stop rules + per-row state update (:753-786, :806-832); one thread.
__device__ void finish_row(const SamplerArgs& a, const SamplerRow& pr, SamplerState st, int b, int token, int amax,
                           int ambiguous, int eff_len) {
    if (ambiguous & 4) {
        // parity mode, a tie order the device could not reproduce: the row STALLS (done = 2)
        // without committing the step -- no token, no state advance, so later steps of the
        // graph recompute the same logits for it -- until the host re-runs the step with
        // std::sort (t5g_host_sample) and writes the state back
        st.done = 2;
        if (a.flags) a.flags[b] = ambiguous | (amax == a.eos ? 2 : 0);
        a.state[b] = st;
        return;
    }
    bool force = (token == a.eos) || (amax == a.eos);
    if (a.text_guard > 0) force = force || (eff_len > max(1, st.first_input_len) * a.text_guard);
    bool budget = st.target_total >= 0 &&
                  (double)st.cur_num_gen > (double)(st.target_total - st.prompt_offset) + (double)a.budget_extra;
    // capacity: the last generated-token slot, or a self-attention cache with no room
    // for the next key, ends the row with EOS (only reachable without tgt_y_lens)
    const bool cap = st.cur_num_gen + 1 >= a.max_gen || st.current_length >= a.max_len;
    if (force || budget || cap) token = a.eos;
    bool in_sil = false;
    for (int s = 0; s < pr.n_silence; ++s) in_sil |= (a.silence[pr.silence_off + s] == token);
    if (in_sil && token == st.prev_token)
        st.consec_silence += 1;
    else
        st.consec_silence = 0;
    st.prev_token = token;
    a.out_tokens[(long)b * a.max_gen + st.cur_num_gen] = token;
    st.cur_num_gen += 1;
    st.current_length += 1;
    st.last_token = token;
    st.ambiguous_steps += ambiguous & 1;
    if (token == a.eos) {
        st.done = 1;
    } else {
        double v = (double)(st.current_length - 1) / (double)max(1, st.est_total - 1) * (double)a.progress_scale;
        v = v < (double)a.progress_scale ? v : (double)a.progress_scale;
        st.next_pos = (float)v;
        a.kv_len[b] = st.current_length;
        a.next_pos[b] = st.next_pos;
        a.next_token[b] = token;
    }
    if (a.flags) a.flags[b] = ambiguous | (amax == a.eos ? 2 : 0);
    a.state[b] = st;
}

// A row's state and parameters read in ONE batch at this point: without the register pins
// the compiler fetches some fields lazily after later branches (one dependent round trip
// each) and hoists the `done` test above the logit requests.
__device__ __forceinline__ void load_row(const SamplerArgs& a, int b, SamplerState& st, SamplerRow& pr) {
    constexpr int NS = (int)(sizeof(SamplerState) / 4), NR = (int)(sizeof(SamplerRow) / 4);
    static_assert(sizeof(SamplerState) % 4 == 0 && sizeof(SamplerRow) % 4 == 0, "dword structs");
    uint32_t ws[NS], wr[NR];
#pragma unroll
    for (int i = 0; i < NS; ++i) ws[i] = ((const uint32_t*)(a.state + b))[i];
#pragma unroll
    for (int i = 0; i < NR; ++i) wr[i] = ((const uint32_t*)(a.rows + b))[i];
    asm volatile("" ::: "memory");   // every request above is issued before the first pin
#pragma unroll
    for (int i = 0; i < NS; ++i) asm volatile("" : "+v"(ws[i]));
#pragma unroll
    for (int i = 0; i < NR; ++i) asm volatile("" : "+v"(wr[i]));
    __builtin_memcpy(&st, ws, sizeof(st));
    __builtin_memcpy(&pr, wr, sizeof(pr));
}

__global__ __launch_bounds__(SN) void sampler_kernel(SamplerArgs a) {
    __shared__ float redv[NW];
    __shared__ int redi[NW];
    __shared__ unsigned wh[NW][256];
    __shared__ unsigned hsum[256];
    __shared__ float gval[256];     // compact list of distinct values of one coarse bin
    __shared__ int gcnt[256];
    __shared__ int tie_idx[TIE_CAP];
    __shared__ uint32_t xs[SN * SP2];
    __shared__ int sh_int[8];
    __shared__ float sh_f[4];

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    // fs_slow requested with the state (no branch around the load: any valid address)
    const int fsv = *(a.fs_slow ? a.fs_slow + b : &a.state[b].done);
    SamplerState st;
    SamplerRow pr;
    load_row(a, b, st, pr);
    const int slow = a.fs_slow ? fsv : 1;
    if (st.done) return;
    if (!slow) return;   // finished by sampler_fast_kernel this step
    const int V = a.V;
    const bf16_t* lg = a.logits + (long)b * a.ldl;

    Packed x{xs + tid};
#pragma unroll
    for (int jp = 0; jp < SP2; ++jp) {
        const int i = 2 * (tid + SN * jp);
        uint32_t w;
        if (i + 1 < V && ((a.ldl & 1) == 0)) {
            w = *(const uint32_t*)(lg + i);
        } else {
            const uint32_t lo = i < V ? lg[i] : 0xff80u, hi = i + 1 < V ? lg[i + 1] : 0xff80u;
            w = lo | (hi << 16);
        }
        xs[tid + SN * jp] = w;
    }
    __syncthreads();
    // ---- 1. edits (:717-742)
    const int eff_len = max(0, st.current_length - st.prompt_offset);
    int kk = pr.top_k;
    if (pr.top_k_list_len > 0) kk = a.top_k_list[pr.top_k_list_off + min(pr.top_k_list_len - 1, st.cur_num_gen)];
    bool in_sil_prev = false;
    for (int s = 0; s < pr.n_silence; ++s) in_sil_prev |= (a.silence[pr.silence_off + s] == st.prev_token);
    const bool sil_rule = pr.stop_repetition > 0 && in_sil_prev && st.consec_silence > pr.stop_repetition;
    const float sil_f = (float)(st.consec_silence - (pr.stop_repetition - 1));
    if (tid == 0) {
        bf16_t* xh = (bf16_t*)xs;  // element index i lives at half-word i of the pair array
        float v = bf2f(xh[a.eos]);
        if (eff_len == 0) v = rbf(-1e9f);
        if (st.cur_num_gen <= a.eos_guard) v = rbf(-10000.0f);
        if (pr.eos_disabled) v = -INFINITY;
        xh[a.eos] = f2bf(v);
        if (sil_rule && st.prev_token >= 0 && st.prev_token < V) {
            const float u = bf2f(xh[st.prev_token]);
            xh[st.prev_token] = f2bf(u < 0.f ? u * sil_f : u / sil_f);
        }
    }
    __syncthreads();
    // ---- 2. argmax of the edited logits (:753-755)
    int amax;
    {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const int i = eidx(tid, j);
            const float v = x.get(j);
            if (i < V && (v > bv || bi == 0x7fffffff)) { bv = v; bi = i; }
        }
        amax = block_argmax(bv, bi, redv, redi);
    }
    // ---- 3. temperature
    if (pr.temperature != 1.0f) {
#pragma unroll
        for (int j = 0; j < SPER; ++j) x.set(j, x.get(j) / pr.temperature);
    }
    float top_p = pr.top_p;
    // ---- 4. min_p (:92-99)
    if (pr.min_p > 0.f && pr.min_p < 1.f) {
        float lm = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPER; ++j) lm = fmaxf(lm, x.get(j));
        const float m = block_max(lm, redv);
        float ls = 0.f;
#pragma unroll
        for (int j = 0; j < SPER; ++j) ls += expf(x.get(j) - m);
        const float inv = 1.0f / block_sum(ls, redv);
        const float thr = rbf(pr.min_p);
        int rm = 0;
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (eidx(tid, j) < V) rm += (rbf(expf(x.get(j) - m) * inv) < thr) ? 1 : 0;
        const int removed = block_count(rm, redi);
        if (removed < V) {
#pragma unroll
            for (int j = 0; j < SPER; ++j)
                if (rbf(expf(x.get(j) - m) * inv) < thr) x.set(j, -INFINITY);
            kk = 0;
            top_p = 1.0f;
        }
    }
    // ---- 5. top-k threshold (k-th largest, ties kept) (:101-105)
    if (kk > 0) {
        const int k = min(kk, V);
        // candidate prefilter: only values >= M - delta (delta grown until >= k of them)
        // enter the histograms, which keeps LDS-atomic contention off the bulk
        float thr0 = -INFINITY;
        if (k < V) {
            float lm = -INFINITY;
#pragma unroll
            for (int j = 0; j < SPER; ++j) lm = fmaxf(lm, x.get(j));
            const float M = block_max(lm, redv);
            float delta = 2.0f;
            for (int it = 0; it < 6; ++it) {
                const float t0 = M - delta;
                int c = 0;
#pragma unroll
                for (int j = 0; j < SPER; ++j) c += (eidx(tid, j) < V && x.get(j) >= t0) ? 1 : 0;
                if (block_count(c, redi) >= k) {
                    thr0 = t0;
                    break;
                }
                delta *= 4.0f;
            }
        }
        hist_clear(wh);
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (eidx(tid, j) < V && x.get(j) >= thr0) atomicAdd(&wh[wid][okey(x.get(j)) >> 8], 1u);
        hist_reduce(wh, hsum);
        if (wid == 0) find_bin_wave0(hsum, k, &sh_int[0], &sh_int[1]);
        __syncthreads();
        const uint32_t hb = (uint32_t)sh_int[0];
        const int need = k - sh_int[1];
        hist_clear(wh);
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (eidx(tid, j) < V && x.get(j) >= thr0) {
                const uint32_t kq = okey(x.get(j));
                if ((kq >> 8) == hb) atomicAdd(&wh[wid][kq & 255u], 1u);
            }
        hist_reduce(wh, hsum);
        if (wid == 0) find_bin_wave0(hsum, need, &sh_int[2], &sh_int[3]);
        __syncthreads();
        const float thr = key2f((hb << 8) | (uint32_t)sh_int[2]);
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (x.get(j) < thr) x.set(j, -INFINITY);
    }
    // ---- 6. top-p (:118-129)
    int ambiguous = 0;
    if (top_p < 1.0f) {
        float lm = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPER; ++j) lm = fmaxf(lm, x.get(j));
        const float m = block_max(lm, redv);
        float ls = 0.f;
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const float v = x.get(j);
            if (v > -INFINITY) ls += expf(v - m);
        }
        const float inv = 1.0f / block_sum(ls, redv);
        const float thr = rbf(top_p);
        // candidate prefilter: the top values whose probability mass already exceeds
        // top_p (the cut lies inside them); falls back to every value otherwise
        float thr0 = -INFINITY;
        {
            float delta = 4.0f;
            for (int it = 0; it < 4; ++it) {
                const float t0 = m - delta;
                float ms = 0.f;
#pragma unroll
                for (int j = 0; j < SPER; ++j) {
                    const float v = x.get(j);
                    if (v >= t0) ms += rbf(expf(v - m) * inv);
                }
                if (block_sum(ms, redv) > thr + 0.02f) {
                    thr0 = t0;
                    break;
                }
                delta *= 2.0f;
            }
        }
        __shared__ unsigned coarse[256];
    restart_walk:
        hist_clear(wh);
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const float v = x.get(j);
            if (v > -INFINITY && v >= thr0) atomicAdd(&wh[wid][okey(v) >> 8], 1u);
        }
        hist_reduce(wh, hsum);
        if (tid < 256) coarse[tid] = hsum[tid];
        if (tid == 0) {
            sh_int[4] = 0;      // state: 0 walking, 1 cut found, 2 exhausted
            sh_int[5] = 255;    // next coarse bin to visit
            sh_f[0] = 0.f;      // running fp32 cumsum
        }
        __syncthreads();
        while (true) {
            if (tid == 0 && sh_int[4] == 0) {
                int bb = sh_int[5];
                while (bb >= 0 && coarse[bb] == 0) --bb;
                if (bb < 0) sh_int[4] = 2;
                sh_int[5] = bb;
            }
            hist_clear(wh);  // (has a barrier)
            if (sh_int[4] != 0) break;
            const uint32_t hb = (uint32_t)sh_int[5];
#pragma unroll
            for (int j = 0; j < SPER; ++j) {
                const float v = x.get(j);
                if (v > -INFINITY && v >= thr0) {
                    const uint32_t kq = okey(v);
                    if ((kq >> 8) == hb) atomicAdd(&wh[wid][kq & 255u], 1u);
                }
            }
            hist_reduce(wh, hsum);
            if (wid == 0) {  // compact the non-empty fine bins, descending
                int c[4];
                int loc = 0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    c[r] = hsum[255 - 4 * lane - r] ? 1 : 0;
                    loc += c[r];
                }
                int inc = loc;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    int t = __shfl_up(inc, o, 64);
                    if (lane >= o) inc += t;
                }
                int pos = inc - loc;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int lb = 255 - 4 * lane - r;
                    if (c[r]) {
                        gval[pos] = key2f((hb << 8) | (uint32_t)lb);
                        gcnt[pos] = (int)hsum[lb];
                        ++pos;
                    }
                }
                if (lane == 63) sh_int[6] = inc;
            }
            __syncthreads();
            if (tid == 0) {
                float acc = sh_f[0];
                const int ng = sh_int[6];
                for (int q = 0; q < ng && sh_int[4] == 0; ++q) {
                    const float v = gval[q];
                    const int c = gcnt[q];
                    const float pv = rbf(expf(v - m) * inv);
                    for (int r = 0; r < c; ++r) {
                        acc += pv;
                        if (rbf(acc) > thr) {
                            sh_int[4] = 1;
                            sh_f[1] = v;      // cut value
                            sh_int[1] = r + 1;  // members of the cut group kept
                            sh_int[2] = c;      // group size
                            break;
                        }
                    }
                }
                sh_f[0] = acc;
                sh_int[5] = sh_int[5] - 1;
            }
            __syncthreads();
        }
        if (sh_int[4] == 2 && thr0 > -INFINITY) {  // cut not inside the candidates: use all
            thr0 = -INFINITY;
            __syncthreads();
            goto restart_walk;
        }
        if (sh_int[4] == 1) {
            const float vc = sh_f[1];
            const int keep = sh_int[1], gsz = sh_int[2];
#pragma unroll
            for (int j = 0; j < SPER; ++j)
                if (x.get(j) < vc) x.set(j, -INFINITY);
            if (keep < gsz) {
                // production tie-break: keep the `keep` lowest indices of the tie group; in
                // parity mode (reference noise) the row stalls for the host's std::sort
                ambiguous = (a.noise_mt || a.noise) ? 1 | 4 : 1;
                if (tid == 0) sh_int[7] = 0;
                __syncthreads();
#pragma unroll
                for (int j = 0; j < SPER; ++j) {
                    const int i = eidx(tid, j);
                    if (x.get(j) == vc) {
                        const int p = atomicAdd(&sh_int[7], 1);
                        if (p < TIE_CAP) tie_idx[p] = i;
                    }
                }
                __syncthreads();
                const int cnt = min(sh_int[7], TIE_CAP);
                // rank of each collected member = #members with a smaller index
#pragma unroll
                for (int j = 0; j < SPER; ++j) {
                    const int i = eidx(tid, j);
                    if (x.get(j) == vc) {
                        int rank = 0;
                        for (int q = 0; q < cnt; ++q) rank += tie_idx[q] < i;
                        if (rank >= keep) x.set(j, -INFINITY);
                    }
                }
            }
        }
    }
    // ---- 7. softmax + multinomial-as-argmax(p / q)
    int token;
    {
        float lm = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPER; ++j) lm = fmaxf(lm, x.get(j));
        const float m = block_max(lm, redv);
        float ls = 0.f;
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const float v = x.get(j);
            if (v > -INFINITY) ls += expf(v - m);
        }
        const float inv = 1.0f / block_sum(ls, redv);
        float bv = -1.f;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const int i = eidx(tid, j);
            if (i >= V) continue;
            const float xv = x.get(j);
            if (xv == -INFINITY) continue;  // p = 0 -> r = 0 can never beat a survivor
            const float p = rbf(expf(xv - m) * inv);
            float r = 0.f;
            if (p > 0.f) r = rbf(p / draw_q(a, pr, st, b, i));
            if (r > bv || (r == bv && i < bi)) { bv = r; bi = i; }
        }
        token = block_argmax(bv, bi, redv, redi);
    }
    // ---- 8. stop rules + state (:753-786, :806-832)
    if (tid == 0) finish_row(a, pr, st, b, token, amax, ambiguous, eff_len);
}


// ============================================================================
// Multi-block fast path. The single-block kernel above keeps a whole 65 541-entry
// row in one CU; with top-k active (the reference's defaults: k = 30, p = 0.9,
// inference_commandline_hf.py:80-83) everything after the top-k filter involves only
// the survivors, so the row is split over FS_NB blocks:
//   every block: edits + argmax + temperature over its slice, then its LOCAL top-k
//     candidates (all values >= the slice's k-th largest, ties included);
//   the last block to arrive (atomic ticket): merges the candidates (the global top-k
//     is a subset of them), takes the k-th largest as the threshold, sorts the
//     survivors (value desc, index asc), runs the top-p walk over distinct values,
//     softmaxes the final survivors and samples argmax(bf16(p / q)) -- the same
//     arithmetic as the single-block kernel -- then applies the stop rules.
// Rows the fast path cannot take (min_p, top-k off or > FS_KMAX, a slice with more
// than FS_CAP candidates, more than FS_SMAX survivors) are flagged in fs_slow and
// finished by the single-block kernel launched right after.
// st_sc1 / ld_sc1 (common.h): the fast path's cross-block candidate hand-off

constexpr int FT = 256;
// The candidate hand-off below (sc1 write-through stores, a drained vmcnt, one relaxed
// agent-scope ticket add, sc1 loads by the last block) is the gfx950 form of the CDNA
// guide's G16 pattern; another target's cache / counter model would need acquire-release.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "sampler_fast_kernel's cross-block hand-off is written for gfx950"
#endif
__device__ __forceinline__ bool lane_ok(int t) { return t < FS_NB; }
constexpr int FEPT = 24;   // V <= FS_NB * FT * FEPT = 98304

__device__ __forceinline__ float block_argmax_v(float v, int& idx, float* redv, int* redi) {
    wave_argmax(v, idx);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) { redv[w] = v; redi[w] = idx; }
    __syncthreads();
    float bv = redv[0];
    int bi = redi[0];
    const int nw = (int)(blockDim.x >> 6);
    for (int i = 1; i < nw; ++i)
        if (redv[i] > bv || (redv[i] == bv && redi[i] < bi)) { bv = redv[i]; bi = redi[i]; }
    idx = bi;
    return bv;
}

__global__ __launch_bounds__(FT) void sampler_fast_kernel(SamplerArgs a) {
    __shared__ float redv[FT / 64];
    __shared__ int redi[FT / 64];
    __shared__ unsigned wh[FT / 64][256];
    __shared__ unsigned hsum[256];
    __shared__ int sh_int[8];
    __shared__ float cv[FS_NB * FS_CAP];
    __shared__ int ci[FS_NB * FS_CAP];
    __shared__ float sv[FS_SMAX];
    __shared__ int si[FS_SMAX];
    __shared__ int soff[FS_NB + 1];
    __shared__ int is_last;

    const int sl = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, wid = tid >> 6;
    T5G_TS_START();
    // the slice's logits depend on nothing: request them first (clamped addresses, no
    // branch), so the row's state / parameters / silence list arrive meanwhile
    const int V = a.V;
    const int SL = (V + FS_NB - 1) / FS_NB;
    const int i0 = sl * SL, i1 = min(V, i0 + SL);
    const bf16_t* lg = a.logits + (long)b * a.ldl;
    bf16_t raw[FEPT];
#pragma unroll
    for (int j = 0; j < FEPT; ++j) raw[j] = lg[max(0, min(i0 + tid + FT * j, i1 - 1))];
    asm volatile("" ::: "memory");   // the logit requests go out before the row state is read
    SamplerState st;
    SamplerRow pr;
    load_row(a, b, st, pr);
    if (st.done) return;
    T5G_TS_COMMIT();
    int kk = pr.top_k;
    if (pr.top_k_list_len > 0) kk = a.top_k_list[pr.top_k_list_off + min(pr.top_k_list_len - 1, st.cur_num_gen)];
    const bool fast = kk > 0 && kk <= FS_KMAX && !(pr.min_p > 0.f && pr.min_p < 1.f);
    if (!fast) {
        if (sl == 0 && tid == 0) a.fs_slow[b] = 1;
        return;
    }
    const int k = min(kk, V);
    // ---- 1-3. edits, argmax of the edited logits, temperature (as sampler_kernel)
    const int eff_len = max(0, st.current_length - st.prompt_offset);
    bool in_sil_prev = false;
    for (int q = 0; q < pr.n_silence; ++q) in_sil_prev |= (a.silence[pr.silence_off + q] == st.prev_token);
    const bool sil_rule = pr.stop_repetition > 0 && in_sil_prev && st.consec_silence > pr.stop_repetition;
    const float sil_f = (float)(st.consec_silence - (pr.stop_repetition - 1));
    float x[FEPT];
    float bv = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < FEPT; ++j) {
        const int i = i0 + tid + FT * j;
        x[j] = -INFINITY;
        if (i < i1) {
            float v = bf2f(raw[j]);
            if (i == a.eos) {
                if (eff_len == 0) v = rbf(-1e9f);
                if (st.cur_num_gen <= a.eos_guard) v = rbf(-10000.0f);
                if (pr.eos_disabled) v = -INFINITY;
                v = rbf(v);
            }
            if (sil_rule && i == st.prev_token) v = rbf(v < 0.f ? v * sil_f : v / sil_f);
            if (v > bv || bi == 0x7fffffff) { bv = v; bi = i; }
            x[j] = pr.temperature != 1.0f ? rbf(v / pr.temperature) : v;
        }
    }
    const float amv = block_argmax_v(bv, bi, redv, redi);
    T5G_TS(1);
    // ---- 5a. local top-k candidates (k-th largest of the slice, ties kept)
    float thr = -INFINITY;
    if (i1 - i0 > k) {
        hist_clear(wh);
#pragma unroll
        for (int j = 0; j < FEPT; ++j)
            if (i0 + tid + FT * j < i1) atomicAdd(&wh[wid][okey(x[j]) >> 8], 1u);
        hist_reduce(wh, hsum);
        if (wid == 0) find_bin_wave0(hsum, k, &sh_int[0], &sh_int[1]);
        __syncthreads();
        const uint32_t hb = (uint32_t)sh_int[0];
        const int need = k - sh_int[1];
        hist_clear(wh);
#pragma unroll
        for (int j = 0; j < FEPT; ++j)
            if (i0 + tid + FT * j < i1) {
                const uint32_t kq = okey(x[j]);
                if ((kq >> 8) == hb) atomicAdd(&wh[wid][kq & 255u], 1u);
            }
        hist_reduce(wh, hsum);
        if (wid == 0) find_bin_wave0(hsum, need, &sh_int[2], &sh_int[3]);
        __syncthreads();
        thr = key2f((hb << 8) | (uint32_t)sh_int[2]);
    }
    if (tid == 0) sh_int[4] = 0;
    __syncthreads();
    float* gv = a.fs_val + ((long)b * FS_NB + sl) * FS_CAP;
    int* gi = a.fs_idx + ((long)b * FS_NB + sl) * FS_CAP;
#pragma unroll
    for (int j = 0; j < FEPT; ++j) {
        const int i = i0 + tid + FT * j;
        if (i < i1 && x[j] >= thr) {
            const int p = atomicAdd(&sh_int[4], 1);
            if (p < FS_CAP) {
                st_sc1(gv + p, x[j]);
                st_sc1(gi + p, i);
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        st_sc1(a.fs_cnt + b * FS_NB + sl, sh_int[4] > FS_CAP ? -1 : sh_int[4]);
        st_sc1(a.fs_amv + b * FS_NB + sl, amv);
        st_sc1(a.fs_ami + b * FS_NB + sl, bi);
    }
    T5G_TS(2);
    // ---- arrival ticket: the last slice block of the row finishes it. CDNA guide G16
    // valid form row 1: the candidates went out as sc1 (write-through) stores, every
    // storing wave drains them, one lane adds to the row's ticket, the block whose add
    // returns FS_NB-1 reads them back with sc1 loads -- no fences (the two all-thread
    // __threadfence()s this replaces cost ~8 us per step).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
        is_last = __hip_atomic_fetch_add(&a.fs_ticket[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  (unsigned)(FS_NB - 1);
    __syncthreads();
    if (!is_last) return;
    T5G_TS(3);
    // slice counts / argmaxes: one load per lane of wave 0, scan + argmax in registers
    if (wid == 0) {
        int c = 0, mi = 0x7fffffff;
        float mv = -INFINITY;
        if (lane_ok(tid)) {
            c = ld_sc1(a.fs_cnt + b * FS_NB + tid);
            mv = ld_sc1(a.fs_amv + b * FS_NB + tid);
            mi = ld_sc1(a.fs_ami + b * FS_NB + tid);
        }
        const unsigned long long badm = __ballot(c < 0);
        int inc = max(c, 0);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(inc, o, 64);
            if (tid >= o) inc += t;
        }
        if (tid < FS_NB) soff[tid + 1] = inc;
        if (tid == 0) {
            soff[0] = 0;
            sh_int[5] = badm != 0ull;
            a.fs_ticket[b] = 0;
        }
        wave_argmax(mv, mi);
        if (tid == 0) sh_int[6] = mi;
    }
    __syncthreads();
    if (sh_int[5]) {
        if (tid == 0) a.fs_slow[b] = 1;
        return;
    }
    const int amax = sh_int[6];
    const int n = soff[FS_NB];
    for (int q = tid; q < n; q += FT) {
        int sidx = 0;
#pragma unroll
        for (int t = 1; t < FS_NB; ++t) sidx += (q >= soff[t]);
        const long src = ((long)b * FS_NB + sidx) * FS_CAP + (q - soff[sidx]);
        cv[q] = ld_sc1(a.fs_val + src);
        ci[q] = ld_sc1(a.fs_idx + src);
    }
    __syncthreads();
    T5G_TS(4);
    // ---- 5b. global k-th largest over the merged candidates
    float gthr = -INFINITY;
    if (n > k) {
        hist_clear(wh);
        for (int q = tid; q < n; q += FT) atomicAdd(&wh[wid][okey(cv[q]) >> 8], 1u);
        hist_reduce(wh, hsum);
        if (wid == 0) find_bin_wave0(hsum, k, &sh_int[0], &sh_int[1]);
        __syncthreads();
        const uint32_t hb = (uint32_t)sh_int[0];
        const int need = k - sh_int[1];
        hist_clear(wh);
        for (int q = tid; q < n; q += FT) {
            const uint32_t kq = okey(cv[q]);
            if ((kq >> 8) == hb) atomicAdd(&wh[wid][kq & 255u], 1u);
        }
        hist_reduce(wh, hsum);
        if (wid == 0) find_bin_wave0(hsum, need, &sh_int[2], &sh_int[3]);
        __syncthreads();
        gthr = key2f((hb << 8) | (uint32_t)sh_int[2]);
    }
    if (tid == 0) sh_int[4] = 0;
    __syncthreads();
    for (int q = tid; q < n; q += FT)
        if (cv[q] >= gthr) {
            const int p = atomicAdd(&sh_int[4], 1);
            if (p < FS_SMAX) {
                sv[p] = cv[q];
                si[p] = ci[q];
            }
        }
    __syncthreads();
    const int ns = sh_int[4];
    if (ns > FS_SMAX) {
        if (tid == 0) a.fs_slow[b] = 1;
        return;
    }
    // survivors sorted by (value desc, index asc) into cv / ci
    if (tid < ns) {
        const float v = sv[tid];
        const int i = si[tid];
        int rank = 0;
        for (int r = 0; r < ns; ++r) rank += (sv[r] > v) || (sv[r] == v && si[r] < i);
        cv[rank] = v;
        ci[rank] = i;
    }
    __syncthreads();
    const float m = cv[0];
    T5G_TS(5);
    // ---- 6. top-p walk over distinct values (:118-129)
    int nkeep = ns, ambiguous = 0;
    if (pr.top_p < 1.0f) {
        float ls = 0.f;
        if (tid < ns && cv[tid] > -INFINITY) ls = expf(cv[tid] - m);
        const float inv = 1.0f / block_sum(ls, redv);
        if (wid == 0) {
            // wave 0: every survivor's bf16 probability in parallel (lane q%64, slot q/64),
            // then the cumsum walk in survivor order with register reads (v_readlane,
            // uniform index): sequential fp32 accumulation, each prefix rounded to bf16,
            // exactly the reference's order; a cut inside a tie group is ambiguous
            constexpr int NS = FS_SMAX / 64;
            float vr[NS], pr_[NS];
#pragma unroll
            for (int s2 = 0; s2 < NS; ++s2) {
                const int q = tid + 64 * s2;
                vr[s2] = q < ns ? cv[q] : -INFINITY;
                pr_[s2] = vr[s2] > -INFINITY ? rbf(expf(vr[s2] - m) * inv) : 0.f;
            }
            auto lane_get = [&](const float(&r)[NS], int q) __attribute__((always_inline)) {
                float out = -INFINITY;
#pragma unroll
                for (int s2 = 0; s2 < NS; ++s2)
                    if ((q >> 6) == s2)
                        out = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(r[s2]), q & 63));
                return out;
            };
            const float pthr = rbf(pr.top_p);
            float acc = 0.f;
            int keep_n = ns, amb = 0;
            for (int q = 0; q < ns; ++q) {
                const float v = lane_get(vr, q);
                if (v == -INFINITY) break;
                acc += lane_get(pr_, q);
                if (rbf(acc) > pthr) {
                    keep_n = q + 1;
                    amb = q + 1 < ns && lane_get(vr, q + 1) == v;
                    break;
                }
            }
            if (tid == 0) {
                sh_int[0] = keep_n;
                sh_int[1] = amb;
            }
        }
        __syncthreads();
        nkeep = sh_int[0];
        ambiguous = sh_int[1];
    }
    // ---- 7. softmax over the kept survivors + multinomial-as-argmax(p / q). The normaliser
    // depends only on how many survivors are kept (a cut group's members are equal), so the
    // r of every survivor up to the end of the cut group is known before the group's order
    float ls = 0.f;
    if (tid < nkeep && cv[tid] > -INFINITY) ls = expf(cv[tid] - m);
    const float inv = 1.0f / block_sum(ls, redv);
    const float vc = cv[nkeep - 1];
    int g1 = nkeep;   // end of the cut group (ambiguous: the group runs past nkeep)
    if (ambiguous) {
        if (tid == 0) {
            int e1 = nkeep;
            while (e1 < ns && cv[e1] == vc) ++e1;
            int e0 = nkeep - 1;
            while (e0 > 0 && cv[e0 - 1] == vc) --e0;
            sh_int[2] = e1;
            sh_int[3] = e0;
        }
        __syncthreads();
        g1 = sh_int[2];
    }
    auto r_of = [&](int q) -> float {
        const float p = rbf(expf(cv[q] - m) * inv);
        return p > 0.f ? rbf(p / draw_q(a, pr, st, b, ci[q])) : 0.f;
    };
    float rq = -1.f;
    if (tid < g1 && cv[tid] > -INFINITY) rq = r_of(tid);
    if (ambiguous && (a.noise_mt || a.noise)) {
        // parity mode: which members of the cut group are kept matters only if one of them
        // can win -- beat the best survivor above the group
        const int g0 = sh_int[3];
        int iw = tid < g0 ? ci[tid] : 0x7fffffff, ig = (tid >= g0 && tid < g1) ? ci[tid] : 0x7fffffff;
        const float rw = block_argmax_v(tid < g0 ? rq : -2.f, iw, redv, redi);
        const float rg = block_argmax_v((tid >= g0 && tid < g1) ? rq : -2.f, ig, redv, redi);
        if (rg > rw || (rg == rw && ig < iw)) {
            // the kept members are those torch.sort puts first: follow its std::sort on the
            // survivors (csrc/sort_emu.h), one thread. Survivors by token index (= initial
            // slot): spos / sval / stag (cv / ci slot)
            int* spos = (int*)&wh[0][0];
            int* stag = (int*)&wh[1][0];
            float* sval = sv;
            int nf = 0;   // finite survivors (a -inf tail sorts among the -inf entries)
            while (nf < ns && cv[nf] > -INFINITY) ++nf;
            if (tid < nf) {
                const int i = ci[tid];
                int r = 0;
                for (int q = 0; q < nf; ++q) r += ci[q] < i;
                spos[r] = i;
                sval[r] = cv[tid];
                stag[r] = tid;
            }
            __syncthreads();
            // <= 63 survivors: the replay on wave 0 (one survivor per lane, sort_emu.h
            // se_sort_wave); more: one thread (se_sort). Same steps, same slots.
            if (nf <= 63) {
                if (wid == 0) {
                    SEWave W{V, nf, tid < nf ? spos[tid] : 0x7fffffff, tid < nf ? sval[tid] : -INFINITY,
                             tid < nf ? stag[tid] : 0, 0};
                    int* stk = (int*)&wh[2][0];
                    const int f = se_sort_wave(W, stk, stk + SE_STACK, stk + 2 * SE_STACK);
                    if (tid < nf) {
                        spos[tid] = W.pos;
                        sval[tid] = W.val;
                        stag[tid] = W.tag;
                    }
                    if (tid == 0) sh_int[7] = f;
                }
                __syncthreads();
            }
            if (tid == 0) {
                SortEmu E{V, nf, spos, sval, stag, 0};
                const int sfail = nf <= 63 ? sh_int[7] : se_sort(E);
                if (sfail || vc == -INFINITY) {
                    sh_int[1] = 1 | 4;   // not reproducible here: stall for the host
                } else {
                    // the cut group [g0, g1) of cv / ci, reordered by final slot
                    int k = 0;
                    for (int q = 0; q < nf; ++q)
                        if (sval[q] == vc) si[k++] = ci[stag[q]];
                    for (int q = 0; q < k; ++q) ci[g0 + q] = si[q];
                }
            }
            __syncthreads();
            ambiguous = sh_int[1];
            if (tid >= g0 && tid < g1 && cv[tid] > -INFINITY) rq = r_of(tid);   // the group's new order
        }
    }
    float rbv = -1.f;
    int rbi = 0x7fffffff;
    if (tid < nkeep && cv[tid] > -INFINITY) {
        rbv = rq;
        rbi = ci[tid];
    }
    int token = rbi;
    block_argmax_v(rbv, token, redv, redi);
    if (tid == 0) {
        a.fs_slow[b] = 0;
        finish_row(a, pr, st, b, token, amax, ambiguous, eff_len);
    }
    T5G_TS(6);
}

// test entry: se_sort_wave on one wave over caller arrays (S <= 63), fail code in out[0]
__global__ __launch_bounds__(64) void sort_emu_wave_kernel(int n, int S, int* pos, float* val, int* tag, int* out) {
    __shared__ int stk[3 * SE_STACK];
    const int l = threadIdx.x;
    SEWave W{n, S, l < S ? pos[l] : 0x7fffffff, l < S ? val[l] : -INFINITY, l < S ? tag[l] : 0, 0};
    const int f = se_sort_wave(W, stk, stk + SE_STACK, stk + 2 * SE_STACK);
    if (l < S) {
        pos[l] = W.pos;
        val[l] = W.val;
        tag[l] = W.tag;
    }
    if (l == 0) out[0] = f;
}

int sort_emu_wave(int n, int S, int* pos, float* val, int* tag, int* out, hipStream_t st) {
    if (S < 0 || S > 63 || n < 0 || !out || (S > 0 && (!pos || !val || !tag))) return -1;
    hipLaunchKernelGGL(sort_emu_wave_kernel, dim3(1), dim3(64), 0, st, n, S, pos, val, tag, out);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

size_t sampler_fast_ws_bytes(int B) {
    return (size_t)B * ((size_t)FS_NB * FS_CAP * 8 + (size_t)FS_NB * 12 + 8);
}

int sample(const SamplerArgs& a, hipStream_t st) {
    if (a.B <= 0) return 0;
    if (a.V > SN * SPER) return -1;
    if (a.fs_slow) {
        if (a.V > FS_NB * FT * FEPT || !a.fs_val || !a.fs_ticket) return -1;
        hipLaunchKernelGGL(sampler_fast_kernel, dim3(FS_NB, (unsigned)a.B), dim3(FT), 0, st, a);
    }
    hipLaunchKernelGGL(sampler_kernel, dim3((unsigned)a.B), dim3(SN), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

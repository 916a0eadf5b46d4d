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
//      lowest indices and counts the step as ``ambiguous`` (parity mode resolves
//      such steps on the host).
//   7. token = first argmax of bf16(bf16(softmax(x)) / q), q = the exponential
//      draw torch.multinomial makes (parity: uploaded; production: Philox4x32-10)
//   8. force-stop / time budget / silence-run state; next PM position computed in
//      double like the reference's Python float math (:817-823).
#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

constexpr int SN = 1024;
constexpr int SPER = 65;  // V <= SN * SPER = 66560

__device__ __forceinline__ uint32_t okey(float v) {
    uint32_t b = (uint32_t)f2bf(v);
    return (b & 0x8000u) ? (~b & 0xffffu) : (b | 0x8000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
    uint32_t b = (k & 0x8000u) ? (k & 0x7fffu) : (~k & 0xffffu);
    return bf2f(b);
}

// (value, index) arg-max with first-index tie break; red2 holds 2*32 words
__device__ __forceinline__ int block_argmax(float v, int idx, float* redv, int* redi) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        float ov = __shfl_xor(v, o, 64);
        int oi = __shfl_xor(idx, o, 64);
        if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
    }
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) { redv[w] = v; redi[w] = idx; }
    __syncthreads();
    float bv = redv[0];
    int bi = redi[0];
    for (int i = 1; i < SN / 64; ++i) {
        if (redv[i] > bv || (redv[i] == bv && redi[i] < bi)) { bv = redv[i]; bi = redi[i]; }
    }
    return bi;
}

__device__ __forceinline__ int block_count(int c, int* redi) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    __syncthreads();
    if (l == 0) redi[w] = c;
    __syncthreads();
    int s = 0;
    for (int i = 0; i < SN / 64; ++i) s += redi[i];
    return s;
}

// Philox4x32-10 -> one uint32 per (seed, row, step, index)
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

__global__ __launch_bounds__(SN) void sampler_kernel(SamplerArgs a) {
    __shared__ float redv[32];
    __shared__ int redi[32];
    __shared__ unsigned hist[256];
    __shared__ unsigned hist2[256];
    __shared__ unsigned eqmask[(SN * SPER + 31) / 32];
    __shared__ int sh_int[8];
    __shared__ float sh_f[4];

    const int b = blockIdx.x;
    const int tid = threadIdx.x;
    SamplerState st = a.state[b];
    if (st.done) return;
    const SamplerRow pr = a.rows[b];
    const int V = a.V;
    const bf16_t* lg = a.logits + (long)b * a.ldl;

    float x[SPER];
#pragma unroll
    for (int j = 0; j < SPER; ++j) {
        int i = tid + SN * j;
        x[j] = i < V ? bf2f(lg[i]) : -INFINITY;
    }
    // ---- 1. edits (:717-742)
    const int eff_len = max(0, st.current_length - st.prompt_offset);
    int kk = pr.top_k;
    if (pr.top_k_list_len > 0) kk = a.top_k_list[pr.top_k_list_off + min(pr.top_k_list_len - 1, st.cur_num_gen)];
    bool in_sil_prev = false;
    for (int s = 0; s < pr.n_silence; ++s) in_sil_prev |= (a.silence[pr.silence_off + s] == st.prev_token);
    const bool sil_rule = pr.stop_repetition > 0 && in_sil_prev && st.consec_silence > pr.stop_repetition;
    const float sil_f = (float)(st.consec_silence - (pr.stop_repetition - 1));
#pragma unroll
    for (int j = 0; j < SPER; ++j) {
        const int i = tid + SN * j;
        if (i == a.eos) {
            if (eff_len == 0) x[j] = rbf(-1e9f);
            if (st.cur_num_gen <= a.eos_guard) x[j] = rbf(-10000.0f);
            if (pr.eos_disabled) x[j] = -INFINITY;
        }
        if (sil_rule && i == st.prev_token) x[j] = x[j] < 0.f ? rbf(x[j] * sil_f) : rbf(x[j] / sil_f);
    }
    // ---- 2. argmax of the edited logits (:753-755)
    int amax;
    {
        float bv = -INFINITY;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const int i = tid + SN * j;
            if (i < V && (x[j] > bv || bi == 0x7fffffff)) { bv = x[j]; bi = i; }
        }
        amax = block_argmax(bv, bi, redv, redi);
    }
    // ---- 3. temperature
    if (pr.temperature != 1.0f) {
#pragma unroll
        for (int j = 0; j < SPER; ++j) x[j] = rbf(x[j] / pr.temperature);
    }
    float top_p = pr.top_p;
    // ---- 4. min_p (:92-99)
    if (pr.min_p > 0.f && pr.min_p < 1.f) {
        float lm = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPER; ++j) lm = fmaxf(lm, x[j]);
        const float m = block_max(lm, redv);
        float ls = 0.f;
#pragma unroll
        for (int j = 0; j < SPER; ++j) ls += expf(x[j] - m);
        const float inv = 1.0f / block_sum(ls, redv);
        const float thr = rbf(pr.min_p);
        int rm = 0;
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (tid + SN * j < V) rm += (rbf(expf(x[j] - m) * inv) < thr) ? 1 : 0;
        const int removed = block_count(rm, redi);
        if (removed < V) {
#pragma unroll
            for (int j = 0; j < SPER; ++j)
                if (rbf(expf(x[j] - m) * inv) < thr) x[j] = -INFINITY;
            kk = 0;
            top_p = 1.0f;
        }
    }
    // ---- 5. top-k threshold (k-th largest, ties kept) (:101-105)
    if (kk > 0) {
        const int k = min(kk, V);
        for (int i = tid; i < 256; i += SN) hist[i] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (tid + SN * j < V) atomicAdd(&hist[okey(x[j]) >> 8], 1u);
        __syncthreads();
        if (tid == 0) {
            int above = 0, bsel = 0;
            for (int bb = 255; bb >= 0; --bb) {
                if (above + (int)hist[bb] >= k) { bsel = bb; break; }
                above += hist[bb];
            }
            sh_int[0] = bsel;
            sh_int[1] = k - above;
        }
        for (int i = tid; i < 256; i += SN) hist2[i] = 0;
        __syncthreads();
        const uint32_t hb = (uint32_t)sh_int[0];
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (tid + SN * j < V) {
                uint32_t kq = okey(x[j]);
                if ((kq >> 8) == hb) atomicAdd(&hist2[kq & 255u], 1u);
            }
        __syncthreads();
        if (tid == 0) {
            int need = sh_int[1], above = 0, lsel = 0;
            for (int bb = 255; bb >= 0; --bb) {
                if (above + (int)hist2[bb] >= need) { lsel = bb; break; }
                above += hist2[bb];
            }
            sh_f[0] = key2f((hb << 8) | (uint32_t)lsel);
        }
        __syncthreads();
        const float thr = sh_f[0];
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (x[j] < thr) x[j] = -INFINITY;
    }
    // ---- 6. top-p (:118-129)
    int ambiguous = 0;
    if (top_p < 1.0f) {
        float lm = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPER; ++j) lm = fmaxf(lm, x[j]);
        const float m = block_max(lm, redv);
        float ls = 0.f;
#pragma unroll
        for (int j = 0; j < SPER; ++j) ls += expf(x[j] - m);
        const float inv = 1.0f / block_sum(ls, redv);
        const float thr = rbf(top_p);
        for (int i = tid; i < 256; i += SN) hist[i] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SPER; ++j)
            if (x[j] > -INFINITY) atomicAdd(&hist[okey(x[j]) >> 8], 1u);
        __syncthreads();
        // walk high bins from the top; sh_int[2] = state (0 walking, 1 cut found, 2 exhausted)
        float acc = 0.f;  // meaningful in thread 0 only
        if (tid == 0) { sh_int[2] = 0; sh_int[3] = 255; }
        __syncthreads();
        while (true) {
            if (tid == 0 && sh_int[2] == 0) {
                int bb = sh_int[3];
                while (bb >= 0 && hist[bb] == 0) --bb;
                if (bb < 0) sh_int[2] = 2;
                sh_int[3] = bb;
            }
            for (int i = tid; i < 256; i += SN) hist2[i] = 0;
            __syncthreads();
            if (sh_int[2] != 0) break;
            const uint32_t hb = (uint32_t)sh_int[3];
#pragma unroll
            for (int j = 0; j < SPER; ++j)
                if (x[j] > -INFINITY) {
                    uint32_t kq = okey(x[j]);
                    if ((kq >> 8) == hb) atomicAdd(&hist2[kq & 255u], 1u);
                }
            __syncthreads();
            if (tid == 0) {
                for (int lb = 255; lb >= 0 && sh_int[2] == 0; --lb) {
                    const int c = (int)hist2[lb];
                    if (c == 0) continue;
                    const float v = key2f((hb << 8) | (uint32_t)lb);
                    const float pv = rbf(expf(v - m) * inv);
                    for (int r = 0; r < c; ++r) {
                        acc += pv;
                        if (rbf(acc) > thr) {
                            sh_int[2] = 1;
                            sh_f[1] = v;           // cut value
                            sh_int[4] = r + 1;     // members of the cut group kept
                            sh_int[5] = c;         // group size
                            break;
                        }
                    }
                }
                sh_int[3] = sh_int[3] - 1;
            }
            __syncthreads();
        }
        if (sh_int[2] == 1) {
            const float vc = sh_f[1];
            const int keep = sh_int[4], gsz = sh_int[5];
#pragma unroll
            for (int j = 0; j < SPER; ++j)
                if (x[j] < vc) x[j] = -INFINITY;
            if (keep < gsz) {
                ambiguous = 1;
                for (int i = tid; i < (SN * SPER + 31) / 32; i += SN) eqmask[i] = 0;
                __syncthreads();
#pragma unroll
                for (int j = 0; j < SPER; ++j) {
                    const int i = tid + SN * j;
                    if (x[j] == vc) atomicOr(&eqmask[i >> 5], 1u << (i & 31));
                }
                __syncthreads();
                if (tid == 0) {  // keep the lowest `keep` indices of the tie group
                    int left = keep;
                    for (int w = 0; w < (V + 31) / 32; ++w) {
                        unsigned bits = eqmask[w];
                        unsigned out = 0;
                        while (bits) {
                            unsigned lowb = bits & (~bits + 1u);
                            if (left > 0) { out |= lowb; --left; }
                            bits &= bits - 1u;
                        }
                        eqmask[w] = out;
                    }
                }
                __syncthreads();
#pragma unroll
                for (int j = 0; j < SPER; ++j) {
                    const int i = tid + SN * j;
                    if (x[j] == vc && !((eqmask[i >> 5] >> (i & 31)) & 1u)) x[j] = -INFINITY;
                }
            }
        }
    }
    // ---- 7. softmax + multinomial-as-argmax(p / q)
    int token;
    {
        float lm = -INFINITY;
#pragma unroll
        for (int j = 0; j < SPER; ++j) lm = fmaxf(lm, x[j]);
        const float m = block_max(lm, redv);
        float ls = 0.f;
#pragma unroll
        for (int j = 0; j < SPER; ++j) ls += expf(x[j] - m);
        const float inv = 1.0f / block_sum(ls, redv);
        const bf16_t* nz = a.noise ? a.noise + ((long)b * a.noise_steps + st.cur_num_gen) * V : nullptr;
        float bv = -1.f;
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < SPER; ++j) {
            const int i = tid + SN * j;
            if (i >= V) continue;
            const float p = rbf(expf(x[j] - m) * inv);
            float r = 0.f;
            if (p > 0.f) {
                float q;
                if (nz) {
                    q = bf2f(nz[i]);
                } else {
                    uint32_t u = philox((uint32_t)i, (uint32_t)st.cur_num_gen, (uint32_t)b, pr.seed_lo, pr.seed_hi);
                    float uf = ((float)(u >> 8) + 1.0f) * (1.0f / 16777216.0f);
                    q = rbf(-logf(uf));
                    if (q <= 0.f) q = 5.9604645e-08f;
                }
                r = rbf(p / q);
            }
            if (r > bv || (r == bv && i < bi)) { bv = r; bi = i; }
        }
        token = block_argmax(bv, bi, redv, redi);
    }
    // ---- 8. stop rules + state (:753-786, :806-832)
    if (tid == 0) {
        bool force = (token == a.eos) || (amax == a.eos);
        if (a.text_guard > 0) force = force || (eff_len > max(1, st.first_input_len) * a.text_guard);
        bool budget = st.target_total >= 0 &&
                      (double)st.cur_num_gen > (double)(st.target_total - st.prompt_offset) + (double)a.budget_extra;
        if (force || budget) token = a.eos;
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
        st.ambiguous_steps += ambiguous;
        if (token == a.eos || st.cur_num_gen >= a.max_gen) {
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
}

int sample(const SamplerArgs& a, hipStream_t st) {
    if (a.B <= 0) return 0;
    if (a.V > SN * SPER) return -1;
    hipLaunchKernelGGL(sampler_kernel, dim3((unsigned)a.B), dim3(SN), 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g

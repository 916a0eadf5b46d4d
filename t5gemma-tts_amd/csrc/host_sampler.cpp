// Host (CPU) sampler used ONLY in parity mode to resolve the rare "ambiguous"
// steps the device sampler flags: a top-p cut falling inside a group of tied
// bf16 logits, where the reference's kept set depends on the order torch.sort
// leaves equal keys in. torch's CPU sort (dim size 65541, stable=False) is
// libstdc++ std::sort over (value, index) pairs with a value-only descending
// comparator (NaN first); calling std::sort with that comparator on the same
// initial index-ordered array reproduces the reference's permutation exactly.
//
// This is part of libt5gtts.so (product library, C++), not of the oracle: it is
// the production fallback for exact-parity mode and is cross-checked against the
// reference's sampler goldens in tests/test_lib_cpu.py.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "sort_emu.h"
#include "t5gtts.h"

namespace {
inline float bf2f(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
inline uint16_t f2bf(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
inline float rbf(float f) { return bf2f(f2bf(f)); }

struct KV {
    float v;
    int64_t i;
};

// bf16(softmax_fp32(x)) over the whole vector
void softmax_bf16(const std::vector<float>& x, std::vector<float>& p) {
    float m = -INFINITY;
    for (float v : x) m = std::max(m, v);
    float s = 0.f;
    for (float v : x) s += std::exp(v - m);
    const float inv = 1.0f / s;
    p.resize(x.size());
    for (size_t i = 0; i < x.size(); ++i) p[i] = rbf(std::exp(x[i] - m) * inv);
}
}  // namespace

extern "C" int t5g_host_sample(const uint16_t* logits, int32_t V, const t5g_sampler_row* row,
                               const int32_t* top_k_list, const int32_t* silence, const t5g_sampler_state* st_in,
                               const uint16_t* noise, int32_t eos, int32_t eos_guard, float budget_extra,
                               int32_t text_guard, float progress_scale, int32_t max_gen, int32_t max_len,
                               t5g_sampler_state* st_out, int32_t* token_out) {
    if (!logits || !row || !st_in || !noise || !st_out || !token_out || V <= 0) return T5G_EINVAL;
    t5g_sampler_state st = *st_in;
    std::vector<float> x(V);
    for (int i = 0; i < V; ++i) x[i] = bf2f(logits[i]);
    // 1. edits
    const int eff_len = std::max(0, st.current_length - st.prompt_offset);
    if (eff_len == 0) x[eos] = rbf(-1e9f);
    int kk = row->top_k;
    if (row->top_k_list_len > 0) kk = top_k_list[row->top_k_list_off + std::min(row->top_k_list_len - 1, st.cur_num_gen)];
    if (st.cur_num_gen <= eos_guard) x[eos] = rbf(-10000.0f);
    if (row->eos_disabled) x[eos] = -INFINITY;
    bool in_sil_prev = false;
    for (int s = 0; s < row->n_silence; ++s) in_sil_prev |= silence[row->silence_off + s] == st.prev_token;
    if (row->stop_repetition > 0 && in_sil_prev && st.consec_silence > row->stop_repetition) {
        const float f = (float)(st.consec_silence - (row->stop_repetition - 1));
        float& v = x[st.prev_token];
        v = v < 0.f ? rbf(v * f) : rbf(v / f);
    }
    // 2. argmax of edited logits
    int amax = 0;
    for (int i = 1; i < V; ++i)
        if (x[i] > x[amax]) amax = i;
    // 3. temperature
    if (row->temperature != 1.0f)
        for (float& v : x) v = rbf(v / row->temperature);
    float top_p = row->top_p;
    std::vector<float> p;
    // 4. min_p
    if (row->min_p > 0.f && row->min_p < 1.f) {
        softmax_bf16(x, p);
        const float thr = rbf(row->min_p);
        int removed = 0;
        for (int i = 0; i < V; ++i) removed += p[i] < thr;
        if (removed < V) {
            for (int i = 0; i < V; ++i)
                if (p[i] < thr) x[i] = -INFINITY;
            kk = 0;
            top_p = 1.0f;
        }
    }
    // 5. top-k
    if (kk > 0) {
        const int k = std::min(kk, V);
        std::vector<float> tmp(x);
        std::nth_element(tmp.begin(), tmp.begin() + (k - 1), tmp.end(), [](float a, float b) { return a > b; });
        const float thr = tmp[k - 1];
        for (float& v : x)
            if (v < thr) v = -INFINITY;
    }
    // 6. top-p with torch.sort's exact permutation
    if (top_p < 1.0f) {
        std::vector<KV> kvs(V);
        for (int i = 0; i < V; ++i) kvs[i] = {x[i], i};
        std::sort(kvs.begin(), kvs.end(), [](const KV& a, const KV& b) {
            return (std::isnan(a.v) && !std::isnan(b.v)) || (a.v > b.v);
        });
        std::vector<float> sv(V);
        for (int i = 0; i < V; ++i) sv[i] = kvs[i].v;
        softmax_bf16(sv, p);
        const float thr = rbf(top_p);
        float acc = 0.f;
        std::vector<char> rm(V, 0);
        for (int i = 0; i < V; ++i) {
            acc += p[i];
            rm[i] = rbf(acc) > thr;
        }
        for (int i = V - 1; i >= 1; --i) rm[i] = rm[i - 1];
        rm[0] = 0;
        for (int i = 0; i < V; ++i)
            if (rm[i]) x[kvs[i].i] = -INFINITY;
    }
    // 7. softmax + argmax(p / q)
    softmax_bf16(x, p);
    int token = 0;
    float best = -1.f;
    for (int i = 0; i < V; ++i) {
        const float r = rbf(p[i] / bf2f(noise[i]));
        if (r > best) {
            best = r;
            token = i;
        }
    }
    // 8. stop rules + state
    bool force = token == eos || amax == eos;
    if (text_guard > 0) force = force || eff_len > std::max(1, st.first_input_len) * text_guard;
    const bool budget = st.target_total >= 0 &&
                        (double)st.cur_num_gen > (double)(st.target_total - st.prompt_offset) + (double)budget_extra;
    const bool cap = st.cur_num_gen + 1 >= max_gen || st.current_length >= max_len;   // as sampler.hip
    if (force || budget || cap) token = eos;
    bool in_sil = false;
    for (int s = 0; s < row->n_silence; ++s) in_sil |= silence[row->silence_off + s] == token;
    st.consec_silence = (in_sil && token == st.prev_token) ? st.consec_silence + 1 : 0;
    st.prev_token = token;
    st.cur_num_gen += 1;
    st.current_length += 1;
    st.last_token = token;
    if (token == eos) {
        st.done = 1;
    } else {
        double v = (double)(st.current_length - 1) / (double)std::max(1, st.est_total - 1) * (double)progress_scale;
        v = std::min(v, (double)progress_scale);
        st.next_pos = (float)v;
    }
    *st_out = st;
    *token_out = token;
    return T5G_OK;
}

// Host build of the device sampler's sparse std::sort emulation (csrc/sort_emu.h), for the
// CPU tests: S survivors at slots pos[] (ascending) with values val[] in an array of n
// otherwise -inf entries; on return pos[] / val[] / tag[] are ordered by final slot.
extern "C" int t5g_sort_emu(int32_t n, int32_t S, int32_t* pos, float* val, int32_t* tag) {
    if (n <= 0 || S < 0 || S > n || (S > 0 && (!pos || !val || !tag))) return T5G_EINVAL;
    for (int i = 1; i < S; ++i)
        if (pos[i] <= pos[i - 1] || pos[i] >= n) return T5G_EINVAL;
    t5g::SortEmu E{n, S, pos, val, tag, 0};
    return t5g::se_sort(E) ? T5G_EUNSUPPORTED : T5G_OK;
}

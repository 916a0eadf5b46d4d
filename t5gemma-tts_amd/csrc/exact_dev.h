// Exact-order (parity mode) device pieces shared by the per-op kernels (norm.hip, xmm.hip,
// xattn.hip) and the persistent exact decode layer (xlayer.hip): one definition, so the two
// paths compute the same bits.
#pragma once
#include "common.h"

namespace t5g {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

// chunk sum of one 16 x 16 tile: E and O chains over the chunk, then E + O
__device__ __forceinline__ f32x4_t xmm_chunk(const u32x4& w, const u32x4& x) {
    f32x4_t e = {0.f, 0.f, 0.f, 0.f}, o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        e = __builtin_amdgcn_mfma_f32_16x16x4f32(bf_lo(w[t]), bf_lo(x[t]), e, 0, 0, 0);
        o = __builtin_amdgcn_mfma_f32_16x16x4f32(bf_hi(w[t]), bf_hi(x[t]), o, 0, 0, 0);
    }
    f32x4_t c;
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = __fadd_rn(e[i], o[i]);
    return c;
}

// RoPE of one rotation pair as rope_store_kernel computes it (attn.hip): the three bf16
// tensor ops of apply_rotary_pos_emb
__device__ __forceinline__ void xd_rope(float x1, float x2, float c, float sn, float& o1, float& o2) {
    o1 = rbf(rbf(x1 * c) + rbf(-x2 * sn));
    o2 = rbf(rbf(x2 * c) + rbf(x1 * sn));
}

// Sum of squares in the order of torch 2.10's CPU float sum over a contiguous row
// (exact / parity mode). aten SumKernel.cpp cascade_sum -> vectorized_inner_sum, AVX2
// kernel (the AVX-512 stub is not registered): the row is a sequence of 8-float vectors
// (thread c holds vector c); row_sum interleaves 4 vector accumulators (vector c ->
// accumulator c % 4, row c / 4); multi_row_sum folds each accumulator's rows in a
// cascade of 4 levels of 16 rows; accumulators 1..3 are added to 0, vectors past the last
// whole row of 4 go to accumulator 0 first; finally the 8 lanes are summed in order.
// Verified bit for bit against torch on random rows (tools/cpu_order).
__device__ __forceinline__ float ref_sumsq(const float (&v)[8], bool active, int nvec, float* sq) {
    const int c = threadIdx.x;
    if (active) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sq[c * 8 + j] = __fmul_rn(v[j], v[j]);
    }
    __syncthreads();
    float a0 = 0.f;
    if (c < 32) {
        const int k = c >> 3, j = c & 7;
        const int size_ilp = nvec / 4;
        float a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int i = 0;
        // each level-0 row of 16 is read into registers first (one LDS round trip, not 16
        // dependent ones), then added in order
        while (i + 16 <= size_ilp) {
            float t[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) t[q] = sq[((i + q) * 4 + k) * 8 + j];
#pragma unroll
            for (int q = 0; q < 16; ++q) a0 = __fadd_rn(a0, t[q]);
            i += 16;
            a1 = __fadd_rn(a1, a0);
            a0 = 0.f;
            if (i & 0xF0) continue;
            a2 = __fadd_rn(a2, a1);
            a1 = 0.f;
            if (i & 0xF00) continue;
            a3 = __fadd_rn(a3, a2);
            a2 = 0.f;
        }
        {
            float t[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) t[q] = sq[(min(i + q, max(size_ilp - 1, 0)) * 4 + k) * 8 + j];
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (i + q < size_ilp) a0 = __fadd_rn(a0, t[q]);
        }
        a0 = __fadd_rn(__fadd_rn(__fadd_rn(a0, a1), a2), a3);
        if (k == 0)
            for (int t = size_ilp * 4; t < nvec; ++t) a0 = __fadd_rn(a0, sq[t * 8 + j]);
    }
    // the 8 lanes ((acc0 + acc1) + acc2) + acc3, then their sum in lane order, in wave 0 (the
    // cascade threads are its lanes 0..31); the total goes to every thread through one LDS word
    if (c < 64) {
        const int l = c & 7;
        float a = c < 32 ? a0 : 0.f;
        const float s1 = __shfl(a, l + 8, 64), s2 = __shfl(a, l + 16, 64), s3 = __shfl(a, l + 24, 64);
        const float lane_sum = __fadd_rn(__fadd_rn(__fadd_rn(a, s1), s2), s3);   // valid in lanes 0..7
        float tot = 0.f;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) tot = __fadd_rn(tot, __shfl(lane_sum, jj, 64));
        if (c == 0) sq[nvec * 8] = tot;
    }
    __syncthreads();
    // no trailing barrier: the next sum of squares writes sq[< nvec 8] only, and reads it (and
    // rewrites this word) after its own barrier
    return sq[nvec * 8];
}

// the exact RMSNorm(1 + w) of one row held 8 values per thread (norm.hip rms8<true>)
__device__ __forceinline__ void rms8_exact(float (&v)[8], bool active, int d, u32x4 w8, float eps, float* sq) {
    const float tot = ref_sumsq(v, active, d / 8, sq);
    float r = 1.0f / sqrtf(tot / (float)d + eps);
    if (!active) return;
    float wf[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        wf[2 * j] = bf_lo(w8[j]);
        wf[2 * j + 1] = bf_hi(w8[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rbf((v[j] * r) * (1.0f + wf[j]));
}

}  // namespace t5g

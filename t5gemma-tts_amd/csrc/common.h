// Shared device helpers for the T5Gemma-TTS gfx950 kernels.
// bf16 is carried as raw uint16 bits; all arithmetic is fp32 with explicit
// round-to-nearest-even back to bf16 wherever the reference's bf16 tensor op
// rounds (see DESIGN.md "numerics contract").
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef short bf16x8_s __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8_b __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// RNE fp32 -> bf16 (NaN preserved as quiet NaN). Branch-free: both results are
// computed and selected (v_cndmask), so unrolled callers stay straight-line code.
__device__ __forceinline__ bf16_t f2bf(float f) {
    const uint32_t u = __float_as_uint(f);
    const uint32_t rne = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
    const uint32_t qnan = (u >> 16) | 0x40u;
    return (bf16_t)(((u & 0x7fffffffu) > 0x7f800000u) ? qnan : rne);
}
// round an fp32 value to the nearest bf16 value, returned as fp32
__device__ __forceinline__ float rbf(float f) { return bf2f(f2bf(f)); }

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// block-wide sum for blockDim.x <= 1024; `red` needs 32 floats of LDS
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    int nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i];   // fixed order: deterministic
    return s;
}
__device__ __forceinline__ float block_max(float v, float* red) {
    v = wave_max(v);
    int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    int nw = (blockDim.x + 63) >> 6;
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    float s = -INFINITY;
    for (int i = 0; i < nw; ++i) s = fmaxf(s, red[i]);
    return s;
}

__device__ __forceinline__ float gelu_tanh(float x) {
    // torch gelu(approximate='tanh'): 0.5*x*(1+tanh(sqrt(2/pi)*(x+0.044715*x^3)))
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    float inner = k0 * (x + k1 * x * x * x);
    return 0.5f * x * (1.f + tanhf(inner));
}
__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}

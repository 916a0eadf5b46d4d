// Probe of the f32-input MFMA shapes for the parity Linears (xmm.hip):
//  1. operand / result lane layout of v_mfma_f32_4x4x1_16b_f32 (one-hot A lane);
//  2. bitwise: each form vs a VALU fmaf chain on random data;
//  3. issue rate: cycles per instruction, back-to-back independent accumulators, one wave.
// Build + run: hipcc -O3 --offload-arch=gfx950 tools/micro_mfma4.hip -o /tmp/mm4 && /tmp/mm4
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(float* out) {   // out[a][lane][4]
    const int lane = threadIdx.x;
    for (int a = 0; a < 64; ++a) {
        const float av = lane == a ? 1.0f : 0.0f;
        const float bv = (float)(lane + 1);
        f32x4 c = {0.f, 0.f, 0.f, 0.f};
        c = __builtin_amdgcn_mfma_f32_4x4x1f32(av, bv, c, 0, 0, 0);
        for (int r = 0; r < 4; ++r) out[(a * 64 + lane) * 4 + r] = c[r];
    }
}

__device__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ float rnd(uint32_t s) {   // bf16-valued floats over a wide exponent range
    const uint32_t h = hsh(s);
    const float m = (float)((h & 0xffff) - 32768) / 32768.0f;
    const int e = (int)((h >> 16) % 24) - 12;
    const float v = ldexpf(m, e);
    return __uint_as_float(__float_as_uint(v) & 0xffff0000u);
}

// 4x4x1: each instruction one fma step per element; chain of 64 steps with per-lane operands
__global__ void exact_kernel(int* bad4, int* bad16) {
    const int lane = threadIdx.x;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    __shared__ float As[64][64], Bs[64][64];
    for (int s = 0; s < 64; ++s) {
        As[s][lane] = rnd(s * 64 + lane);
        Bs[s][lane] = rnd(100000 + s * 64 + lane);
    }
    __syncthreads();
    for (int s = 0; s < 64; ++s) c = __builtin_amdgcn_mfma_f32_4x4x1f32(As[s][lane], Bs[s][lane], c, 0, 0, 0);
    // reference from the layout found in probe 1 (A lane = 4b + i, B lane = 4b + j, D lane = 4b + j, reg i)
    int bad = 0;
    const int b = lane >> 2, j = lane & 3;
    for (int r = 0; r < 4; ++r) {
        float ref = 0.f;
        for (int s = 0; s < 64; ++s) ref = fmaf(As[s][4 * b + r], Bs[s][4 * b + j], ref);
        bad += __float_as_uint(ref) != __float_as_uint(c[r]);
    }
    atomicAdd(bad4, bad);
    // 16x16x4 for comparison (the shape xmm uses): chain over 16 instructions x 4 k
    f32x4 d = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < 16; ++s) d = __builtin_amdgcn_mfma_f32_16x16x4f32(As[s][lane], Bs[s][lane], d, 0, 0, 0);
    bad = 0;
    const int jj = lane & 15, q = lane >> 4;
    for (int r = 0; r < 4; ++r) {
        const int i = q * 4 + r;
        float ref = 0.f;
        for (int s = 0; s < 16; ++s)
            for (int k = 0; k < 4; ++k) ref = fmaf(As[s][k * 16 + i], Bs[s][k * 16 + jj], ref);
        bad += __float_as_uint(ref) != __float_as_uint(d[r]);
    }
    atomicAdd(bad16, bad);
}

template <int SHAPE>
__global__ void rate_kernel(float* sink, long long* cyc, int iters) {
    f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const float a = (float)threadIdx.x, b = 1.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (SHAPE == 4) {
            c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c3, 0, 0, 0);
        } else {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    sink[threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
    if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
    float* d_out;
    hipMalloc(&d_out, 64 * 64 * 4 * sizeof(float));
    hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, d_out);
    static float h[64 * 64 * 4];
    hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    // for each one-hot A lane a: which (D lane, reg) are nonzero and which B lane they read
    printf("layout 4x4x1_16b: A lane a -> nonzero D (lane:reg=B lane)\n");
    for (int a = 0; a < 8; ++a) {
        printf("  a=%2d:", a);
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) {
                const float v = h[(a * 64 + l) * 4 + r];
                if (v != 0.f) printf(" %d:%d=%d", l, r, (int)v - 1);
            }
        printf("\n");
    }
    int *d_b4, *d_b16;
    hipMalloc(&d_b4, 4);
    hipMalloc(&d_b16, 4);
    hipMemset(d_b4, 0, 4);
    hipMemset(d_b16, 0, 4);
    hipLaunchKernelGGL(exact_kernel, dim3(1), dim3(64), 0, 0, d_b4, d_b16);
    int b4 = 0, b16 = 0;
    hipMemcpy(&b4, d_b4, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&b16, d_b16, 4, hipMemcpyDeviceToHost);
    printf("exact vs fmaf chain: 4x4x1_16b %d / 256 differ, 16x16x4 %d / 256 differ\n", b4, b16);
    long long* d_c;
    hipMalloc(&d_c, 8);
    float* sink;
    hipMalloc(&sink, 256 * 4);
    const int iters = 4096;
    long long c4 = 0, c16 = 0;
    hipLaunchKernelGGL(rate_kernel<4>, dim3(1), dim3(64), 0, 0, sink, d_c, iters);
    hipMemcpy(&c4, d_c, 8, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(rate_kernel<16>, dim3(1), dim3(64), 0, 0, sink, d_c, iters);
    hipMemcpy(&c16, d_c, 8, hipMemcpyDeviceToHost);
    printf("issue: 4x4x1_16b %.1f cyc/instr, 16x16x4 %.1f cyc/instr (s_memtime units, one wave)\n",
           (double)c4 / (4.0 * iters), (double)c16 / (4.0 * iters));
    return 0;
}

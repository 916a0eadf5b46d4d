// Launch-latency floor on MI355X: per-kernel time of back-to-back dependent launches
// captured in a hipGraph (as the decode step is), for (a) an empty kernel, (b) 8 blocks
// doing one dependent global load -> store, (c) the same with 256 blocks, (d) a block
// reduction with two __syncthreads. Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/micro_latency tools/micro_latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_empty() {}
__global__ void k_copy(const float* __restrict__ a, float* __restrict__ b, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i] + 1.0f;
}
__global__ void k_reduce(const float* __restrict__ a, float* __restrict__ b, int n) {
    __shared__ float red[16];
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = i < n ? a[i] : 0.f;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float s = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    __syncthreads();
    if (i < n) b[i] = a[i] * s;
}

template <typename F>
static float time_graph(hipStream_t st, int n, F launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int i = 0; i < n; ++i) launch(i);
    hipStreamEndCapture(st, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, st);
    hipStreamSynchronize(st);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    for (int r = 0; r < 5; ++r) hipGraphLaunch(ge, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return ms * 1000.f / (5 * n);
}

int main() {
    hipStream_t st;
    CHK(hipStreamCreate(&st));
    const int N = 1 << 22;
    float *a, *b;
    CHK(hipMalloc(&a, N * 4));
    CHK(hipMalloc(&b, N * 4));
    CHK(hipMemset(a, 0, N * 4));
    CHK(hipMemset(b, 0, N * 4));
    const int n = 400;
    printf("empty kernel, 1 block:          %.2f us\n", time_graph(st, n, [&](int) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st); }));
    printf("empty kernel, 1024 blocks:      %.2f us\n", time_graph(st, n, [&](int) { hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, st); }));
    printf("copy 8 blocks x 256 (ping-pong): %.2f us\n", time_graph(st, n, [&](int i) {
        hipLaunchKernelGGL(k_copy, dim3(8), dim3(256), 0, st, (i & 1) ? b : a, (i & 1) ? a : b, 2048); }));
    printf("copy 256 blocks x 256:          %.2f us\n", time_graph(st, n, [&](int i) {
        hipLaunchKernelGGL(k_copy, dim3(256), dim3(256), 0, st, (i & 1) ? b : a, (i & 1) ? a : b, 65536); }));
    printf("reduce 8 blocks x 320:          %.2f us\n", time_graph(st, n, [&](int i) {
        hipLaunchKernelGGL(k_reduce, dim3(8), dim3(320), 0, st, (i & 1) ? b : a, (i & 1) ? a : b, 2560); }));
    printf("copy 2048 blocks x 256 (2 MB):  %.2f us\n", time_graph(st, n, [&](int i) {
        hipLaunchKernelGGL(k_copy, dim3(2048), dim3(256), 0, st, (i & 1) ? b : a, (i & 1) ? a : b, 524288); }));
    return 0;
}

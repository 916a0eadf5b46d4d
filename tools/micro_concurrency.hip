// Do parallel branches of a captured hipGraph run concurrently on MI355X? A chain of 40
// short dependent kernels (stream A) beside one long 64-block streaming kernel (stream B),
// captured with an event fork/join, timed against each branch alone. Also: the same
// pair launched eagerly on two streams, and a low-priority stream for the long kernel.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/micro_concurrency tools/micro_concurrency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_short(const float* __restrict__ a, float* __restrict__ b, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i] * 0.5f + 1.0f;
}
// each block streams `per` bytes (uint4) and folds them
__global__ void k_stream(const uint4* __restrict__ buf, size_t per_u4, uint4* out) {
    const uint4* p = buf + blockIdx.x * per_u4;
    uint4 acc = {0, 0, 0, 0};
    for (size_t i = threadIdx.x; i < per_u4; i += 256 * 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const size_t j = i + 256 * u;
            if (j < per_u4) {
                uint4 v = p[j];
                acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
            }
        }
    }
    if (acc.x == 0x9e3779b9u) out[blockIdx.x] = acc;
}

int main() {
    hipStream_t sa, sb, slo;
    CHK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    int lo_pri = 0, hi_pri = 0;
    CHK(hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
    CHK(hipStreamCreateWithPriority(&slo, hipStreamNonBlocking, lo_pri));
    printf("stream priority range: least %d greatest %d\n", lo_pri, hi_pri);
    const size_t big = (size_t)512 << 20;
    uint4* buf;
    CHK(hipMalloc(&buf, big));
    CHK(hipMemset(buf, 1, big));
    float *a, *b;
    CHK(hipMalloc(&a, 1 << 20));
    CHK(hipMalloc(&b, 1 << 20));
    uint4* out;
    CHK(hipMalloc(&out, 1 << 16));
    const int nshort = 40, sblocks = 64;
    const size_t per_u4 = big / 16 / sblocks;
    auto chain = [&](hipStream_t s) {
        for (int i = 0; i < nshort; ++i)
            hipLaunchKernelGGL(k_short, dim3(8), dim3(256), 0, s, (i & 1) ? b : a, (i & 1) ? a : b, 2048);
    };
    auto longk = [&](hipStream_t s) { hipLaunchKernelGGL(k_stream, dim3(sblocks), dim3(256), 0, s, buf, per_u4, out); };
    hipEvent_t e0, e1, fork, join;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CHK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    auto time_graph = [&](const char* name, int mode) -> int {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(sa, hipStreamCaptureModeGlobal));
        if (mode == 0) {
            chain(sa);
        } else if (mode == 1) {
            longk(sa);
        } else {
            hipStream_t other = mode == 3 ? slo : sb;
            CHK(hipEventRecord(fork, sa));
            CHK(hipStreamWaitEvent(other, fork, 0));
            longk(other);
            chain(sa);
            CHK(hipEventRecord(join, other));
            CHK(hipStreamWaitEvent(sa, join, 0));
        }
        CHK(hipStreamEndCapture(sa, &g));
        CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int r = 0; r < 3; ++r) CHK(hipGraphLaunch(ge, sa));
        CHK(hipStreamSynchronize(sa));
        CHK(hipEventRecord(e0, sa));
        for (int r = 0; r < 10; ++r) CHK(hipGraphLaunch(ge, sa));
        CHK(hipEventRecord(e1, sa));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("graph %-40s %8.1f us\n", name, ms * 100.f);
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
        return 0;
    };
    if (time_graph("chain of 40 short kernels alone", 0)) return 1;
    if (time_graph("long streaming kernel alone", 1)) return 1;
    if (time_graph("both, fork/join (2 branches)", 2)) return 1;
    if (time_graph("both, long on low-priority stream", 3)) return 1;
    // eager two streams
    for (int r = 0; r < 2; ++r) {
        CHK(hipDeviceSynchronize());
        CHK(hipEventRecord(e0, sa));
        CHK(hipStreamWaitEvent(sb, e0, 0));
        for (int k = 0; k < 10; ++k) {
            longk(sb);
            chain(sa);
        }
        CHK(hipEventRecord(join, sb));
        CHK(hipStreamWaitEvent(sa, join, 0));
        CHK(hipEventRecord(e1, sa));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("eager two streams (run %d)                    %8.1f us\n", r, ms * 100.f);
    }
    return 0;
}

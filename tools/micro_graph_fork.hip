// Do two kernels on forked streams run side by side -- eagerly, and inside a captured
// hipGraph (fork: event record + stream wait, join: the same back)? Kernel A (one workgroup)
// polls a flag that kernel B (one workgroup, launched on the other branch) sets; A gives up
// after a bounded number of polls. A reports how many polls it needed: a small count = the
// two ran concurrently, the cap = they ran one after the other.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro_graph_fork.hip -o /tmp/gf
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                          \
        }                                                                      \
    } while (0)

constexpr int MAX_POLLS = 200000;   // ~ tens of ms: a serialised pair ends, it does not hang

__global__ void waiter(unsigned* flag, int* polls) {
    if (threadIdx.x != 0) return;
    int n = 0;
    while (n < MAX_POLLS && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(2);
        ++n;
    }
    polls[0] = n;
}

__global__ void setter(unsigned* flag) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int run(bool graph) {
    unsigned* flag;
    int* polls;
    CK(hipMalloc(&flag, 4));
    CK(hipMalloc(&polls, 4));
    CK(hipMemset(flag, 0, 4));
    CK(hipMemset(polls, 0xff, 4));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    hipGraph_t g = nullptr;
    hipGraphExec_t x = nullptr;
    if (graph) CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, s0));
    CK(hipStreamWaitEvent(s1, fork, 0));
    hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, s0, flag, polls);
    hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, s1, flag);
    CK(hipEventRecord(join, s1));
    CK(hipStreamWaitEvent(s0, join, 0));
    if (graph) {
        CK(hipStreamEndCapture(s0, &g));
        CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
        CK(hipMemset(flag, 0, 4));
        CK(hipDeviceSynchronize());
        CK(hipGraphLaunch(x, s0));
    }
    CK(hipStreamSynchronize(s0));
    int h = -1;
    CK(hipMemcpy(&h, polls, 4, hipMemcpyDeviceToHost));
    printf("%s: waiter polls %d (cap %d) -> %s\n", graph ? "graph" : "eager", h, MAX_POLLS,
           h < MAX_POLLS ? "concurrent" : "serialised");
    if (x) CK(hipGraphExecDestroy(x));
    if (g) CK(hipGraphDestroy(g));
    return 0;
}

int main() {
    if (run(false)) return 1;
    if (run(true)) return 1;
    return 0;
}

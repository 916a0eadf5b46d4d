// Can a dependent kernel chain overlap each kernel's launch and weight loads with its
// predecessor on MI355X? Chain of N weight-streaming kernels (B blocks x 256 threads,
// each block streams its own 16 KB weight slice from HBM, then folds a 1 KB input
// written by the previous kernel into its output). Variants, per kernel:
//  (a) one stream, plain stream order;
//  (b) one stream + the flag wait/signal code (always already satisfied);
//  (c) kernels alternating over two streams (fork/join in one captured graph): kernel i+1
//      starts while kernel i runs, issues its weight loads, then waits on kernel i's
//      completion counter (8 shards, one 128-B line each, sc1 polls + s_sleep, bounded)
//      before reading kernel i's output with sc1 loads. Outputs are sc1 (write-through).
// Prints us per kernel and whether every wait completed and every output is correct.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/micro_overlap tools/micro_overlap.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int SHARDS = 8, SSTRIDE = 32;   // counter shard i at ctr[i * 32] (own 128-B line)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    const uint64_t v = (uint64_t)p;
    return __builtin_amdgcn_make_buffer_rsrc((void*)v, 0, (int)bytes, 0x00020000);
}

__global__ __launch_bounds__(256) void stream_k(const u32x4* __restrict__ W, const uint32_t* in, uint32_t* out,
                                                 int* wait_ctr, int wait_target, int* sig_ctr, int* err, uint32_t salt) {
    const int tid = threadIdx.x;
    // 1. this block's 16 KB of weights: 4 x 16 B per thread, issued first
    const u32x4* wb = W + (size_t)blockIdx.x * 1024;
    u32x4 w[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) w[u] = __builtin_nontemporal_load(wb + tid + 256 * u);
    // 2. wait until every block of the previous kernel has signalled
    __shared__ int ok;
    if (wait_ctr) {
        if (tid == 0) {
            int spins = 0, tot = 0;
            for (;;) {
                tot = 0;
#pragma unroll
                for (int s = 0; s < SHARDS; ++s) tot += __hip_atomic_load(wait_ctr + s * SSTRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tot >= wait_target) break;
                if (++spins > (1 << 22)) { atomicOr(err, 1); break; }
                __builtin_amdgcn_s_sleep(1);
            }
            ok = 1;
        }
        __syncthreads();
    }
    // 3. the previous kernel's output (1 KB), sc1 loads (L1 bypass)
    const __amdgpu_buffer_rsrc_t ir = rsrc(in, 1024);
    const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(ir, (tid & 255) * 4, 0, 16);
    uint32_t acc = x;
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += w[u][0] ^ w[u][3];
    // 4. output: every block writes the same 1 KB (value = input + 1 + salt-independent term
    //    folded to 0 so it is checkable): out[t] = in[t] + 1
    const uint32_t val = x + 1u + (acc == 0x7fffffffu ? 1u : 0u);
    if (blockIdx.x == 0) {
        const __amdgpu_buffer_rsrc_t orr = rsrc(out, 1024);
        __builtin_amdgcn_raw_buffer_store_b32(val, orr, tid * 4, 0, 16);
    }
    (void)salt;
    // 5. signal: drain the sc1 stores, then one lane per block adds to its shard
    if (sig_ctr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(sig_ctr + (blockIdx.x % SHARDS) * SSTRIDE, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int main(int argc, char** argv) {
    const int N = 40;
    const int B = argc > 1 ? atoi(argv[1]) : 512;
    hipStream_t s0, s1;
    CHK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CHK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    // distinct weights per kernel (N x B x 16 KB), larger than the 256 MB Infinity Cache
    const size_t per_k = (size_t)B * 16384;
    u32x4* W;
    CHK(hipMalloc(&W, per_k * N));
    CHK(hipMemset(W, 0, per_k * N));
    uint32_t* io;   // N+1 buffers of 1 KB
    CHK(hipMalloc(&io, 1024 * (N + 1)));
    int* ctr;
    const size_t ctr_bytes = (size_t)N * SHARDS * SSTRIDE * 4;
    CHK(hipMalloc(&ctr, ctr_bytes));
    int* err;
    CHK(hipMalloc(&err, 4));
    hipEvent_t e0, e1, fork, join;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CHK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    auto kernel = [&](int i, hipStream_t s, bool flags) {
        hipLaunchKernelGGL(stream_k, dim3(B), dim3(256), 0, s, (const u32x4*)((char*)W + per_k * i),
                           (const uint32_t*)(io + 256 * i), io + 256 * (i + 1),
                           (flags && i > 0) ? ctr + (size_t)(i - 1) * SHARDS * SSTRIDE : (int*)nullptr, B,
                           flags ? ctr + (size_t)i * SHARDS * SSTRIDE : (int*)nullptr, err, 0u);
    };
    for (int mode = 0; mode < 3; ++mode) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
        CHK(hipMemsetAsync(ctr, 0, ctr_bytes, s0));
        CHK(hipMemsetAsync(io, 0, 1024, s0));
        if (mode < 2) {
            for (int i = 0; i < N; ++i) kernel(i, s0, mode == 1);
        } else {
            CHK(hipEventRecord(fork, s0));
            CHK(hipStreamWaitEvent(s1, fork, 0));
            for (int i = 0; i < N; ++i) kernel(i, (i & 1) ? s1 : s0, true);
            CHK(hipEventRecord(join, s1));
            CHK(hipStreamWaitEvent(s0, join, 0));
        }
        CHK(hipStreamEndCapture(s0, &g));
        CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CHK(hipMemset(err, 0, 4));
        for (int r = 0; r < 2; ++r) CHK(hipGraphLaunch(ge, s0));
        CHK(hipStreamSynchronize(s0));
        CHK(hipEventRecord(e0, s0));
        const int reps = 10;
        for (int r = 0; r < reps; ++r) CHK(hipGraphLaunch(ge, s0));
        CHK(hipEventRecord(e1, s0));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        int herr = 0;
        std::vector<uint32_t> last(256);
        CHK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        CHK(hipMemcpy(last.data(), io + 256 * N, 1024, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int t = 0; t < 256; ++t) bad += last[t] != (uint32_t)N;
        const char* names[] = {"one stream, plain", "one stream + wait/signal", "two streams, overlapped"};
        printf("B=%4d %-28s %7.2f us per kernel  (timeouts %d, wrong outputs %d)\n", B, names[mode],
               ms * 1000.f / (reps * N), herr, bad);
        hipGraphExecDestroy(ge);
        hipGraphDestroy(g);
    }
    return 0;
}

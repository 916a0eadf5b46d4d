// Address-translation cost on MI355X: dependent-load latency of one lane chasing a chain
// whose hops land (a) in one hot 64 KB block, (b) on new cache lines inside a 32 MB
// region (few 2 MB pages), (c) each on a different 2 MB page of a 6 GB region, and the
// duration of a 256-block launch whose blocks each read one 64 KB slice from a distinct
// 2 MB page vs from consecutive slices of a few pages.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/bin/micro_tlb tools/micro_tlb.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void chase(const uint64_t* __restrict__ buf, uint64_t start, int hops, uint64_t* out) {
    uint64_t cur = start;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < hops; ++i) cur = __builtin_nontemporal_load(buf + cur);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    out[0] = t1 - t0;
    out[1] = cur;
}

// each block streams 64 KB from base + blockIdx.x * stride
__global__ void slices(const uint4* __restrict__ buf, size_t stride_u4, uint4* out) {
    const uint4* p = buf + blockIdx.x * stride_u4;
    uint4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        uint4 v = p[threadIdx.x + 256 * i];
        acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
    }
    if (acc.x == 0x12345678u) out[blockIdx.x] = acc;
}

int main() {
    const size_t big = (size_t)6 << 30;   // 6 GB
    uint64_t* buf;
    CHK(hipMalloc(&buf, big));
    uint64_t* out;
    CHK(hipMalloc(&out, 64 * 1024));
    const size_t n = big / 8;
    // chains: index of next element stored at element
    auto build = [&](std::vector<std::pair<size_t, size_t>>& links) {
        for (auto& l : links) CHK(hipMemcpy(buf + l.first, &l.second, 8, hipMemcpyHostToDevice));
        return 0;
    };
    const int hops = 200;
    struct Case { const char* name; size_t stride; size_t region; };
    Case cases[] = {{"hot 64 KB block (stride 256 B, wraps)", 32, 8192},
                    {"new line, 32 MB region (stride 160 KB)", 20480, (size_t)4 << 20},
                    {"new 2 MB page each hop (stride 30 MB)", (size_t)30 << 17, n}};
    for (auto& c : cases) {
        std::vector<std::pair<size_t, size_t>> links;
        size_t cur = 0;
        for (int i = 0; i < hops; ++i) {
            size_t nx = (cur + c.stride) % c.region;
            links.push_back({cur, nx});
            cur = nx;
        }
        if (build(links)) return 1;
        uint64_t h[2];
        for (int r = 0; r < 3; ++r) {   // 3rd run: TLB / caches as warm as they get for this chain
            hipLaunchKernelGGL(chase, dim3(1), dim3(1), 0, 0, buf, (uint64_t)0, hops, out);
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
            printf("%-42s run %d: %7.1f ns per dependent load\n", c.name, r, h[0] * 10.0 / hops);
        }
    }
    // flush-ish: sweep 1 GB between measurements
    auto sweep = [&]() { hipLaunchKernelGGL(slices, dim3(16384), dim3(256), 0, 0, (const uint4*)buf + ((size_t)2 << 30) / 16, (size_t)4096, (uint4*)out); };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct S { const char* name; size_t stride_bytes; };
    S ss[] = {{"256 blocks x 64 KB, consecutive (16 MB, 8 pages)", 64 << 10},
              {"256 blocks x 64 KB, one 2 MB page each (512 MB)", 2 << 20},
              {"256 blocks x 64 KB, 20 MB apart (5 GB)", 20 << 20}};
    for (auto& s : ss) {
        for (int r = 0; r < 3; ++r) {
            sweep();
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(slices, dim3(256), dim3(256), 0, 0, (const uint4*)buf, s.stride_bytes / 16, (uint4*)out);
            hipEventRecord(e1, 0);
            CHK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("%-52s run %d: %7.2f us\n", s.name, r, ms * 1000.f);
        }
    }
    return 0;
}

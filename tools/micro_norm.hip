// The decode-step resid_norm (norm.hip, 8 rows x 2304, four fp32 split-K slabs in) as a
// dependent chain of N launches in one hipGraph, against the trivial-kernel floor of
// tools/micro_chain.hip: is its ~4.9 us in the step the kernel or the surroundings?
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I t5gemma-tts_amd/csrc \
//   tools/micro_norm.hip -o tools/bin/micro_norm
#include "../t5gemma-tts_amd/csrc/norm.hip"

#include <stdio.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

using namespace t5g;

int main() {
    const int M = 8, d = 2304, NS = 4, N = 200, REP = 20;
    float* part;
    bf16_t *w1, *w2, *h0, *h1, *xn;
    CK(hipMalloc(&part, (size_t)NS * M * d * 4));
    CK(hipMalloc(&w1, d * 2));
    CK(hipMalloc(&w2, d * 2));
    CK(hipMalloc(&h0, M * d * 2));
    CK(hipMalloc(&h1, M * d * 2));
    CK(hipMalloc(&xn, M * d * 2));
    CK(hipMemset(part, 0, (size_t)NS * M * d * 4));
    CK(hipMemset(w1, 0, d * 2));
    CK(hipMemset(w2, 0, d * 2));
    CK(hipMemset(h0, 0, M * d * 2));
    CK(hipMemset(h1, 0, M * d * 2));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int variant = 0; variant < 3; ++variant) {
        hipGraph_t g = nullptr;
        hipGraphExec_t ge = nullptr;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < N; ++i) {
            NormArgs n;
            memset(&n, 0, sizeof(n));
            n.M = M;
            n.d = d;
            n.eps = 1e-6f;
            if (variant == 2) {
                n.delta = xn;   // bf16 delta instead of slabs
            } else {
                n.part = part;
                n.nsplit = variant == 0 ? NS : 1;
                n.ldp = d;
            }
            n.post_w = w1;
            n.resid = (i & 1) ? h1 : h0;
            n.pre_w = w2;
            n.resid_out = (i & 1) ? h0 : h1;
            n.normed_out = variant == 2 ? (bf16_t*)part : xn;
            if (resid_norm(n, st)) { printf("launch failed\n"); return 1; }
        }
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int r = 0; r < REP; ++r) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const char* vn[3] = {"4 fp32 slabs + post + resid + pre", "1 fp32 slab + post + resid + pre", "bf16 delta + post + resid + pre"};
        printf("{\"variant\": \"resid_norm chain, %s\", \"us_per_launch\": %.3f}\n", vn[variant], ms * 1000.f / (N * REP));
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    return 0;
}

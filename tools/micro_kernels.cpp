// Per-kernel latency of the decode-step kernels in isolation (hipGraph of back-to-back
// launches, like the engine's captured decode iteration), at the 2b-2b decode shapes
// (B = 8, d = 2304, 8 q / 4 kv heads x 256). Links libt5gtts.so's internal launchers.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I t5gemma-tts_amd/csrc \
//        tools/micro_kernels.cpp -L t5gemma-tts_amd/lib -lt5gtts -Wl,-rpath,$PWD/t5gemma-tts_amd/lib \
//        -o tools/bin/micro_kernels
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <functional>
#include <vector>

#include "t5g_kernels.h"

using namespace t5g;

static float time_graph(hipStream_t st, int n, const std::function<void(int)>& launch) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int i = 0; i < n; ++i) launch(i);
    hipStreamEndCapture(st, &g);
    if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) return -1.f;
    hipGraphLaunch(ge, st);
    hipStreamSynchronize(st);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    for (int r = 0; r < 5; ++r) hipGraphLaunch(ge, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    return ms * 1000.f / (5 * n);
}

template <typename T>
static T* dalloc(size_t n) {
    void* p = nullptr;
    hipMalloc(&p, n * sizeof(T));
    hipMemset(p, 0, n * sizeof(T));
    return (T*)p;
}

int main() {
    hipStream_t st;
    hipStreamCreate(&st);
    const int B = 8, d = 2304, D = 256, Hq = 8, Hkv = 4, G = 2, Lmax = 1024, Tx = 64;
    const int qdim = Hq * D, kvdim = Hkv * D, qkv = qdim + 2 * kvdim;
    // activations / slabs
    bf16_t* h = dalloc<bf16_t>(B * d);
    bf16_t* xn = dalloc<bf16_t>(B * d);
    bf16_t* w1 = dalloc<bf16_t>(d);
    bf16_t* w2 = dalloc<bf16_t>(d);
    float* part = dalloc<float>(8 * B * 4096);
    float* apart = dalloc<float>((size_t)B * Hkv * 16 * G * (D + 2));
    bf16_t* att = dalloc<bf16_t>(B * qdim);
    bf16_t* Kc = dalloc<bf16_t>((size_t)B * Hkv * Lmax * D);
    bf16_t* Vc = dalloc<bf16_t>((size_t)B * Hkv * Lmax * D);
    bf16_t* Kx = dalloc<bf16_t>((size_t)B * Hkv * Tx * D);
    bf16_t* Vx = dalloc<bf16_t>((size_t)B * Hkv * Tx * D);
    int* kv_len = dalloc<int>(B);
    int* x_len = dalloc<int>(B);
    float* pos = dalloc<float>(B);
    float* inv_freq = dalloc<float>(D / 2);
    float* tab = dalloc<float>(B * D);
    std::vector<int> hl(B, 527), hx(B, 60);
    hipMemcpy(kv_len, hl.data(), B * 4, hipMemcpyHostToDevice);
    hipMemcpy(x_len, hx.data(), B * 4, hipMemcpyHostToDevice);
    const int n = 200;

    // ---- norms
    auto norm = [&](int nsplit, bool post) {
        NormArgs a;
        memset(&a, 0, sizeof(a));
        a.M = B;
        a.d = d;
        a.eps = 1e-6f;
        if (nsplit) {
            a.part = part;
            a.nsplit = nsplit;
            a.ldp = d;
        } else {
            a.delta = xn;
        }
        a.post_w = post ? w1 : nullptr;
        a.resid = h;
        a.pre_w = w2;
        a.resid_out = h;
        a.normed_out = xn;
        return a;
    };
    {
        NormArgs a = norm(4, true);
        printf("resid_norm part4+post+pre : %6.2f us\n", time_graph(st, n, [&](int) { resid_norm(a, st); }));
        NormArgs b = norm(8, true);
        printf("resid_norm part8+post+pre : %6.2f us\n", time_graph(st, n, [&](int) { resid_norm(b, st); }));
        NormArgs c = norm(0, false);
        printf("resid_norm delta+pre      : %6.2f us\n", time_graph(st, n, [&](int) { resid_norm(c, st); }));
    }
    // ---- attention decode
    auto attn = [&](bool cross, bool qpart, int nsplit) {
        AttnArgs a;
        memset(&a, 0, sizeof(a));
        a.Q = att;
        a.ldq = qdim;
        a.Mq = B;
        a.K = cross ? Kx : Kc;
        a.V = cross ? Vx : Vc;
        a.kv_hstride = (long)(cross ? Tx : Lmax) * D;
        a.kv_bstride = a.kv_hstride * Hkv;
        a.kv_len = cross ? x_len : kv_len;
        a.Hkv = Hkv;
        a.D = D;
        a.G = G;
        a.causal = cross ? 0 : 1;
        a.scale = 1.0f / 16;
        a.chunk = 64;
        a.nsplit = nsplit;
        a.kv_cap = cross ? Tx : Lmax;
        a.part = apart;
        a.O = att;
        a.ldo = qdim;
        if (qpart) {
            a.Qpart = part;
            a.q_nsplit = cross ? 4 : 2;
            a.ldqp = cross ? qdim : qkv;
            a.pos = pos;
            a.inv_freq = inv_freq;
            a.rope_tab = tab;
        }
        return a;
    };
    {
        AttnArgs a = attn(false, true, 16);
        printf("attn self  L=527 16 splits: %6.2f us (incl. combine)\n",
               time_graph(st, n, [&](int) { attention_decode(a, st); }));
        AttnArgs a2 = attn(false, true, 9);
        printf("attn self  L=527  9 splits: %6.2f us (incl. combine)\n",
               time_graph(st, n, [&](int) { attention_decode(a2, st); }));
        AttnArgs b = attn(true, true, 1);
        printf("attn cross Tx=60 1 split  : %6.2f us\n", time_graph(st, n, [&](int) { attention_decode(b, st); }));
        AttnArgs c = attn(true, false, 1);
        printf("attn cross Tx=60 q direct : %6.2f us\n", time_graph(st, n, [&](int) { attention_decode(c, st); }));
    }
    // ---- rope table + rope store
    printf("rope_table                : %6.2f us\n",
           time_graph(st, n, [&](int) { rope_table(pos, inv_freq, B, D, tab, st); }));
    {
        RopeArgs r;
        memset(&r, 0, sizeof(r));
        r.Xpart = part;
        r.nsplit = 2;
        r.ldx = qkv;
        r.M = B;
        r.D = D;
        r.nk = Hkv;
        r.nv = Hkv;
        r.col0 = qdim;
        r.rope_q = r.rope_k = 1;
        r.pos = pos;
        r.inv_freq = inv_freq;
        r.kv_len = kv_len;
        r.rope_tab = tab;
        r.Qout = att;
        r.ldq = qdim;
        r.Kc = Kc;
        r.Vc = Vc;
        r.c_hstride = (long)Lmax * D;
        r.c_bstride = r.c_hstride * Hkv;
        printf("rope_store k/v            : %6.2f us\n", time_graph(st, n, [&](int) { rope_store(r, st); }));
    }
    // ---- GEMMs with rotating weights (26 layers, HBM-cold)
    auto gemm_case = [&](const char* name, int N, int K, int splits, int epi) {
        const int nl = 26;
        const int ng = ((N + 15) / 16 + 3) / 4 * 4;
        std::vector<bf16_t*> W(nl);
        for (int l = 0; l < nl; ++l) W[l] = dalloc<bf16_t>((size_t)ng * 16 * K);
        void* Y = dalloc<float>((size_t)splits * B * N + 16);
        bf16_t* X = dalloc<bf16_t>((size_t)B * K);
        GemmArgs g;
        memset(&g, 0, sizeof(g));
        g.X = X;
        g.ldx = K;
        g.M = B;
        g.N = N;
        g.NG = ng;
        g.KB = K / 32;
        g.splits = splits;
        g.Y = Y;
        g.ldy = epi == EPI_GEGLU ? N / 2 : N;
        const double bytes = (double)N * K * 2;
        float us = time_graph(st, 208, [&](int i) {
            g.W = W[i % nl];
            gemm_p16(g, epi, st);
        });
        printf("gemm %-22s: %6.2f us  %7.1f GB/s\n", name, us, bytes / us / 1e3);
        for (auto p : W) hipFree(p);
        hipFree(Y);
        hipFree(X);
    };
    gemm_case("qkv 4096x2304 s2", qkv, d, 2, EPI_F32);
    gemm_case("qkv 4096x2304 s4", qkv, d, 4, EPI_F32);
    gemm_case("o 2304x2048 s4", d, qdim, 4, EPI_F32);
    gemm_case("o 2304x2048 s8", d, qdim, 8, EPI_F32);
    gemm_case("o 2304x2048 s2", d, qdim, 2, EPI_F32);
    gemm_case("gate_up 18432x2304", 2 * 9216, d, 1, EPI_GEGLU);
    gemm_case("down 2304x9216 s8", d, 9216, 8, EPI_F32);
    gemm_case("down 2304x9216 s16", d, 9216, 16, EPI_F32);
    gemm_case("down 2304x9216 s4", d, 9216, 4, EPI_F32);
    return 0;
}

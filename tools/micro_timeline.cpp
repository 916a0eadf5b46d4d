// Block-level timeline of one T5Gemma 2b-2b decoder layer at batch 8 (decode step), the
// same kernel chain the engine captures (engine.hip decoder_pass), run on the diagnostic
// library variant (build.py --dbg: every block of the instrumented kernels records the
// 100 MHz device clock at numbered points, common.h T5G_TS). For the third of four layers
// (distinct weights per layer, HBM-cold like inside a 26-layer step) it prints, per
// kernel: first/last block start and end relative to the layer start, the gap from the
// previous kernel's last block end, median block time and its in-block phases, and how
// many blocks the busiest CU ran.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I t5gemma-tts_amd/csrc \
//   tools/micro_timeline.cpp -L t5gemma-tts_amd/lib -lt5gtts_dbg -Wl,-rpath,$PWD/t5gemma-tts_amd/lib \
//   -o tools/bin/micro_timeline
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <vector>

#include "t5g_kernels.h"

using namespace t5g;

extern "C" int t5g_dbg_set_gemm(void*);
extern "C" int t5g_dbg_set_norm(void*);
extern "C" int t5g_dbg_set_attn(void*);

template <typename T>
static T* dalloc(size_t n, float fill = 0.f) {
    void* p = nullptr;
    if (hipMalloc(&p, n * sizeof(T)) != hipSuccess) { printf("oom\n"); exit(1); }
    hipMemset(p, 0, n * sizeof(T));
    return (T*)p;
}

static const int SEQ_PER_LAYER = 16, MAXB = 4096;

// side-branch prefetch: block b reads its share of [p, p + bytes) with default-policy
// loads (allocating in the Infinity Cache) and folds it into a never-taken store
__global__ __launch_bounds__(256) void prefetch_kernel(const uint4* __restrict__ p, size_t n16, uint4* sink) {
    const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const size_t lo = (size_t)blockIdx.x * per, hi = lo + per < n16 ? lo + per : n16;
    uint32_t acc = 0;
    for (size_t i = lo + threadIdx.x; i < hi; i += 256 * 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const size_t j = i + 256 * u;
            if (j < hi) { const uint4 v = p[j]; acc ^= v.x ^ v.w; }
        }
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = make_uint4(acc, 0, 0, 0);
}

int main(int argc, char** argv) {
    const int L_self = argc > 1 ? atoi(argv[1]) : 527;
    const int tickets = argc > 2 ? atoi(argv[2]) : 0;     // in-launch attention merge
    const int x_split = argc > 3 ? atoi(argv[3]) : 1;     // cross-attention key splits
    const int pf_blocks = argc > 4 ? atoi(argv[4]) : 0;   // side-branch MALL prefetch of the MLP weights
    hipStream_t st;
    hipStreamCreate(&st);
    const int B = 8, d = 2304, f = 9216, D = 256, Hq = 8, Hkv = 4, G = 2, Lmax = 911, Tx = 64, nl = 4;
    const int qdim = Hq * D, kvdim = Hkv * D, qkv = qdim + 2 * kvdim;
    auto ng = [](int N) { return ((N + 15) / 16 + 3) / 4 * 4; };
    struct LW { bf16_t *qkv, *o, *cq, *co, *gu, *down, *kc, *vc, *xk, *xv, *pw, *qw; };
    std::vector<LW> lw(nl);
    for (auto& w : lw) {
        w.qkv = dalloc<bf16_t>((size_t)ng(qkv) * 16 * d);
        w.o = dalloc<bf16_t>((size_t)ng(d) * 16 * qdim);
        w.cq = dalloc<bf16_t>((size_t)ng(qdim) * 16 * d);
        w.co = dalloc<bf16_t>((size_t)ng(d) * 16 * qdim);
        w.gu = dalloc<bf16_t>((size_t)ng(2 * f) * 16 * d);
        w.down = dalloc<bf16_t>((size_t)ng(d) * 16 * f);
        w.kc = dalloc<bf16_t>((size_t)B * Hkv * Lmax * D);
        w.vc = dalloc<bf16_t>((size_t)B * Hkv * Lmax * D);
        w.xk = dalloc<bf16_t>((size_t)B * Hkv * Tx * D);
        w.xv = dalloc<bf16_t>((size_t)B * Hkv * Tx * D);
        w.pw = dalloc<bf16_t>(d);
        w.qw = dalloc<bf16_t>(d);
    }
    bf16_t* h = dalloc<bf16_t>(B * d);
    bf16_t* xn = dalloc<bf16_t>(B * d);
    bf16_t* att = dalloc<bf16_t>(B * qdim);
    bf16_t* act = dalloc<bf16_t>(B * f);
    float* part = dalloc<float>((size_t)8 * B * qkv);
    float* apart = dalloc<float>((size_t)B * Hkv * 16 * G * (D + 2));
    int* kv_len = dalloc<int>(B);
    int* x_len = dalloc<int>(B);
    int* ctr = dalloc<int>(B * Hkv);
    float* pos = dalloc<float>(B);
    float* inv_freq = dalloc<float>(D / 2);
    float* tab = dalloc<float>(B * D);
    std::vector<int> hl(B, L_self), hx(B, 60);
    hipMemcpy(kv_len, hl.data(), B * 4, hipMemcpyHostToDevice);
    hipMemcpy(x_len, hx.data(), B * 4, hipMemcpyHostToDevice);
    const size_t nseq = (size_t)nl * SEQ_PER_LAYER;
    const size_t words = nseq * MAXB * 8;
    unsigned long long *tg = dalloc<unsigned long long>(words), *tn = dalloc<unsigned long long>(words),
                       *ta = dalloc<unsigned long long>(words);
    t5g_dbg_set_gemm(tg);
    t5g_dbg_set_norm(tn);
    t5g_dbg_set_attn(ta);

    auto gemm = [&](const bf16_t* X, int ldx, const bf16_t* W, int N, int K, int splits, void* Y, int ldy, int epi,
                    int seq) {
        GemmArgs g;
        memset(&g, 0, sizeof(g));
        g.X = X; g.ldx = ldx; g.M = B; g.W = W; g.N = N; g.NG = ng(N); g.KB = K / 32; g.splits = splits;
        g.Y = Y; g.ldy = ldy; g.dbg_seq = seq;
        if (gemm_p16(g, epi, st)) printf("gemm launch failed seq %d\n", seq);
    };
    auto norm = [&](int nsplit, const LW& w, int seq) {
        NormArgs a;
        memset(&a, 0, sizeof(a));
        a.M = B; a.d = d; a.eps = 1e-6f; a.part = part; a.nsplit = nsplit; a.ldp = d;
        a.post_w = w.pw; a.resid = h; a.pre_w = w.qw; a.resid_out = h; a.normed_out = xn; a.dbg_seq = seq;
        if (resid_norm(a, st)) printf("norm launch failed\n");
    };
    auto attn = [&](bool cross, const LW& w, int seq) {
        AttnArgs a;
        memset(&a, 0, sizeof(a));
        a.Q = att; a.ldq = qdim; a.Mq = B;
        a.K = cross ? w.xk : w.kc; a.V = cross ? w.xv : w.vc;
        a.kv_hstride = (long)(cross ? Tx : Lmax) * D; a.kv_bstride = a.kv_hstride * Hkv;
        a.kv_len = cross ? x_len : kv_len; a.Hkv = Hkv; a.D = D; a.G = G; a.causal = cross ? 0 : 1;
        a.scale = 1.0f / 16; a.chunk = 64; a.nsplit = cross ? x_split : (Lmax + 63) / 64; a.kv_cap = cross ? Tx : Lmax;
        a.counters = tickets ? ctr : nullptr;
        a.part = apart; a.O = att; a.ldo = qdim;
        a.Qpart = part; a.q_nsplit = cross ? 4 : 2; a.ldqp = cross ? qdim : qkv;
        a.pos = pos; a.inv_freq = inv_freq; a.rope_tab = tab;
        if (!cross) { a.append = 1; a.k_col0 = qdim; a.v_col0 = qdim + kvdim; }
        a.dbg_seq = seq;
        if (attention_decode(a, st)) printf("attn launch failed\n");
    };
    hipStream_t side;
    hipStreamCreateWithFlags(&side, hipStreamNonBlocking);
    hipEvent_t evf[8], evj[8];
    for (int i = 0; i < 8; ++i) {
        hipEventCreateWithFlags(&evf[i], hipEventDisableTiming);
        hipEventCreateWithFlags(&evj[i], hipEventDisableTiming);
    }
    uint4* sink = dalloc<uint4>(4096);
    auto layer = [&](int l) {
        const LW& w = lw[l];
        const int s = l * SEQ_PER_LAYER;
        if (pf_blocks > 0) {
            // fork: the side stream streams this layer's gate/up + down weights into the
            // Infinity Cache while the attention half of the layer runs
            hipEventRecord(evf[l], st);
            hipStreamWaitEvent(side, evf[l], 0);
            hipLaunchKernelGGL(prefetch_kernel, dim3(pf_blocks), dim3(256), 0, side, (const uint4*)w.gu,
                               (size_t)ng(2 * f) * 16 * d * 2 / 16, sink);
            hipLaunchKernelGGL(prefetch_kernel, dim3(pf_blocks), dim3(256), 0, side, (const uint4*)w.down,
                               (size_t)ng(d) * 16 * f * 2 / 16, sink);
            hipEventRecord(evj[l], side);
        }
        gemm(xn, d, w.qkv, qkv, d, 2, part, qkv, EPI_F32, s + 0);
        attn(false, w, s + 1);
        gemm(att, qdim, w.o, d, qdim, 4, part, d, EPI_F32, s + 2);
        norm(4, w, s + 3);
        gemm(xn, d, w.cq, qdim, d, 4, part, qdim, EPI_F32, s + 4);
        attn(true, w, s + 5);
        gemm(att, qdim, w.co, d, qdim, 4, part, d, EPI_F32, s + 6);
        norm(4, w, s + 7);
        gemm(xn, d, w.gu, 2 * f, d, 1, act, f, EPI_GEGLU, s + 8);
        gemm(act, f, w.down, d, f, 8, part, d, EPI_F32, s + 9);
        norm(8, w, s + 10);
        if (pf_blocks > 0) hipStreamWaitEvent(st, evj[l], 0);   // join before the next layer
    };
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int l = 0; l < nl; ++l) layer(l);
    hipStreamEndCapture(st, &g);
    if (hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) { printf("instantiate failed\n"); return 1; }
    for (int r = 0; r < 3; ++r) hipGraphLaunch(ge, st);
    hipStreamSynchronize(st);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    const int reps = 10;
    for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("prefetch blocks %d, ", pf_blocks);
    printf("L_self %d tickets %d x_split %d: %.1f us per layer (graph of %d layers, event-timed)\n", L_self, tickets,
           x_split, ms * 1000.f / (reps * nl), nl);
    for (auto* p : {tg, tn, ta}) hipMemsetAsync(p, 0, words * 8, st);
    hipGraphLaunch(ge, st);
    if (hipStreamSynchronize(st) != hipSuccess) { printf("run failed\n"); return 1; }
    std::vector<unsigned long long> hg(words), hn(words), ha(words);
    hipMemcpy(hg.data(), tg, words * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hn.data(), tn, words * 8, hipMemcpyDeviceToHost);
    hipMemcpy(ha.data(), ta, words * 8, hipMemcpyDeviceToHost);

    struct K { const char* name; std::vector<unsigned long long>* buf; int seq, start, end; std::vector<int> mids; };
    const int l = 2, s = l * SEQ_PER_LAYER;
    std::vector<K> ks = {
        {"qkv gemm s2", &hg, s + 0, 0, 3, {1, 2}}, {"self attn", &ha, s + 1, 0, 5, {1, 2, 4}},
        {"  combine", &ha, s + 1, 3, 6, {}}, {"o gemm s4", &hg, s + 2, 0, 3, {1, 2}},
        {"norm p4", &hn, s + 3, 0, 2, {1}}, {"cq gemm s4", &hg, s + 4, 0, 3, {1, 2}},
        {"cross attn", &ha, s + 5, 0, 5, {1, 2, 4}}, {"  x-combine", &ha, s + 5, 3, 6, {}}, {"co gemm s4", &hg, s + 6, 0, 3, {1, 2}},
        {"norm p4", &hn, s + 7, 0, 2, {1}}, {"gate_up gemm", &hg, s + 8, 0, 3, {1, 2}},
        {"down gemm s8", &hg, s + 9, 0, 3, {1, 2}}, {"norm p8", &hn, s + 10, 0, 2, {1}}};
    unsigned long long t0 = ~0ull;
    for (auto& k : ks)
        for (int b = 0; b < MAXB; ++b) {
            unsigned long long v = (*k.buf)[((size_t)k.seq * MAXB + b) * 8 + k.start];
            if (v) t0 = std::min(t0, v);
        }
    double prev_end = 0;
    printf("%-14s %6s %8s %8s %8s %8s %7s %8s  %s\n", "kernel", "blocks", "start0", "startN", "end0", "endN", "gap",
           "blk_med", "phases(med, from block start) | max blocks/CU");
    for (auto& k : ks) {
        std::vector<double> st0, en, dur;
        std::vector<std::vector<double>> mid(k.mids.size());
        std::map<unsigned long long, int> cu;
        for (int b = 0; b < MAXB; ++b) {
            const size_t base = ((size_t)k.seq * MAXB + b) * 8;
            unsigned long long a0 = (*k.buf)[base + k.start], a1 = (*k.buf)[base + k.end];
            if (!a0 || !a1) continue;
            st0.push_back((a0 - t0) / 100.0);
            en.push_back((a1 - t0) / 100.0);
            dur.push_back((a1 - a0) / 100.0);
            for (size_t i = 0; i < k.mids.size(); ++i) {
                unsigned long long m = (*k.buf)[base + k.mids[i]];
                if (m) mid[i].push_back((m - a0) / 100.0);
            }
            const unsigned long long hw = (*k.buf)[base + 7];
            const unsigned long long cukey = ((hw >> 32) << 16) | ((hw >> 8) & 0xffff & ~0x0u) ;
            cu[((hw >> 32) << 16) | (((hw & 0xffffffffull) >> 8) & 0x3f) | ((((hw & 0xffffffffull) >> 13) & 7) << 8)]++;
            (void)cukey;
        }
        if (st0.empty()) { printf("%-14s no records\n", k.name); continue; }
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        const double s0 = *std::min_element(st0.begin(), st0.end()), sN = *std::max_element(st0.begin(), st0.end());
        const double e0 = *std::min_element(en.begin(), en.end()), eN = *std::max_element(en.begin(), en.end());
        int mx = 0;
        for (auto& kv : cu) mx = std::max(mx, kv.second);
        printf("%-14s %6zu %8.2f %8.2f %8.2f %8.2f %7.2f %8.2f  ", k.name, st0.size(), s0, sN, e0, eN, s0 - prev_end,
               med(dur));
        for (auto& m : mid) printf("%6.2f ", m.empty() ? -1.0 : med(m));
        printf("| %d on %zu CUs\n", mx, cu.size());
        prev_end = eN;
    }
    return 0;
}

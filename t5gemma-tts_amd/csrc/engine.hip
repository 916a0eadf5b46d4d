// Engine: owns the HBM arena (KV caches, activations, sampler state) and runs the
// T5Gemma-TTS generate() phases as sequences of the gfx950 kernels; the decode
// iteration (sampler + 26-layer single-token step + predict head) is captured
// once into a hipGraph and replayed, with all per-step scalars (lengths,
// positions, tokens) living in device memory so the graph is static.
//
// Call-stack correspondence (reference hf_export/modeling_t5gemma_voice.py):
//   t5g_encode   -> :596-615 encoder + :198-230 cross K/V (computed once per call)
//   t5g_prefill  -> :630-694 BOS+prompt decoder pass, :693 last hidden, :789 head
//   t5g_decode   -> :788-848 loop body (sample_helper, embedding, decoder step)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#include <vector>

#include "../../include/t5gtts.h"
#include "t5g_kernels.h"

using namespace t5g;

#define HIPCHK(x)                                  \
    do {                                           \
        if ((x) != hipSuccess) return T5G_EHIP;    \
    } while (0)
#define RC(x)                       \
    do {                            \
        int _rc = (x);              \
        if (_rc) return _rc == -1 ? T5G_EINVAL : (_rc == -3 ? T5G_EUNSUPPORTED : T5G_EHIP); \
    } while (0)

static inline int ng_pad(int N) { return ((N + 15) / 16 + 3) / 4 * 4; }

struct t5g_engine {
    t5g_config c;
    t5g_weights w;
    std::vector<t5g_layer_weights> enc, dec;
    int q_dim, kv_dim, qkv_dim, V, Vpad;
    int max_tok;  // packed token capacity for encode / prefill
    // arena
    std::vector<void*> allocs;
    int64_t bytes = 0;
    // packed-token activations (encode / prefill)
    bf16_t *h, *xn, *qkv, *q, *att, *act, *tmp, *mem;
    float* part;          // split-K slabs (max over uses)
    float* apart;         // attention partials
    int64_t part_elems, apart_elems;
    bf16_t *enc_k, *enc_v;                 // encoder self K/V [B][Hkv][max_text][D]
    std::vector<bf16_t*> ck, cv, sk, sv;   // per decoder layer cross / self caches
    int* enc_len;                          // [B] text lengths
    // decode (rows = max_batch)
    bf16_t *dh, *dxn, *dq, *datt, *dact, *dhh, *logits;
    bf16_t *dh2, *dv;     // fused decode: second residual buffer, sub-block output rows
    // Decode-step GEMV variant, chosen at creation by T5G_FUSED_DECODE (measured on MI355X,
    // tools/micro_gemv.py): unset/0 = split-K MFMA GEMVs + separate norm
    // kernels (fastest); 1 = norm prologues fused into row-major VALU GEMVs; 2 = fused
    // prologues on the P16 MFMA GEMVs.
    bool fused_decode = false;
    bool fused_p16 = false;
    int logits_ld;
    // sampler
    SamplerRow* rows;
    SamplerState* state;
    int* topk_list;
    int* silence;
    int* out_tokens;
    int* kv_len;
    float* next_pos;
    int* next_token;
    int* flags;
    int* last_rows;
    int* attn_tickets_buf;  // [max_batch][Hkv] in-launch split-merge counters (self-re-arming)
    float* rope_tab;    // [max_batch][D] per-row cos|sin of the decode step's PM position
    // multi-block sampler scratch (sampler.hip fast path)
    float* fs_val;
    int* fs_idx;
    int* fs_cnt;
    float* fs_amv;
    int* fs_ami;
    unsigned* fs_ticket;
    int* fs_slow;
    bool fast_sampler = true;   // T5G_SAMPLER_FAST=0 at creation: single-block sampler only
    // decode attention: key-split partials merged in-launch by the last block of each
    // (row, kv head) (T5G_ATTN_TICKETS=1) instead of a combine launch; cross attention
    // keys split over T5G_XATTN_SPLIT blocks per (row, kv head). Both off by default:
    // measured on MI355X (tools/micro_timeline.cpp) neither beats the combine launch.
    bool attn_tickets = false;
    // decode gate/up on gemv_dec (one block per CU, 1152 single-group units dealt
    // round-robin: 18.3 us vs 19.7 us for the 576-block P16 GEMM); T5G_GU_GEMV=0 reverts
    bool gu_gemv = true;
    bool down_gemv = false;   // T5G_DOWN_GEMV=1: decode down projection on gemv_dec split-K (probe)
    int s_down = 8;           // decode down-projection k-slices (T5G_S_DOWN, 2..8; probe)
    int s_qkv = 2, s_o = 4;   // decode qkv / (o, cross-q, cross-o) k-slices (T5G_S_QKV, T5G_S_O, 2..4 = QSMAX; probe)
    // decode norms folded into the consuming GEMV (PRO_LEAD: blocks 0..M-1 finish and
    // publish the rows, the others poll per-row flags): one launch fewer per site.
    // T5G_LEAD_NORM = site mask (1 next-layer qkv, 2 cross-q, 4 gate/up). Off by default:
    // measured on MI355X the in-launch hand-off costs what the launch boundary did
    // (gate/up 23.2 us vs 18.0 + 4.9 norm; all sites 3019 vs 3411 tok/s).
    int lead_sites = 0;
    unsigned* lead_flags = nullptr;   // [n_dec_layers][3 sites][16 rows]: last published epoch
    unsigned* lead_epoch = nullptr;   // step epoch, advanced by the step's rope_table launch
    unsigned* lead_tmo = nullptr;     // poll give-up word (t5g_engine_status)
    float* qslab = nullptr;           // [max_batch][qkv_dim] fp32 q|k|v of the lead GEMVs
    int xsplit = 1;
    int B = 0;            // rows of the current call
    const bf16_t* noise = nullptr;
    int noise_steps = 0;
    // graph
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    int graph_B = -1;
    hipStream_t graph_stream = nullptr;
    hipStream_t cap_stream = nullptr;
};

template <typename T>
static int alloc(t5g_engine* e, T** p, int64_t n) {
    void* ptr = nullptr;
    int64_t bytes = ((n * (int64_t)sizeof(T)) + 255) / 256 * 256;
    if (hipMalloc(&ptr, (size_t)bytes) != hipSuccess) return T5G_ENOMEM;
    hipMemset(ptr, 0, (size_t)bytes);
    e->allocs.push_back(ptr);
    e->bytes += bytes;
    *p = (T*)ptr;
    return 0;
}

extern "C" int64_t t5g_packed_bytes(int32_t N, int32_t K) {
    if (K % 32) return -1;
    return (int64_t)ng_pad(N) * 16 * K * 2;
}

extern "C" int t5g_pack_weight(const void* src, int32_t N, int32_t K, int64_t ld, void* dst, void* stream) {
    if (!src || !dst || N <= 0 || K <= 0 || K % 32) return T5G_EINVAL;
    RC(pack_p16((const bf16_t*)src, N, K, ld, (bf16_t*)dst, ng_pad(N), (hipStream_t)stream));
    return T5G_OK;
}

extern "C" int t5g_engine_destroy(t5g_engine* e) {
    if (!e) return T5G_OK;
    if (e->gexec) hipGraphExecDestroy(e->gexec);
    if (e->graph) hipGraphDestroy(e->graph);
    if (e->cap_stream) hipStreamDestroy(e->cap_stream);
    for (void* p : e->allocs) hipFree(p);
    delete e;
    return T5G_OK;
}

extern "C" int64_t t5g_engine_workspace_bytes(const t5g_engine* e) { return e ? e->bytes : -1; }

extern "C" int t5g_engine_create(const t5g_config* cfg, const t5g_weights* w, t5g_engine** out) {
    if (!cfg || !w || !out) return T5G_EINVAL;
    const t5g_config& c = *cfg;
    if (c.hidden % 32 || c.intermediate % 32 || c.n_enc_layers > T5G_MAX_LAYERS ||
        c.n_dec_layers > T5G_MAX_LAYERS || c.max_batch <= 0 || c.max_text <= 0 || c.max_audio <= 0 ||
        c.n_heads % c.n_kv_heads || c.max_audio > 4096 || c.max_text > 4096)
        return T5G_EINVAL;
    t5g_engine* e = new t5g_engine();
    e->c = c;
    e->w = *w;
    e->enc.assign(w->enc_layers, w->enc_layers + c.n_enc_layers);
    e->dec.assign(w->dec_layers, w->dec_layers + c.n_dec_layers);
    e->q_dim = c.n_heads * c.head_dim;
    e->kv_dim = c.n_kv_heads * c.head_dim;
    e->qkv_dim = e->q_dim + 2 * e->kv_dim;
    e->V = c.n_audio_tokens;
    e->Vpad = ng_pad(e->V) * 16;
    const int B = c.max_batch, d = c.hidden, f = c.intermediate, D = c.head_dim, Hkv = c.n_kv_heads;
    e->max_tok = B * (c.max_text > c.max_audio ? c.max_text : c.max_audio);
    const int64_t T = e->max_tok;
    int rc = 0;
    auto widest = [&](int64_t a, int64_t b) { return a > b ? a : b; };
    rc |= alloc(e, &e->h, T * d);
    rc |= alloc(e, &e->xn, T * d);
    rc |= alloc(e, &e->qkv, T * widest(e->qkv_dim, 2 * e->kv_dim));
    rc |= alloc(e, &e->q, T * e->q_dim);
    rc |= alloc(e, &e->att, T * e->q_dim);
    rc |= alloc(e, &e->act, T * f);
    rc |= alloc(e, &e->tmp, T * widest(widest(d, e->qkv_dim), 2 * e->kv_dim));
    rc |= alloc(e, &e->mem, (int64_t)B * c.max_text * d);
    // split-K slabs: decode uses up to 8 splits of [B][max(d, qkv)]
    e->part_elems = (int64_t)8 * B * widest(widest(d, e->qkv_dim), 2 * e->kv_dim);
    rc |= alloc(e, &e->part, e->part_elems);
    rc |= alloc(e, &e->lead_flags, (int64_t)c.n_dec_layers * 3 * 16);
    rc |= alloc(e, &e->lead_tmo, 4);
    rc |= alloc(e, &e->lead_epoch, 4);
    rc |= alloc(e, &e->qslab, (int64_t)B * widest(e->qkv_dim, d));
    const int G = c.n_heads / c.n_kv_heads;
    const int nsplit_dec = (c.max_audio + 63) / 64;
    // cross-attention key splits: up to max(ceil(max_text / 64), 16) (T5G_XATTN_SPLIT cap)
    const int nsplit_x = (c.max_text + 63) / 64 > 16 ? (c.max_text + 63) / 64 : 16;
    e->apart_elems = (int64_t)B * Hkv * (nsplit_dec > nsplit_x ? nsplit_dec : nsplit_x) * G * (D + 2);
    rc |= alloc(e, &e->apart, e->apart_elems);
    const int64_t enc_cache = (int64_t)B * Hkv * c.max_text * D;
    rc |= alloc(e, &e->enc_k, enc_cache);
    rc |= alloc(e, &e->enc_v, enc_cache);
    const int64_t self_cache = (int64_t)B * Hkv * c.max_audio * D;
    e->ck.resize(c.n_dec_layers);
    e->cv.resize(c.n_dec_layers);
    e->sk.resize(c.n_dec_layers);
    e->sv.resize(c.n_dec_layers);
    for (int l = 0; l < c.n_dec_layers; ++l) {
        rc |= alloc(e, &e->ck[l], enc_cache);
        rc |= alloc(e, &e->cv[l], enc_cache);
        rc |= alloc(e, &e->sk[l], self_cache);
        rc |= alloc(e, &e->sv[l], self_cache);
    }
    rc |= alloc(e, &e->enc_len, B);
    rc |= alloc(e, &e->dh, (int64_t)B * d);
    rc |= alloc(e, &e->dxn, (int64_t)B * d);
    rc |= alloc(e, &e->dq, (int64_t)B * e->q_dim);
    rc |= alloc(e, &e->datt, (int64_t)B * e->q_dim);
    rc |= alloc(e, &e->dact, (int64_t)B * f);
    rc |= alloc(e, &e->dhh, (int64_t)B * d);
    rc |= alloc(e, &e->dh2, (int64_t)B * d);
    rc |= alloc(e, &e->dv, (int64_t)B * d);
    e->logits_ld = e->Vpad;
    rc |= alloc(e, &e->logits, (int64_t)B * e->logits_ld);
    rc |= alloc(e, &e->rows, B);
    rc |= alloc(e, &e->state, B);
    rc |= alloc(e, &e->topk_list, 4096);
    rc |= alloc(e, &e->silence, 4096);
    rc |= alloc(e, &e->out_tokens, (int64_t)B * (c.max_gen > 0 ? c.max_gen : 1));
    rc |= alloc(e, &e->kv_len, B);
    rc |= alloc(e, &e->next_pos, B);
    rc |= alloc(e, &e->next_token, B);
    rc |= alloc(e, &e->flags, B);
    rc |= alloc(e, &e->last_rows, B);
    rc |= alloc(e, &e->attn_tickets_buf, (int64_t)B * Hkv);
    rc |= alloc(e, &e->rope_tab, (int64_t)B * D);
    rc |= alloc(e, &e->fs_val, (int64_t)B * FS_NB * FS_CAP);
    rc |= alloc(e, &e->fs_idx, (int64_t)B * FS_NB * FS_CAP);
    rc |= alloc(e, &e->fs_cnt, (int64_t)B * FS_NB);
    rc |= alloc(e, &e->fs_amv, (int64_t)B * FS_NB);
    rc |= alloc(e, &e->fs_ami, (int64_t)B * FS_NB);
    rc |= alloc(e, &e->fs_ticket, B);
    rc |= alloc(e, &e->fs_slow, B);
    {
        const char* fsv = getenv("T5G_SAMPLER_FAST");
        e->fast_sampler = !(fsv && fsv[0] == '0');
        const char* fdv = getenv("T5G_FUSED_DECODE");
        e->fused_decode = fdv && (fdv[0] == '1' || fdv[0] == '2');
        e->fused_p16 = fdv && fdv[0] == '2';
        const char* atv = getenv("T5G_ATTN_TICKETS");
        e->attn_tickets = atv && atv[0] == '1';
        const char* guv = getenv("T5G_GU_GEMV");
        e->gu_gemv = !(guv && guv[0] == '0');
        const char* dgv = getenv("T5G_DOWN_GEMV");
        e->down_gemv = dgv && dgv[0] == '1';
        const char* sdv = getenv("T5G_S_DOWN");
        if (sdv && atoi(sdv) >= 2 && atoi(sdv) <= 8) e->s_down = atoi(sdv);
        const char* sqv = getenv("T5G_S_QKV");
        if (sqv && atoi(sqv) >= 2 && atoi(sqv) <= 4) e->s_qkv = atoi(sqv);
        const char* sov = getenv("T5G_S_O");
        if (sov && atoi(sov) >= 2 && atoi(sov) <= 4) e->s_o = atoi(sov);
        const char* lnv = getenv("T5G_LEAD_NORM");
        if (lnv) e->lead_sites = atoi(lnv) & 7;
        const char* xsv = getenv("T5G_XATTN_SPLIT");
        e->xsplit = xsv ? atoi(xsv) : 1;
        const int xmax = (c.max_text + 63) / 64 > 16 ? (c.max_text + 63) / 64 : 16;
        if (e->xsplit < (c.max_text + 63) / 64) e->xsplit = (c.max_text + 63) / 64;
        if (e->xsplit > xmax) e->xsplit = xmax;
    }
    if (rc) {
        t5g_engine_destroy(e);
        return T5G_ENOMEM;
    }
    *out = e;
    return T5G_OK;
}

// ---------------------------------------------------------------------------
static int gemm(const bf16_t* X, int ldx, int M, const void* W, int N, int K, int splits, const void* bias,
                void* Y, int ldy, int epi, hipStream_t st, bool prefill = false) {
    GemmArgs a;
    memset(&a, 0, sizeof(a));
    a.prefill = prefill ? 1 : 0;
    a.X = X;
    a.ldx = ldx;
    a.M = M;
    a.W = (const bf16_t*)W;
    a.N = N;
    a.NG = ng_pad(N);
    a.KB = K / 32;
    a.splits = splits;
    a.bias = (const bf16_t*)bias;
    a.Y = Y;
    a.ldy = ldy;
    return gemm_p16(a, epi, st);
}

static NormArgs norm_args(int M, int d, float eps) {
    NormArgs n;
    memset(&n, 0, sizeof(n));
    n.M = M;
    n.d = d;
    n.eps = eps;
    return n;
}

// Self-attention block input is xn (normed) -> result residual update.
// Packed-token path (encoder / prefill / cross prefill) -------------------------------
static int attn_packed(t5g_engine* e, int ntok, const bf16_t* q, const int* tok_row, const int* tok_t,
                       const bf16_t* K, const bf16_t* Vc, int Lmax, const int* kv_len, int causal, int window,
                       bf16_t* out, hipStream_t st) {
    const t5g_config& c = e->c;
    AttnArgs a;
    memset(&a, 0, sizeof(a));
    a.Q = q;
    a.ldq = e->q_dim;
    a.Mq = ntok;
    a.q_row = tok_row;
    a.q_pos = tok_t;
    a.K = K;
    a.V = Vc;
    a.kv_hstride = (long)Lmax * c.head_dim;
    a.kv_bstride = a.kv_hstride * c.n_kv_heads;
    a.kv_len = kv_len;
    a.Hkv = c.n_kv_heads;
    a.D = c.head_dim;
    a.G = c.n_heads / c.n_kv_heads;
    a.causal = causal;
    a.window = window;
    a.scale = c.attn_scale;
    a.softcap = c.softcap;
    a.eager = c.softcap > 0.f;
    a.nsplit = 1;
    a.chunk = Lmax;
    a.O = out;
    a.ldo = e->q_dim;
    return attention(a, st);
}

extern "C" int t5g_encode(t5g_engine* e, int32_t B, int32_t ntok, const int32_t* ids, const int32_t* tok_row,
                          const int32_t* tok_t, const float* pos, const int32_t* text_len, void* stream) {
    if (!e || B <= 0 || ntok <= 0) return T5G_EINVAL;
    const t5g_config& c = e->c;
    if (B > c.max_batch || ntok > B * c.max_text) return T5G_ECAPACITY;
    hipStream_t st = (hipStream_t)stream;
    const int d = c.hidden, f = c.intermediate, D = c.head_dim;
    HIPCHK(hipMemcpyAsync(e->enc_len, text_len, B * sizeof(int), hipMemcpyDeviceToDevice, st));
    for (int l = 0; l < c.n_enc_layers; ++l) {
        const t5g_layer_weights& L = e->enc[l];
        NormArgs n = norm_args(ntok, d, c.rms_eps);
        if (l == 0) {
            n.ids = ids;
            n.table = (const bf16_t*)e->w.enc_embed;
            n.scale = c.normalizer;
        } else {
            n.delta = e->tmp;  // previous layer's down-proj output
            n.post_w = (const bf16_t*)e->enc[l - 1].norms[5];
            n.resid = e->h;
        }
        n.pre_w = (const bf16_t*)L.norms[0];
        n.resid_out = e->h;
        n.normed_out = e->xn;
        RC(resid_norm(n, st));
        RC(gemm(e->xn, d, ntok, L.qkv, e->qkv_dim, d, 1, nullptr, e->qkv, e->qkv_dim, EPI_BF16, st, true));
        RopeArgs r;
        memset(&r, 0, sizeof(r));
        r.X = e->qkv;
        r.ldx = e->qkv_dim;
        r.M = ntok;
        r.D = D;
        r.nq = c.n_heads;
        r.nk = c.n_kv_heads;
        r.nv = c.n_kv_heads;
        r.rope_q = r.rope_k = 1;
        r.pos = pos;
        r.inv_freq = e->w.inv_freq;
        r.tok_row = tok_row;
        r.tok_t = tok_t;
        r.Qout = e->q;
        r.ldq = e->q_dim;
        r.Kc = e->enc_k;
        r.Vc = e->enc_v;
        r.c_hstride = (long)c.max_text * D;
        r.c_bstride = r.c_hstride * c.n_kv_heads;
        RC(rope_store(r, st));
        RC(attn_packed(e, ntok, e->q, tok_row, tok_t, e->enc_k, e->enc_v, c.max_text, e->enc_len, 0,
                       c.enc_sliding[l] ? c.sliding_window : 0, e->att, st));
        RC(gemm(e->att, e->q_dim, ntok, L.o, d, e->q_dim, 1, nullptr, e->tmp, d, EPI_BF16, st, true));
        n = norm_args(ntok, d, c.rms_eps);
        n.delta = e->tmp;
        n.post_w = (const bf16_t*)L.norms[1];
        n.resid = e->h;
        n.pre_w = (const bf16_t*)L.norms[4];
        n.resid_out = e->h;
        n.normed_out = e->xn;
        RC(resid_norm(n, st));
        RC(gemm(e->xn, d, ntok, L.gate_up, 2 * f, d, 1, nullptr, e->act, f, EPI_GEGLU, st, true));
        RC(gemm(e->act, f, ntok, L.down, d, f, 1, nullptr, e->tmp, d, EPI_BF16, st, true));
    }
    // final: h + post_ff(down) -> encoder norm -> memory
    NormArgs n = norm_args(ntok, d, c.rms_eps);
    n.delta = e->tmp;
    n.post_w = (const bf16_t*)e->enc[c.n_enc_layers - 1].norms[5];
    n.resid = e->h;
    n.pre_w = (const bf16_t*)e->w.enc_final_norm;
    n.resid_out = e->h;
    n.normed_out = e->mem;
    RC(resid_norm(n, st));
    // cross-attention K/V of every decoder layer from memory (PM-RoPE on K)
    for (int l = 0; l < c.n_dec_layers; ++l) {
        RC(gemm(e->mem, d, ntok, e->dec[l].cross_kv, 2 * e->kv_dim, d, 1, nullptr, e->qkv, 2 * e->kv_dim,
                EPI_BF16, st, true));
        RopeArgs r;
        memset(&r, 0, sizeof(r));
        r.X = e->qkv;
        r.ldx = 2 * e->kv_dim;
        r.M = ntok;
        r.D = D;
        r.nk = c.n_kv_heads;
        r.nv = c.n_kv_heads;
        r.rope_k = 1;
        r.pos = pos;
        r.inv_freq = e->w.inv_freq;
        r.tok_row = tok_row;
        r.tok_t = tok_t;
        r.Kc = e->ck[l];
        r.Vc = e->cv[l];
        r.c_hstride = (long)c.max_text * D;
        r.c_bstride = r.c_hstride * c.n_kv_heads;
        RC(rope_store(r, st));
    }
    return T5G_OK;
}

// One decoder pass over `M` tokens. Packed mode (tok_row != null): prefill;
// decode mode: M = B rows, positions/slots/tokens from the sampler buffers.
static DecGemmArgs dec_args(int M, const void* W, int N, int K, void* Y, int ldy, int nw);

static int decoder_pass(t5g_engine* e, int M, const int* ids, const int* tok_row, const int* tok_t, const float* pos,
                        bool decode, hipStream_t st) {
    const t5g_config& c = e->c;
    const int d = c.hidden, f = c.intermediate, D = c.head_dim;
    bf16_t* h = decode ? e->dh : e->h;
    bf16_t* xn = decode ? e->dxn : e->xn;
    bf16_t* q = decode ? e->dq : e->q;
    bf16_t* att = decode ? e->datt : e->att;
    bf16_t* act = decode ? e->dact : e->act;
    bf16_t* tmp = e->tmp;
    const int G = c.n_heads / c.n_kv_heads;
    // split-K factors (decode: spread weight streams over >= 512 blocks)
    const int s_qkv = decode ? e->s_qkv : 1, s_o = decode ? e->s_o : 1, s_cq = decode ? e->s_o : 1, s_down = decode ? e->s_down : 1;
    // one cos/sin table per step: every layer's q/k rotation uses the same positions
    const float* tab = nullptr;
    if (decode) {
        RC(rope_table(pos, e->w.inv_freq, M, D, e->rope_tab, st, e->lead_epoch));
        tab = e->rope_tab;
    }
    // PRO_LEAD chain (sdpa decode, M <= 16): the norm after o, cross-o and down (but the
    // last layer's) runs in the first M blocks of the GEMV that consumes it
    const bool lead = decode && e->lead_sites && M <= 16 && !(c.softcap > 0.f) && s_qkv > 1 && s_cq > 1 &&
                      d % 32 == 0 && d <= 4096;
    auto lead_gemv = [&](const void* W, int N, void* Y, int ldy, int nsplit, const void* post_w, const void* pre_w,
                         int site, int epi) -> int {
        DecGemmArgs g = dec_args(M, W, N, d, Y, ldy, 8);
        g.un = 8;
        g.X = xn;
        g.ldx = d;
        g.part = e->part;
        g.nsplit_p = nsplit;
        g.ldp = d;
        g.h_in = h;
        g.h_out = h;
        g.post_w = (const bf16_t*)post_w;
        g.pre_w = (const bf16_t*)pre_w;
        g.eps = c.rms_eps;
        g.flags = e->lead_flags + site * 16;
        g.tmo = e->lead_tmo;
        g.epoch = e->lead_epoch;
        return gemv_dec(g, epi, PRO_LEAD, st);
    };
    for (int l = 0; l < c.n_dec_layers; ++l) {
        const t5g_layer_weights& L = e->dec[l];
        const bool lead_qkv = lead && (e->lead_sites & 1) && l > 0;   // layer 0: embedding norm
        const bool lead_cq = lead && (e->lead_sites & 2), lead_gu = lead && (e->lead_sites & 4);
        if (l == 0) {
            NormArgs n = norm_args(M, d, c.rms_eps);
            n.ids = ids;
            n.table = (const bf16_t*)e->w.audio_embed;
            n.scale = c.normalizer;
            n.pre_w = (const bf16_t*)L.norms[0];
            n.resid_out = h;
            n.normed_out = xn;
            RC(resid_norm(n, st));
        }
        // --- self attention
        RopeArgs r;
        memset(&r, 0, sizeof(r));
        if (lead_qkv) {
            RC(lead_gemv(L.qkv, e->qkv_dim, e->qslab, e->qkv_dim, s_down, e->dec[l - 1].norms[5], L.norms[0],
                         3 * l, EPI_F32));
            r.Xpart = e->qslab;
            r.nsplit = 1;
        } else if (s_qkv > 1) {
            RC(gemm(xn, d, M, L.qkv, e->qkv_dim, d, s_qkv, nullptr, e->part, e->qkv_dim, EPI_F32, st, !decode));
            r.Xpart = e->part;
            r.nsplit = s_qkv;
        } else {
            RC(gemm(xn, d, M, L.qkv, e->qkv_dim, d, 1, nullptr, e->qkv, e->qkv_dim, EPI_BF16, st, !decode));
            r.X = e->qkv;
        }
        r.ldx = e->qkv_dim;
        r.M = M;
        r.D = D;
        // decode: q is rotated inside the attention kernel; only k/v go to the cache here
        r.nq = decode ? 0 : c.n_heads;
        r.col0 = decode ? e->q_dim : 0;
        r.nk = c.n_kv_heads;
        r.nv = c.n_kv_heads;
        r.rope_q = r.rope_k = 1;
        r.pos = pos;
        r.inv_freq = e->w.inv_freq;
        r.tok_row = tok_row;
        r.tok_t = tok_t;
        r.kv_len = e->kv_len;
        r.rope_tab = tab;
        r.Qout = q;
        r.ldq = e->q_dim;
        r.Kc = e->sk[l];
        r.Vc = e->sv[l];
        r.c_hstride = (long)c.max_audio * D;
        r.c_bstride = r.c_hstride * c.n_kv_heads;
        // sdpa decode: the attention kernel appends k/v itself (AttnArgs::append)
        const bool fused_append = decode && !(c.softcap > 0.f) && s_qkv > 1;
        if (!fused_append) RC(rope_store(r, st));
        {
            AttnArgs a;
            memset(&a, 0, sizeof(a));
            a.Q = q;
            a.ldq = e->q_dim;
            a.Mq = M;
            a.q_row = tok_row;
            a.q_pos = tok_t;
            a.K = e->sk[l];
            a.V = e->sv[l];
            a.kv_hstride = (long)c.max_audio * D;
            a.kv_bstride = a.kv_hstride * c.n_kv_heads;
            a.kv_len = e->kv_len;
            a.Hkv = c.n_kv_heads;
            a.D = D;
            a.G = G;
            a.causal = 1;
            a.window = c.dec_sliding[l] ? c.sliding_window : 0;
            a.scale = c.attn_scale;
            a.softcap = c.softcap;
            a.eager = c.softcap > 0.f;
            a.O = att;
            a.ldo = e->q_dim;
            if (decode && !a.eager) {
                a.chunk = 64;
                a.nsplit = (c.max_audio + 63) / 64;
                a.kv_cap = c.max_audio;
                a.part = e->apart;
                a.counters = e->attn_tickets ? e->attn_tickets_buf : nullptr;
                if (s_qkv > 1) {
                    a.Qpart = lead_qkv ? e->qslab : e->part;
                    a.q_nsplit = lead_qkv ? 1 : s_qkv;
                    a.ldqp = e->qkv_dim;
                    a.pos = pos;
                    a.inv_freq = e->w.inv_freq;
                    a.rope_tab = tab;
                    a.append = fused_append ? 1 : 0;
                    a.k_col0 = e->q_dim;
                    a.v_col0 = e->q_dim + e->kv_dim;
                } else {
                    return T5G_EINVAL;
                }
                RC(attention_decode(a, st));
            } else {
                if (decode) {  // eager decode: q rope via rope_store (q only)
                    RopeArgs rq = r;
                    rq.nq = c.n_heads;
                    rq.nk = rq.nv = 0;
                    rq.col0 = 0;
                    RC(rope_store(rq, st));
                }
                a.nsplit = 1;
                a.chunk = c.max_audio;
                RC(attention(a, st));
            }
        }
        RC(gemm(att, e->q_dim, M, L.o, d, e->q_dim, s_o, nullptr, s_o > 1 ? (void*)e->part : (void*)tmp, d,
                s_o > 1 ? EPI_F32 : EPI_BF16, st, !decode));
        if (!lead_cq) {
            NormArgs n = norm_args(M, d, c.rms_eps);
            if (s_o > 1) {
                n.part = e->part;
                n.nsplit = s_o;
                n.ldp = d;
            } else {
                n.delta = tmp;
            }
            n.post_w = (const bf16_t*)L.norms[1];
            n.resid = h;
            n.pre_w = (const bf16_t*)L.norms[2];
            n.resid_out = h;
            n.normed_out = xn;
            RC(resid_norm(n, st));
        }
        // --- PM cross attention
        memset(&r, 0, sizeof(r));
        if (lead_cq) {
            RC(lead_gemv(L.cross_q, e->q_dim, e->qslab, e->q_dim, s_o, L.norms[1], L.norms[2], 3 * l + 1, EPI_F32));
            r.Xpart = e->qslab;
            r.nsplit = 1;
        } else if (s_cq > 1) {
            RC(gemm(xn, d, M, L.cross_q, e->q_dim, d, s_cq, nullptr, e->part, e->q_dim, EPI_F32, st, !decode));
            r.Xpart = e->part;
            r.nsplit = s_cq;
        } else {
            RC(gemm(xn, d, M, L.cross_q, e->q_dim, d, 1, nullptr, q, e->q_dim, EPI_BF16, st, !decode));
            r.X = q;
        }
        r.ldx = e->q_dim;
        r.M = M;
        r.D = D;
        r.nq = c.n_heads;
        r.rope_q = 1;
        r.pos = pos;
        r.inv_freq = e->w.inv_freq;
        r.tok_row = tok_row;
        r.rope_tab = tab;
        r.Qout = q;
        r.ldq = e->q_dim;
        const bool fuse_q = decode && c.softcap <= 0.f && s_cq > 1;
        if (!fuse_q) RC(rope_store(r, st));
        {
            AttnArgs a;
            memset(&a, 0, sizeof(a));
            a.Q = q;
            a.ldq = e->q_dim;
            a.Mq = M;
            a.q_row = tok_row;
            a.q_pos = tok_t;
            a.K = e->ck[l];
            a.V = e->cv[l];
            a.kv_hstride = (long)c.max_text * D;
            a.kv_bstride = a.kv_hstride * c.n_kv_heads;
            a.kv_len = e->enc_len;
            a.Hkv = c.n_kv_heads;
            a.D = D;
            a.G = G;
            a.causal = 0;
            a.window = 0;
            a.scale = c.attn_scale;
            a.softcap = c.softcap;
            a.eager = c.softcap > 0.f;
            a.O = att;
            a.ldo = e->q_dim;
            if (fuse_q) {
                a.chunk = 64;
                a.nsplit = e->xsplit;
                a.kv_cap = c.max_text;
                a.part = e->apart;
                a.counters = e->attn_tickets ? e->attn_tickets_buf : nullptr;
                a.Qpart = lead_cq ? e->qslab : e->part;
                a.q_nsplit = lead_cq ? 1 : s_cq;
                a.ldqp = e->q_dim;
                a.pos = pos;
                a.inv_freq = e->w.inv_freq;
                a.rope_tab = tab;
                RC(attention_decode(a, st));
            } else {
                a.nsplit = 1;
                a.chunk = c.max_text;
                RC(attention(a, st));
            }
        }
        RC(gemm(att, e->q_dim, M, L.cross_o, d, e->q_dim, s_o, nullptr, s_o > 1 ? (void*)e->part : (void*)tmp, d,
                s_o > 1 ? EPI_F32 : EPI_BF16, st, !decode));
        if (!lead_gu) {
            NormArgs n = norm_args(M, d, c.rms_eps);
            if (s_o > 1) {
                n.part = e->part;
                n.nsplit = s_o;
                n.ldp = d;
            } else {
                n.delta = tmp;
            }
            n.post_w = (const bf16_t*)L.norms[3];
            n.resid = h;
            n.pre_w = (const bf16_t*)L.norms[4];
            n.resid_out = h;
            n.normed_out = xn;
            RC(resid_norm(n, st));
        }
        // --- GeGLU MLP (decode: the one-block-per-CU GEMV unless T5G_GU_GEMV=0)
        if (lead_gu) {
            RC(lead_gemv(L.gate_up, 2 * f, act, f, s_o, L.norms[3], L.norms[4], 3 * l + 2, EPI_GEGLU));
        } else if (decode && e->gu_gemv && M <= 16) {
            DecGemmArgs g = dec_args(M, L.gate_up, 2 * f, d, act, f, 8);
            g.X = xn;
            g.ldx = d;
            g.un = 8;
            RC(gemv_dec(g, EPI_GEGLU, PRO_LOAD, st));
        } else {
            RC(gemm(xn, d, M, L.gate_up, 2 * f, d, 1, nullptr, act, f, EPI_GEGLU, st, !decode));
        }
        if (decode && e->down_gemv && M <= 16 && s_down > 1) {
            DecGemmArgs g = dec_args(M, L.down, d, f, e->part, d, 8);
            g.X = act;
            g.ldx = f;
            g.un = 8;
            g.splits = s_down;
            RC(gemv_dec(g, EPI_F32, PRO_LOAD, st));
        } else {
            RC(gemm(act, f, M, L.down, d, f, s_down, nullptr, s_down > 1 ? (void*)e->part : (void*)tmp, d,
                    s_down > 1 ? EPI_F32 : EPI_BF16, st, !decode));
        }
        if (!(lead && (e->lead_sites & 1)) || l == c.n_dec_layers - 1) {
            NormArgs n = norm_args(M, d, c.rms_eps);
            if (s_down > 1) {
                n.part = e->part;
                n.nsplit = s_down;
                n.ldp = d;
            } else {
                n.delta = tmp;
            }
            n.post_w = (const bf16_t*)L.norms[5];
            n.resid = h;
            const bool last = l == c.n_dec_layers - 1;
            n.pre_w = (const bf16_t*)(last ? e->w.dec_final_norm : e->dec[l + 1].norms[0]);
            n.resid_out = h;
            n.normed_out = xn;
            RC(resid_norm(n, st));
        }
    }
    return T5G_OK;
}

// ---------------------------------------------------------------------------
// Fused single-token decoder step (sdpa numerics, M <= 16 rows): 9 launches per layer.
//   qkv   : [norm prologue: previous down output + residual, post_ff/pre_self] -> fp32 q|k|v
//   attn  : self attention (PM-RoPE of q/k, k/v append) + split merge
//   o     : att -> bf16 v
//   cq    : [norm prologue: post_self/pre_cross] -> fp32 q
//   cattn : cross attention over the cached encoder K/V
//   co    : att -> bf16 v
//   gu    : [norm prologue: post_cross/pre_ff] -> GeGLU -> act
//   down  : act (direct from L2) -> bf16 v
// then head1 with the final-norm prologue, head2 (PMDecoderLayer.forward :256-323,
// decoder final norm [tf] :818, predict_layer :469-478).
static bool fused_ok(const t5g_engine* e, int M) {
    const t5g_config& c = e->c;
    return e->fused_decode && !(c.softcap > 0.f) && M >= 1 && M <= 16 && c.hidden % 32 == 0 &&
           c.hidden <= 4096 && (c.hidden <= 2560 || M <= 8) && c.intermediate % 32 == 0;
}

// row-major VALU GEMVs: every decoder projection has its plain copy, batch <= 8 rows
static bool rm_ok(const t5g_engine* e, int M) {
    if (!fused_ok(e, M) || e->fused_p16 || M > 8 || e->c.hidden > 2560 || !e->w.rm_head1) return false;
    for (const t5g_layer_weights& L : e->dec)
        if (!L.rm_qkv || !L.rm_o || !L.rm_gate_up || !L.rm_down || !L.rm_cross_q || !L.rm_cross_o) return false;
    return true;
}

static DecGemmArgs dec_args(int M, const void* W, int N, int K, void* Y, int ldy, int nw) {
    DecGemmArgs g;
    memset(&g, 0, sizeof(g));
    g.M = M;
    g.K = K;
    g.W = (const bf16_t*)W;
    g.N = N;
    g.NG = ng_pad(N);
    g.KB = K / 32;
    g.Y = Y;
    g.ldy = ldy;
    g.nw = nw;
    g.splits = 1;
    return g;
}

static int decode_fused(t5g_engine* e, bool rm, hipStream_t st) {
    const t5g_config& c = e->c;
    // rm: plain row-major weights on the VALU GEMV (exact rows per CU); else P16 on MFMA
    auto gv = [&](DecGemmArgs& g, const void* w_rm, int epi, int pro) -> int {
        if (!rm) return gemv_dec(g, epi, pro, st);
        g.W = (const bf16_t*)w_rm;
        return gemv_rm(g, epi, pro, st);
    };
    const int M = e->B, d = c.hidden, f = c.intermediate, D = c.head_dim;
    const int G = c.n_heads / c.n_kv_heads;
    const int nw_norm = M <= 8 ? 4 : 8;       // prologue rows per wave <= 2
    const int nw_wide = M <= 8 ? 8 : 8;
    bf16_t* hb[2] = {e->dh, e->dh2};
    int hc = 0;
    RC(rope_table(e->next_pos, e->w.inv_freq, M, D, e->rope_tab, st));
    auto norm_pro = [&](DecGemmArgs& g, const void* post_w, const void* pre_w, bool keep) {
        g.v = e->dv;
        g.h_in = hb[hc];
        g.post_w = (const bf16_t*)post_w;
        g.pre_w = (const bf16_t*)pre_w;
        g.eps = c.rms_eps;
        g.h_out = keep ? hb[hc ^ 1] : nullptr;
        hc ^= 1;
    };
    for (int l = 0; l < c.n_dec_layers; ++l) {
        const t5g_layer_weights& L = e->dec[l];
        // --- self attention
        {
            DecGemmArgs g = dec_args(M, L.qkv, e->qkv_dim, d, e->part, e->qkv_dim, nw_wide);
            int pro;
            if (l == 0) {
                pro = PRO_EMBED;
                g.ids = e->next_token;
                g.table = (const bf16_t*)e->w.audio_embed;
                g.scale = c.normalizer;
                g.pre_w = (const bf16_t*)L.norms[0];
                g.eps = c.rms_eps;
                g.h_out = hb[0];
                hc = 0;
            } else {
                pro = PRO_NORM;
                norm_pro(g, e->dec[l - 1].norms[5], L.norms[0], true);
            }
            RC(gv(g, L.rm_qkv, EPI_F32, pro));
        }
        {
            AttnArgs a;
            memset(&a, 0, sizeof(a));
            a.Q = e->dq;
            a.ldq = e->q_dim;
            a.Mq = M;
            a.K = e->sk[l];
            a.V = e->sv[l];
            a.kv_hstride = (long)c.max_audio * D;
            a.kv_bstride = a.kv_hstride * c.n_kv_heads;
            a.kv_len = e->kv_len;
            a.Hkv = c.n_kv_heads;
            a.D = D;
            a.G = G;
            a.causal = 1;
            a.window = c.dec_sliding[l] ? c.sliding_window : 0;
            a.scale = c.attn_scale;
            a.O = e->datt;
            a.ldo = e->q_dim;
            a.chunk = 64;
            a.nsplit = (c.max_audio + 63) / 64;
            a.kv_cap = c.max_audio;
            a.part = e->apart;
            a.counters = e->attn_tickets ? e->attn_tickets_buf : nullptr;
            a.Qpart = e->part;
            a.q_nsplit = 1;
            a.ldqp = e->qkv_dim;
            a.pos = e->next_pos;
            a.inv_freq = e->w.inv_freq;
            a.rope_tab = e->rope_tab;
            a.append = 1;
            a.k_col0 = e->q_dim;
            a.v_col0 = e->q_dim + e->kv_dim;
            RC(attention_decode(a, st));
        }
        {
            DecGemmArgs g = dec_args(M, L.o, d, e->q_dim, e->dv, d, nw_wide);
            g.X = e->datt;
            g.ldx = e->q_dim;
            RC(gv(g, L.rm_o, EPI_BF16, rm ? PRO_DIRECT : PRO_LOAD));
        }
        // --- PM cross attention
        {
            DecGemmArgs g = dec_args(M, L.cross_q, e->q_dim, d, e->part, e->q_dim, nw_wide);
            norm_pro(g, L.norms[1], L.norms[2], true);
            RC(gv(g, L.rm_cross_q, EPI_F32, PRO_NORM));
        }
        {
            AttnArgs a;
            memset(&a, 0, sizeof(a));
            a.Q = e->dq;
            a.ldq = e->q_dim;
            a.Mq = M;
            a.K = e->ck[l];
            a.V = e->cv[l];
            a.kv_hstride = (long)c.max_text * D;
            a.kv_bstride = a.kv_hstride * c.n_kv_heads;
            a.kv_len = e->enc_len;
            a.Hkv = c.n_kv_heads;
            a.D = D;
            a.G = G;
            a.causal = 0;
            a.scale = c.attn_scale;
            a.O = e->datt;
            a.ldo = e->q_dim;
            a.chunk = 64;
            a.nsplit = e->xsplit;
            a.kv_cap = c.max_text;
            a.part = e->apart;
            a.counters = e->attn_tickets ? e->attn_tickets_buf : nullptr;
            a.Qpart = e->part;
            a.q_nsplit = 1;
            a.ldqp = e->q_dim;
            a.pos = e->next_pos;
            a.inv_freq = e->w.inv_freq;
            a.rope_tab = e->rope_tab;
            RC(attention_decode(a, st));
        }
        {
            DecGemmArgs g = dec_args(M, L.cross_o, d, e->q_dim, e->dv, d, nw_wide);
            g.X = e->datt;
            g.ldx = e->q_dim;
            RC(gv(g, L.rm_cross_o, EPI_BF16, rm ? PRO_DIRECT : PRO_LOAD));
        }
        // --- GeGLU MLP
        {
            DecGemmArgs g = dec_args(M, L.gate_up, 2 * f, d, e->dact, f, nw_norm);
            norm_pro(g, L.norms[3], L.norms[4], true);
            RC(gv(g, L.rm_gate_up, EPI_GEGLU, PRO_NORM));
        }
        {
            DecGemmArgs g = dec_args(M, L.down, d, f, e->dv, d, nw_wide);
            g.X = e->dact;
            g.ldx = f;
            RC(gv(g, L.rm_down, EPI_BF16, PRO_DIRECT));
        }
    }
    // predict head: final decoder norm fused into head1's prologue
    {
        DecGemmArgs g = dec_args(M, e->w.head1, d, d, e->dhh, d, nw_wide);
        norm_pro(g, e->dec[c.n_dec_layers - 1].norms[5], e->w.dec_final_norm, false);
        g.x_out = e->dxn;
        g.bias = (const bf16_t*)e->w.head1_bias;
        RC(gv(g, e->w.rm_head1, EPI_BIAS_GELU, PRO_NORM));
    }
    RC(gemm(e->dhh, d, M, e->w.head2, e->V, d, 1, e->w.head2_bias, e->logits, e->logits_ld, EPI_BIAS_BF16, st));
    return T5G_OK;
}

// one decoder step + predict head for the e->B rows fed by the sampler buffers
static int head(t5g_engine* e, const bf16_t* xn_rows, int B, hipStream_t st);
static int decode_forward(t5g_engine* e, hipStream_t st) {
    if (rm_ok(e, e->B)) return decode_fused(e, true, st);
    if (fused_ok(e, e->B) && e->fused_p16) return decode_fused(e, false, st);
    int rc = decoder_pass(e, e->B, e->next_token, nullptr, nullptr, e->next_pos, true, st);
    if (rc) return rc;
    return head(e, e->dxn, e->B, st);
}

static int head(t5g_engine* e, const bf16_t* xn_rows, int B, hipStream_t st) {
    const t5g_config& c = e->c;
    const int d = c.hidden;
    RC(gemm(xn_rows, d, B, e->w.head1, d, d, 1, e->w.head1_bias, e->dhh, d, EPI_BIAS_GELU, st));
    RC(gemm(e->dhh, d, B, e->w.head2, e->V, d, 1, e->w.head2_bias, e->logits, e->logits_ld, EPI_BIAS_BF16, st));
    return T5G_OK;
}

extern "C" int t5g_prefill(t5g_engine* e, int32_t B, int32_t ntok, const int32_t* ids, const int32_t* tok_row,
                           const int32_t* tok_t, const float* pos, const int32_t* kv_len,
                           const int32_t* last_index, void* stream) {
    if (!e || B <= 0 || ntok <= 0) return T5G_EINVAL;
    const t5g_config& c = e->c;
    if (B > c.max_batch || ntok > B * c.max_audio) return T5G_ECAPACITY;
    hipStream_t st = (hipStream_t)stream;
    e->B = B;
    HIPCHK(hipMemcpyAsync(e->kv_len, kv_len, B * sizeof(int), hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(e->last_rows, last_index, B * sizeof(int), hipMemcpyDeviceToDevice, st));
    int rc = decoder_pass(e, ntok, ids, tok_row, tok_t, pos, false, st);
    if (rc) return rc;
    // the last decoder_pass norm wrote final-normed hidden of every token into xn;
    // gather each row's last token
    NormArgs n = norm_args(B, c.hidden, c.rms_eps);
    // copy rows: reuse resid_norm as a gather (delta = xn, no norms)
    n.delta = e->xn;
    n.out_rows = e->last_rows;
    n.resid_out = e->dxn;
    RC(resid_norm(n, st));
    return head(e, e->dxn, B, st);
}

extern "C" int t5g_sampler_setup(t5g_engine* e, int32_t B, const t5g_sampler_row* rows, const t5g_sampler_state* init,
                                 const int32_t* top_k_list, int32_t n_top_k_list, const int32_t* silence,
                                 int32_t n_silence, const void* noise, int32_t noise_steps, void* stream) {
    if (!e || B <= 0 || B > e->c.max_batch || !rows || !init) return T5G_EINVAL;
    if (n_top_k_list > 4096 || n_silence > 4096) return T5G_ECAPACITY;
    static_assert(sizeof(t5g_sampler_row) == sizeof(SamplerRow), "row layout");
    static_assert(sizeof(t5g_sampler_state) == sizeof(SamplerState), "state layout");
    hipStream_t st = (hipStream_t)stream;
    e->B = B;
    HIPCHK(hipMemcpyAsync(e->rows, rows, B * sizeof(SamplerRow), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->state, init, B * sizeof(SamplerState), hipMemcpyHostToDevice, st));
    if (n_top_k_list > 0)
        HIPCHK(hipMemcpyAsync(e->topk_list, top_k_list, n_top_k_list * sizeof(int), hipMemcpyHostToDevice, st));
    if (n_silence > 0)
        HIPCHK(hipMemcpyAsync(e->silence, silence, n_silence * sizeof(int), hipMemcpyHostToDevice, st));
    if (e->noise != (const bf16_t*)noise || e->noise_steps != noise_steps) {
        // noise pointer is baked into the captured graph
        if (e->gexec) {
            hipGraphExecDestroy(e->gexec);
            e->gexec = nullptr;
        }
        if (e->graph) {
            hipGraphDestroy(e->graph);
            e->graph = nullptr;
        }
    }
    e->noise = (const bf16_t*)noise;
    e->noise_steps = noise_steps;
    HIPCHK(hipMemsetAsync(e->out_tokens, 0xff, (size_t)B * e->c.max_gen * sizeof(int), st));
    return T5G_OK;
}

static SamplerArgs sampler_args(t5g_engine* e, const bf16_t* logits, int ld, int B) {
    SamplerArgs s;
    memset(&s, 0, sizeof(s));
    s.logits = logits;
    s.ldl = ld;
    s.V = e->V;
    s.B = B;
    s.rows = e->rows;
    s.state = e->state;
    s.top_k_list = e->topk_list;
    s.silence = e->silence;
    s.noise = e->noise;
    s.noise_steps = e->noise_steps;
    s.eos = e->c.eos;
    s.eos_guard = e->c.eos_guard;
    s.budget_extra = e->c.budget_extra;
    s.text_guard = e->c.text_guard;
    s.progress_scale = e->c.progress_scale;
    s.out_tokens = e->out_tokens;
    s.max_gen = e->c.max_gen;
    s.max_len = e->c.max_audio;
    s.kv_len = e->kv_len;
    s.next_pos = e->next_pos;
    s.next_token = e->next_token;
    s.flags = e->flags;
    s.fs_val = e->fs_val;
    s.fs_idx = e->fs_idx;
    s.fs_cnt = e->fs_cnt;
    s.fs_amv = e->fs_amv;
    s.fs_ami = e->fs_ami;
    s.fs_ticket = e->fs_ticket;
    s.fs_slow = e->fast_sampler ? e->fs_slow : nullptr;
    return s;
}

static int decode_iter(t5g_engine* e, hipStream_t st) {
    const int B = e->B;
    RC(sample(sampler_args(e, e->logits, e->logits_ld, B), st));
    return decode_forward(e, st);
}

extern "C" int t5g_decode(t5g_engine* e, int32_t n_steps, int32_t use_graph, void* stream) {
    if (!e || e->B <= 0) return T5G_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    if (!use_graph) {
        for (int i = 0; i < n_steps; ++i) {
            int rc = decode_iter(e, st);
            if (rc) return rc;
        }
        return T5G_OK;
    }
    if (!e->gexec || e->graph_B != e->B) {
        if (e->gexec) hipGraphExecDestroy(e->gexec);
        if (e->graph) hipGraphDestroy(e->graph);
        e->gexec = nullptr;
        e->graph = nullptr;
        if (!e->cap_stream) HIPCHK(hipStreamCreateWithFlags(&e->cap_stream, hipStreamNonBlocking));
        HIPCHK(hipStreamBeginCapture(e->cap_stream, hipStreamCaptureModeThreadLocal));
        int rc = decode_iter(e, e->cap_stream);
        hipGraph_t g = nullptr;
        hipError_t ec = hipStreamEndCapture(e->cap_stream, &g);
        if (rc) {
            if (g) hipGraphDestroy(g);
            return rc;
        }
        if (ec != hipSuccess) return T5G_EHIP;
        e->graph = g;
        HIPCHK(hipGraphInstantiate(&e->gexec, g, nullptr, nullptr, 0));
        e->graph_B = e->B;
    }
    for (int i = 0; i < n_steps; ++i) HIPCHK(hipGraphLaunch(e->gexec, st));
    return T5G_OK;
}

extern "C" int t5g_read_state(t5g_engine* e, t5g_sampler_state* out, int32_t B, void* stream) {
    if (!e || !out || B <= 0 || B > e->c.max_batch) return T5G_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(out, e->state, B * sizeof(SamplerState), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return T5G_OK;
}

extern "C" int t5g_read_tokens(t5g_engine* e, int32_t* out, int32_t B, void* stream) {
    if (!e || !out || B <= 0 || B > e->c.max_batch) return T5G_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(out, e->out_tokens, (size_t)B * e->c.max_gen * sizeof(int), hipMemcpyDeviceToHost, st));
    unsigned tmo = 0;
    HIPCHK(hipMemcpyAsync(&tmo, e->lead_tmo, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return tmo ? T5G_ESYNC : T5G_OK;
}

extern "C" int t5g_write_state(t5g_engine* e, const t5g_sampler_state* s, int32_t row, int32_t slot, int32_t token,
                               void* stream) {
    if (!e || !s || row < 0 || row >= e->c.max_batch || slot < 0 || slot >= e->c.max_gen) return T5G_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    static thread_local t5g_sampler_state hs;
    static thread_local int32_t hv[3];
    hs = *s;
    HIPCHK(hipMemcpyAsync(e->state + row, &hs, sizeof(SamplerState), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->out_tokens + (size_t)row * e->c.max_gen + slot, &token, sizeof(int),
                          hipMemcpyHostToDevice, st));
    if (!s->done) {
        hv[0] = s->current_length;
        hv[1] = token;
        float p = s->next_pos;
        HIPCHK(hipMemcpyAsync(e->kv_len + row, &hv[0], sizeof(int), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->next_token + row, &hv[1], sizeof(int), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->next_pos + row, &p, sizeof(float), hipMemcpyHostToDevice, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    return T5G_OK;
}

extern "C" int t5g_step_only(t5g_engine* e, void* stream) {
    if (!e || e->B <= 0) return T5G_EINVAL;
    return decode_forward(e, (hipStream_t)stream);
}

extern "C" int t5g_read_flags(t5g_engine* e, int32_t* out, int32_t B, void* stream) {
    if (!e || !out || B <= 0 || B > e->c.max_batch) return T5G_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(out, e->flags, B * sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return T5G_OK;
}

extern "C" void* t5g_logits_ptr(t5g_engine* e, int32_t* ld) {
    if (!e) return nullptr;
    if (ld) *ld = e->logits_ld;
    return e->logits;
}

extern "C" int t5g_copy_logits(t5g_engine* e, void* dst, int32_t B, void* stream) {
    if (!e || !dst || B <= 0 || B > e->c.max_batch) return T5G_EINVAL;
    HIPCHK(hipMemcpyAsync(dst, e->logits, (size_t)B * e->logits_ld * sizeof(bf16_t), hipMemcpyDeviceToDevice,
                          (hipStream_t)stream));
    return T5G_OK;
}

extern "C" int t5g_sample_only(t5g_engine* e, int32_t B, const void* logits, int32_t ld, void* stream) {
    if (!e || B <= 0 || B > e->c.max_batch) return T5G_EINVAL;
    RC(sample(sampler_args(e, (const bf16_t*)logits, ld, B), (hipStream_t)stream));
    return T5G_OK;
}

extern "C" int t5g_gemm(const void* X, int32_t ldx, int32_t M, const void* Wp, int32_t N, int32_t K, int32_t splits,
                        const void* bias, void* Y, int32_t ldy, int32_t epi, void* stream) {
    if (!X || !Wp || !Y || M <= 0 || N <= 0 || K % 32) return T5G_EINVAL;
    const bool prefill = (epi & T5G_GEMM_PREFILL) != 0;
    RC(gemm((const bf16_t*)X, ldx, M, Wp, N, K, splits, bias, Y, ldy, epi & 0xff, (hipStream_t)stream, prefill));
    return T5G_OK;
}

extern "C" int t5g_time_gemm(const void* X, int32_t ldx, int32_t M, const void* const* Wp_list, int32_t n_w,
                             int32_t N, int32_t K, int32_t splits, void* Y, int32_t ldy, int32_t epi, int32_t iters,
                             void* stream, float* avg_us) {
    if (iters <= 0 || !avg_us || !Wp_list || n_w <= 0) return T5G_EINVAL;
    for (int i = 0; i < n_w; ++i)
        if (!Wp_list[i]) return T5G_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    const bool pf = (epi & T5G_GEMM_PREFILL) != 0;
    epi &= 0xff;
    RC(gemm((const bf16_t*)X, ldx, M, Wp_list[0], N, K, splits, nullptr, Y, ldy, epi, st, pf));  // warm
    HIPCHK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i)
        RC(gemm((const bf16_t*)X, ldx, M, Wp_list[i % n_w], N, K, splits, nullptr, Y, ldy, epi, st, pf));
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    *avg_us = ms * 1000.f / iters;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return T5G_OK;
}

extern "C" int t5g_time_decode_step(t5g_engine* e, int32_t iters, void* stream, float* avg_us) {
    if (!e || iters <= 0 || !avg_us || e->B <= 0) return T5G_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) {
        int rc = decode_forward(e, st);
        if (rc) return rc;
    }
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    *avg_us = ms * 1000.f / iters;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return T5G_OK;
}

extern "C" int64_t t5g_attention_decode_work_bytes(int32_t B, int32_t Hq, int32_t Hkv, int32_t D, int32_t cap) {
    if (B <= 0 || Hkv <= 0 || Hq % Hkv || D <= 0 || cap <= 0) return -1;
    const int64_t nsplit = (cap + 63) / 64;
    return (int64_t)B * Hkv * nsplit * (Hq / Hkv) * (D + 2) * 4;
}

extern "C" int t5g_attention_decode(const t5g_attn_decode_args* g, void* stream) {
    if (!g || !g->q || !g->k_cache || !g->v_cache || !g->kv_len || !g->out || !g->work) return T5G_EINVAL;
    if (g->B <= 0 || g->n_kv_heads <= 0 || g->n_heads % g->n_kv_heads || g->cap <= 0 || g->cap > 4096)
        return T5G_EINVAL;
    AttnArgs a;
    memset(&a, 0, sizeof(a));
    a.Q = (const bf16_t*)g->q;
    a.ldq = g->n_heads * g->head_dim;
    a.Mq = g->B;
    a.K = (const bf16_t*)g->k_cache;
    a.V = (const bf16_t*)g->v_cache;
    a.kv_hstride = (long)g->cap * g->head_dim;
    a.kv_bstride = a.kv_hstride * g->n_kv_heads;
    a.kv_len = g->kv_len;
    a.Hkv = g->n_kv_heads;
    a.D = g->head_dim;
    a.G = g->n_heads / g->n_kv_heads;
    a.causal = g->causal;
    a.window = g->window;
    a.scale = g->scale;
    a.O = (bf16_t*)g->out;
    a.ldo = a.ldq;
    a.chunk = 64;
    a.nsplit = (g->cap + 63) / 64;
    a.kv_cap = g->cap;
    a.part = (float*)g->work;
    RC(attention_decode(a, (hipStream_t)stream));
    return T5G_OK;
}

static_assert(sizeof(t5g_gemv_args) == 152, "t5g_gemv_args layout");

static int gemv_from_abi(const t5g_gemv_args* g, const void* W, DecGemmArgs* out) {
    if (!g || !W || !g->Y || g->M <= 0 || g->N <= 0 || g->K <= 0 || g->K % 32) return T5G_EINVAL;
    DecGemmArgs a = dec_args(g->M, W, g->N, g->K, g->Y, g->ldy, g->nw);
    a.X = (const bf16_t*)g->X;
    a.ldx = g->ldx;
    a.v = (const bf16_t*)g->v;
    a.h_in = (const bf16_t*)g->h_in;
    a.ids = g->ids;
    a.table = (const bf16_t*)g->table;
    a.scale = g->scale;
    a.eps = g->eps;
    a.post_w = (const bf16_t*)g->post_w;
    a.pre_w = (const bf16_t*)g->pre_w;
    a.bias = (const bf16_t*)g->bias;
    a.h_out = (bf16_t*)g->h_out;
    a.x_out = (bf16_t*)g->x_out;
    a.un = g->un;
    a.max_grid = g->max_grid;
    a.splits = g->splits > 1 ? g->splits : 1;
    *out = a;
    return T5G_OK;
}

static int gemv_any(const DecGemmArgs& a, const t5g_gemv_args* g, hipStream_t st) {
    return g->layout == 1 ? gemv_rm(a, g->epi, g->pro, st) : gemv_dec(a, g->epi, g->pro, st);
}

extern "C" int t5g_gemv(const t5g_gemv_args* g, void* stream) {
    DecGemmArgs a;
    int rc = gemv_from_abi(g, g ? g->W : nullptr, &a);
    if (rc) return rc;
    RC(gemv_any(a, g, (hipStream_t)stream));
    return T5G_OK;
}

extern "C" int t5g_time_gemv(const t5g_gemv_args* g, const void* const* Wp_list, int32_t n_w, int32_t iters,
                             void* stream, float* avg_us) {
    if (!g || !Wp_list || n_w <= 0 || iters <= 0 || !avg_us) return T5G_EINVAL;
    std::vector<DecGemmArgs> as((size_t)n_w);
    for (int i = 0; i < n_w; ++i) {
        int rc = gemv_from_abi(g, Wp_list[i], &as[i]);
        if (rc) return rc;
    }
    hipStream_t st = (hipStream_t)stream;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    RC(gemv_any(as[0], g, st));  // warm
    HIPCHK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) RC(gemv_any(as[i % n_w], g, st));
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    *avg_us = ms * 1000.f / iters;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return T5G_OK;
}

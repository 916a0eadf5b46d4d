// Whisper recognizer (openai-whisper ModelDimensions; large-v3-turbo = 128 mels, 32 x 1280
// encoder, 4 x 1280 decoder) for gfx950, fp32 end to end on the f32 MFMA GEMM of
// xc2_common.h. Restates whisper/audio.py log_mel_spectrogram and whisper/model.py
// AudioEncoder / TextDecoder / ResidualAttentionBlock / MultiHeadAttention (checked
// against the transformers port [tf] models/whisper/modeling_whisper.py, the in-container
// architecture oracle). See include/whisper.h for the data flow.
//
// HBM layout (one utterance): activations time-major [T][C] fp32; the text decoder's
// self-attention cache [n_text_ctx][C] per layer for K and V; the cross-attention K / V
// [n_audio_ctx][C] per decoder layer, computed once per encoded window.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "whisper.h"
#include "xc2_common.h"

namespace xc2 {
namespace {

// --------------------------------------------------------------------- log-mel
// frame f, slot i < 416: x[f*160 + i - 200] of the signal (wav then zeros to n_total
// samples) reflected at both ends (torch.stft center=True, pad_mode "reflect"), times the
// periodic Hann window; slots >= 400 are the GEMM's K padding
__global__ void whs_frames_kernel(const float* wav, int n, int n_total, const float* window, float* frames) {
    const int f = blockIdx.x;
    for (int i = threadIdx.x; i < WHS_FFT_K; i += blockDim.x) {
        float v = 0.f;
        if (i < WHS_N_FFT) {
            long s = (long)f * WHS_HOP + i - WHS_N_FFT / 2;
            if (s < 0) s = -s;
            if (s >= n_total) s = 2L * (n_total - 1) - s;
            v = (s < n ? wav[s] : 0.f) * window[i];
        }
        frames[(long)f * WHS_FFT_K + i] = v;
    }
}

// |X_k|^2 from the DFT GEMM's interleaved (re, im) columns; bins >= 201 zero
__global__ void whs_power_kernel(const float* spec, float* pw) {
    const int f = blockIdx.x;
    for (int k = threadIdx.x; k < WHS_BINS_PAD; k += blockDim.x) {
        float v = 0.f;
        if (k < WHS_BINS) {
            const float re = spec[(long)f * WHS_FFT_K + 2 * k], im = spec[(long)f * WHS_FFT_K + 2 * k + 1];
            v = re * re + im * im;
        }
        pw[(long)f * WHS_BINS_PAD + k] = v;
    }
}

// global max of the log10 mel (one block), then (max(x, max - 8) + 4) / 4 in place
__global__ __launch_bounds__(1024) void whs_mel_norm_kernel(float* lm, long count) {
    __shared__ float red[16];
    float mx = -INFINITY;
    for (long i = threadIdx.x; i < count; i += blockDim.x) mx = fmaxf(mx, lm[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    mx = red[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) mx = fmaxf(mx, red[i]);
    const float lo = mx - 8.0f;
    for (long i = threadIdx.x; i < count; i += blockDim.x) lm[i] = (fmaxf(lm[i], lo) + 4.0f) / 4.0f;
}

// out[t][k * cin + ci] = X[t * stride + k - pad][ci] (0 outside [0, T_in)), zero K padding
__global__ void whs_im2col_kernel(const float* X, int T_in, int cin, int stride, int pad, float* out, int T_out,
                                  int kpad) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)T_out * kpad) return;
    const int t = (int)(idx / kpad), col = (int)(idx - (long)t * kpad);
    float v = 0.f;
    if (col < 3 * cin) {
        const int k = col / cin, ci = col - k * cin;
        const int ti = t * stride + k - pad;
        if (ti >= 0 && ti < T_in) v = X[(long)ti * cin + ci];
    }
    out[idx] = v;
}

// nn.LayerNorm (eps 1e-5) over rows of C <= 4096: 256 threads, 4 float4 per thread max
__global__ __launch_bounds__(256) void whs_layernorm_kernel(const float* X, float* Y, int C, const float* w,
                                                            const float* b) {
    __shared__ float red[8];
    const long row = blockIdx.x;
    constexpr int V = 4;
    f32x4 x[V];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int c = (threadIdx.x + 256 * j) * 4;
        x[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
        if (c < C) x[j] = *(const f32x4*)(X + row * C + c);
        s += (x[j][0] + x[j][1]) + (x[j][2] + x[j][3]);
    }
    const float mean = bsum(s, red) / (float)C;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int c = (threadIdx.x + 256 * j) * 4;
        if (c < C)
#pragma unroll
            for (int e = 0; e < 4; ++e) ss += (x[j][e] - mean) * (x[j][e] - mean);
    }
    const float rstd = 1.0f / sqrtf(bsum(ss, red) / (float)C + 1e-5f);
#pragma unroll
    for (int j = 0; j < V; ++j) {
        const int c = (threadIdx.x + 256 * j) * 4;
        if (c >= C) continue;
        f32x4 y;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = (x[j][e] - mean) * rstd * w[c + e] + b[c + e];
        *(f32x4*)(Y + row * C + c) = y;
    }
}

// x[i] = token_embedding[tokens[i]] + positional_embedding[offset + i]
__global__ void whs_embed_kernel(const int* tokens, const float* tok_emb, const float* pos, int offset, int C,
                                 int n_vocab, float* X) {
    const int i = blockIdx.x;
    const int id = min(max(tokens[i], 0), n_vocab - 1);
    for (int c = threadIdx.x; c < C; c += blockDim.x)
        X[(long)i * C + c] = tok_emb[(long)id * C + c] + pos[(long)(offset + i) * C + c];
}

// ------------------------------------------------------------------- attention
// softmax(q k^T / 8) v per head (head dim 64), flash-style over 64-key tiles with the f32
// MFMA: block = 128 queries x one head, wave = 32 queries. causal: query i sees keys
// [0, q_off + i] (the decoder's self attention over its cache). Q / K / V / O rows are
// strided (the encoder reads the fused [T][3C] projection buffer in place).
constexpr int AQ = 128, AK = 64, ALD = 68;

__global__ __launch_bounds__(256) void whs_attn_kernel(const float* Q, int ldq, const float* K, const float* V, int ldkv,
                                                       float* O, int ldo, int Tq, int Tk, int causal, int q_off,
                                                       float scale) {
    __shared__ float sm[2 * AK * ALD];
    float* Ks = sm;
    float* Vs = sm + AK * ALD;
    const int h = blockIdx.y, q0 = blockIdx.x * AQ;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, hh = lane >> 5;
    const int qi = q0 + w * 32 + li;
    const bool qv = qi < Tq;
    f32x4 qf[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (qv) v = *(const f32x4*)(Q + (long)qi * ldq + h * 64 + 8 * g + 4 * hh);
        qf[g] = v * scale;
    }
    f32x16 oacc[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[0][r] = oacc[1][r] = 0.f;
    float mrun = -INFINITY, lrun = 0.f;
    const int kend = causal ? min(Tk, q_off + min(q0 + AQ, Tq)) : Tk;
    const int klim = causal ? q_off + qi : Tk - 1;   // last key this lane's query sees
    for (int k0 = 0; k0 < kend; k0 += AK) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (tid >> 4) + 16 * i, c4 = (tid & 15) * 4;
            const int kr = k0 + row;
            f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = kv;
            if (kr < Tk) {
                kv = *(const f32x4*)(K + (long)kr * ldkv + h * 64 + c4);
                vv = *(const f32x4*)(V + (long)kr * ldkv + h * 64 + c4);
            }
            *(f32x4*)&Ks[row * ALD + c4] = kv;
            *(f32x4*)&Vs[row * ALD + c4] = vv;
        }
        __syncthreads();
        f32x16 s[2];
#pragma unroll
        for (int r = 0; r < 16; ++r) s[0][r] = s[1][r] = 0.f;
#pragma unroll
        for (int g = 0; g < 8; ++g)
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
                const f32x4 fk = *(const f32x4*)&Ks[(kt * 32 + li) * ALD + 8 * g + 4 * hh];
#pragma unroll
                for (int e = 0; e < 4; ++e) s[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(fk[e], qf[g][e], s[kt], 0, 0, 0);
            }
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                s[kt][r] = (key < Tk && key <= klim) ? s[kt][r] : -INFINITY;
                mx = fmaxf(mx, s[kt][r]);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        // key 0 is in every query's range and in the first tile, so mnew is finite
        const float mnew = fmaxf(mrun, mx);
        const float alpha = expf(mrun - mnew);
        float ls = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                s[kt][r] = expf(s[kt][r] - mnew);
                ls += s[kt][r];
            }
        ls += __shfl_xor(ls, 32, 64);
        lrun = lrun * alpha + ls;
        mrun = mnew;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            oacc[0][r] *= alpha;
            oacc[1][r] *= alpha;
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int kl = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
#pragma unroll
                for (int dt = 0; dt < 2; ++dt)
                    oacc[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[kl * ALD + dt * 32 + li], s[kt][r], oacc[dt],
                                                                    0, 0, 0);
            }
    }
    __syncthreads();
    float* slab = sm + w * 32 * ALD;
    const float inv = 1.0f / lrun;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int d = dt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            slab[li * ALD + d] = oacc[dt][r] * inv;
        }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int qq = (lane >> 4) + 4 * i, c4 = (lane & 15) * 4;
        const int q = q0 + w * 32 + qq;
        if (q < Tq) *(f32x4*)(O + (long)q * ldo + h * 64 + c4) = *(const f32x4*)&slab[qq * ALD + c4];
    }
}

// --------------------------------------------------------- decode-step kernels
// fp32 GEMV for M <= 4 rows (the decoder's one-token steps): Y[m][n] = epi(X[m] . W[n] +
// bias[n]) (+ resid[m][n]); one wave per 4 output rows, lanes stride K in float4, every
// W load of the wave issued before the reductions.
constexpr int GV_ROWS = 4, GV_MMAX = 4, GV_KV = 8;   // K <= 64 lanes x 4 x 8 x ... (looped)

__global__ __launch_bounds__(256) void whs_gemv_kernel(const float* X, int ldx, int M, const float* W, int K, int N,
                                                       const float* bias, const float* resid, float* Y, int ldy,
                                                       int epi) {
    const int lane = threadIdx.x & 63;
    const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * GV_ROWS;
    if (n0 >= N) return;
    float acc[GV_MMAX][GV_ROWS];
#pragma unroll
    for (int m = 0; m < GV_MMAX; ++m)
#pragma unroll
        for (int r = 0; r < GV_ROWS; ++r) acc[m][r] = 0.f;
    const int K4 = K / 4;
    for (int kb = 0; kb < K4; kb += 64 * GV_KV) {
        f32x4 wv[GV_ROWS][GV_KV];
#pragma unroll
        for (int r = 0; r < GV_ROWS; ++r) {
            const int n = min(n0 + r, N - 1);
#pragma unroll
            for (int j = 0; j < GV_KV; ++j) {
                const int k4 = kb + lane + 64 * j;
                wv[r][j] = k4 < K4 ? *(const f32x4*)(W + (long)n * K + 4 * k4) : (f32x4){0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int m = 0; m < GV_MMAX; ++m) {
            if (m >= M) break;
#pragma unroll
            for (int j = 0; j < GV_KV; ++j) {
                const int k4 = kb + lane + 64 * j;
                if (k4 >= K4) break;
                const f32x4 xv = *(const f32x4*)(X + (long)m * ldx + 4 * k4);
#pragma unroll
                for (int r = 0; r < GV_ROWS; ++r)
                    acc[m][r] += (xv[0] * wv[r][j][0] + xv[1] * wv[r][j][1]) + (xv[2] * wv[r][j][2] + xv[3] * wv[r][j][3]);
            }
        }
    }
#pragma unroll
    for (int m = 0; m < GV_MMAX; ++m) {
        if (m >= M) break;
#pragma unroll
        for (int r = 0; r < GV_ROWS; ++r) {
            const float v = wsum(acc[m][r]);
            const int n = n0 + r;
            if (lane == r && n < N) {
                float y = v + (bias ? bias[n] : 0.f);
                if (epi == EPI_GELU) y = 0.5f * y * (1.0f + erff(y * 0.70710678118654752f));
                if (resid) y += resid[(long)m * ldy + n];
                Y[(long)m * ldy + n] = y;
            }
        }
    }
}

// one query per head against Tk keys, split over blockIdx.y in chunks of 256 keys (one key
// per thread): partial (max, sum, P.V[64]) per split, merged by whs_attn_merge_kernel
constexpr int AD_CHUNK = 256;

__global__ __launch_bounds__(256) void whs_attn_dec_kernel(const float* Q, const float* K, const float* V, int ldkv,
                                                           int Tk, float scale, float* part) {
    __shared__ float ps[AD_CHUNK];
    __shared__ float red[8];
    __shared__ float accs[4][64];
    const int h = blockIdx.x, s = blockIdx.y, tid = threadIdx.x;
    const int k0 = s * AD_CHUNK, kn = min(AD_CHUNK, Tk - k0);
    float sc = -INFINITY;
    if (tid < kn) {
        const float* kr = K + (long)(k0 + tid) * ldkv + h * 64;
        const float* q = Q + h * 64;
        float a = 0.f;
#pragma unroll
        for (int d = 0; d < 64; d += 4) {
            const f32x4 kv = *(const f32x4*)(kr + d), qv = *(const f32x4*)(q + d);
            a += (qv[0] * kv[0] + qv[1] * kv[1]) + (qv[2] * kv[2] + qv[3] * kv[3]);
        }
        sc = a * scale;
    }
    float mx = sc;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if ((tid & 63) == 0) red[tid >> 6] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float p = tid < kn ? expf(sc - mx) : 0.f;
    ps[tid] = p;
    const float l = bsum(p, red + 4);   // bsum's leading barrier also publishes ps
    // wave g sums keys [64 g, 64 g + 64) of the chunk; rows past the end are clamped (their
    // p is 0), so the 64 loads are unconditional and issue back to back
    const int d = tid & 63, g = tid >> 6;
    float a = 0.f;
#pragma unroll 16
    for (int i = 0; i < 64; ++i) {
        const int t = 64 * g + i;
        a += ps[t] * V[(long)min(k0 + t, Tk - 1) * ldkv + h * 64 + d];
    }
    accs[g][d] = a;
    __syncthreads();
    float* o = part + ((long)h * gridDim.y + s) * 66;
    if (tid < 64) o[2 + tid] = (accs[0][tid] + accs[1][tid]) + (accs[2][tid] + accs[3][tid]);
    if (tid == 0) {
        o[0] = mx;
        o[1] = l;
    }
}

__global__ void whs_attn_merge_kernel(const float* part, int nsplit, float* O) {
    const int h = blockIdx.x, d = threadIdx.x;
    const float* p = part + (long)h * nsplit * 66;
    float M = -INFINITY;
    for (int s = 0; s < nsplit; ++s) M = fmaxf(M, p[s * 66]);
    float l = 0.f, a = 0.f;
    for (int s = 0; s < nsplit; ++s) {
        const float e = expf(p[s * 66] - M);
        l += e * p[s * 66 + 1];
        a += e * p[s * 66 + 2 + d];
    }
    O[h * 64 + d] = a / l;
}

}  // namespace
}  // namespace xc2

using namespace xc2;

struct whs_model {
    whs_config cfg;
    whs_weights w;
    int frames_max;     // mel frames of max_samples (+ 30 s)
    int mel_frames;     // frames of the last whs_log_mel
    float *frames, *spec, *pw, *lm;
    float *col, *h1, *x, *xn, *qkv, *att, *mid;
    float *ck, *cv;     // [n_text_layer][n_audio_ctx][C]
    float *kc, *vc;     // [n_text_layer][n_text_ctx][C]
    float *dx, *dxn, *dq, *datt, *dmid;   // decoder activations [n_text_ctx][...]
    float* apart;       // decode attention split partials [heads][splits][66]
    int encoded;
    size_t bytes;
};

static int whs_alloc(whs_model* m, float** p, long floats) {
    const size_t b = (size_t)(floats > 1 ? floats : 1) * sizeof(float);
    if (hipMalloc((void**)p, b) != hipSuccess) return -4;
    if (hipMemset(*p, 0, b) != hipSuccess) return -2;
    m->bytes += b;
    return 0;
}

static GemmArgs wg(const float* A, int lda, const float* W, int K, int N, const float* bias, float* Cp, int ldc, int M) {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A = A;
    g.lda = lda;
    g.am = RowMap{M, 0, 0};
    g.W = W;
    g.ldw = K;
    g.bias = bias;
    g.C = Cp;
    g.ldc = ldc;
    g.cm = RowMap{M, 0, 0};
    g.M = M;
    g.N = N;
    g.K = K;
    return g;
}

#define WH_TRY(x)            \
    do {                     \
        int _rc = (x);       \
        if (_rc) return _rc; \
    } while (0)
#define WH_LAUNCHED() \
    do { if (hipGetLastError() != hipSuccess) return -2; } while (0)

static int whs_ln(const float* X, float* Y, int T, int C, const float* w, const float* b, hipStream_t st) {
    hipLaunchKernelGGL(whs_layernorm_kernel, dim3(T), dim3(256), 0, st, X, Y, C, w, b);
    WH_LAUNCHED();
    return 0;
}

static int whs_attention(const float* Q, int ldq, const float* K, const float* V, int ldkv, float* O, int ldo, int Tq,
                         int Tk, int heads, int causal, int q_off, hipStream_t st) {
    hipLaunchKernelGGL(whs_attn_kernel, dim3((Tq + AQ - 1) / AQ, heads), dim3(256), 0, st, Q, ldq, K, V, ldkv, O, ldo,
                       Tq, Tk, causal, q_off, 0.125f);
    WH_LAUNCHED();
    return 0;
}

// decoder GEMMs: the GEMV for one-token steps (M <= 4), the tiled MFMA GEMM otherwise
static int dgemm(const GemmArgs& g, hipStream_t st) {
    if (g.M > GV_MMAX || g.K % 4 || g.lda % 4 || g.am.off || g.am.seq) return gemm(g, st);
    float* Y = g.C + (long)g.cm.off * g.ldc;
    const float* R = g.resid ? g.resid + (long)g.cm.off * g.ldc : nullptr;
    const int blocks = (g.N + 4 * GV_ROWS - 1) / (4 * GV_ROWS);
    hipLaunchKernelGGL(whs_gemv_kernel, dim3(blocks), dim3(256), 0, st, g.A, g.lda, g.M, g.W, g.K, g.N, g.bias, R, Y,
                       g.ldc, g.epi);
    WH_LAUNCHED();
    return 0;
}

// one-token decoder attention: key splits + merge; longer query blocks: the tiled kernel
static int dec_attention(whs_model* m, const float* Q, const float* K, const float* V, int ldkv, float* O, int n,
                         int Tk, int heads, int causal, int q_off, hipStream_t st) {
    if (n != 1) return whs_attention(Q, heads * 64, K, V, ldkv, O, heads * 64, n, Tk, heads, causal, q_off, st);
    const int ns = (Tk + AD_CHUNK - 1) / AD_CHUNK;
    hipLaunchKernelGGL(whs_attn_dec_kernel, dim3(heads, ns), dim3(256), 0, st, Q, K, V, ldkv, Tk, 0.125f, m->apart);
    WH_LAUNCHED();
    hipLaunchKernelGGL(whs_attn_merge_kernel, dim3(heads), dim3(64), 0, st, m->apart, ns, O);
    WH_LAUNCHED();
    return 0;
}

// x += mlp(ln(x)) over T rows (mid: [T][4C])
static int whs_mlp(const whs_block& L, float* x, float* xn, float* mid, int T, int C, hipStream_t st) {
    WH_TRY(whs_ln(x, xn, T, C, L.mlp_ln_w, L.mlp_ln_b, st));
    GemmArgs g = wg(xn, C, L.fc1_w, C, 4 * C, L.fc1_b, mid, 4 * C, T);
    g.epi = EPI_GELU;
    WH_TRY(dgemm(g, st));
    GemmArgs g2 = wg(mid, 4 * C, L.fc2_w, 4 * C, C, L.fc2_b, x, C, T);
    g2.resid = x;
    return dgemm(g2, st);
}

extern "C" {

int whs_create(const whs_config* cfg, const whs_weights* w, whs_model** out) {
    if (!cfg || !w || !out) return -1;
    const whs_config& k = *cfg;
    const int C = k.n_audio_state;
    if (C <= 0 || C % 128 || C > 4096 || k.n_text_state != C || k.n_audio_head * 64 != C || k.n_text_head * 64 != C ||
        k.n_audio_layer < 0 || k.n_audio_layer > WHS_MAX_LAYERS || k.n_text_layer < 1 ||
        k.n_text_layer > WHS_MAX_LAYERS || k.n_audio_ctx * 2 != WHS_N_FRAMES || k.n_mels <= 0 || k.n_mels > 256 ||
        k.n_vocab <= 0 || k.n_text_ctx <= 0 || k.max_samples <= 0)
        return -1;
    if (w->conv1_kpad < 3 * k.n_mels || w->conv1_kpad % 32 || w->conv2_kpad < 3 * C || w->conv2_kpad % 32) return -1;
    whs_model* m = new whs_model();
    memset(m, 0, sizeof(*m));
    m->cfg = k;
    m->w = *w;
    m->frames_max = k.max_samples / WHS_HOP + WHS_N_FRAMES;
    const long F = m->frames_max, T1 = WHS_N_FRAMES, T = k.n_audio_ctx, Lt = k.n_text_ctx;
    const long col1 = T1 * (long)w->conv1_kpad, col2 = T * (long)w->conv2_kpad;
    const long col = col1 > col2 ? col1 : col2;
    int rc = 0;
    rc = rc ? rc : whs_alloc(m, &m->frames, F * WHS_FFT_K);
    rc = rc ? rc : whs_alloc(m, &m->spec, F * WHS_FFT_K);
    rc = rc ? rc : whs_alloc(m, &m->pw, F * WHS_BINS_PAD);
    rc = rc ? rc : whs_alloc(m, &m->lm, F * k.n_mels);
    rc = rc ? rc : whs_alloc(m, &m->col, col);
    rc = rc ? rc : whs_alloc(m, &m->h1, T1 * C);
    rc = rc ? rc : whs_alloc(m, &m->x, T * C);
    rc = rc ? rc : whs_alloc(m, &m->xn, T * C);
    rc = rc ? rc : whs_alloc(m, &m->qkv, T * 3 * C);
    rc = rc ? rc : whs_alloc(m, &m->att, T * C);
    rc = rc ? rc : whs_alloc(m, &m->mid, T * 4 * C);
    rc = rc ? rc : whs_alloc(m, &m->ck, (long)k.n_text_layer * T * C);
    rc = rc ? rc : whs_alloc(m, &m->cv, (long)k.n_text_layer * T * C);
    rc = rc ? rc : whs_alloc(m, &m->kc, (long)k.n_text_layer * Lt * C);
    rc = rc ? rc : whs_alloc(m, &m->vc, (long)k.n_text_layer * Lt * C);
    rc = rc ? rc : whs_alloc(m, &m->dx, Lt * C);
    rc = rc ? rc : whs_alloc(m, &m->dxn, Lt * C);
    rc = rc ? rc : whs_alloc(m, &m->dq, Lt * C);
    rc = rc ? rc : whs_alloc(m, &m->datt, Lt * C);
    rc = rc ? rc : whs_alloc(m, &m->dmid, Lt * 4 * C);
    rc = rc ? rc : whs_alloc(m, &m->apart, (long)k.n_text_head * (((T > Lt ? T : Lt) + AD_CHUNK - 1) / AD_CHUNK) * 66);
    if (rc) {
        whs_destroy(m);
        return rc;
    }
    *out = m;
    return 0;
}

int whs_destroy(whs_model* m) {
    if (!m) return 0;
    float* bufs[] = {m->frames, m->spec, m->pw, m->lm, m->col, m->h1, m->x, m->xn, m->qkv, m->att,
                     m->mid, m->ck, m->cv, m->kc, m->vc, m->dx, m->dxn, m->dq, m->datt, m->dmid, m->apart};
    for (float* b : bufs)
        if (b) (void)hipFree(b);
    delete m;
    return 0;
}

int64_t whs_workspace_bytes(const whs_model* m) { return m ? (int64_t)m->bytes : 0; }

int32_t whs_mel_frames(const whs_model* m, int32_t n_samples) {
    if (!m || n_samples < 0) return -1;
    return n_samples / WHS_HOP + WHS_N_FRAMES;
}

int whs_log_mel(whs_model* m, const float* wav, int32_t n, float* mel_out, void* stream) {
    if (!m || (!wav && n > 0) || n < 0) return -1;
    if (n > m->cfg.max_samples) return -5;
    hipStream_t st = (hipStream_t)stream;
    const whs_weights& w = m->w;
    const int nm = m->cfg.n_mels;
    const int n_total = n + WHS_N_FRAMES * WHS_HOP;
    const int F = n_total / WHS_HOP;   // stft frames = n_total / hop + 1, the last one dropped
    hipLaunchKernelGGL(whs_frames_kernel, dim3(F), dim3(128), 0, st, wav, n, n_total, w.window, m->frames);
    WH_LAUNCHED();
    WH_TRY(gemm(wg(m->frames, WHS_FFT_K, w.dft, WHS_FFT_K, 2 * WHS_BINS, nullptr, m->spec, WHS_FFT_K, F), st));
    hipLaunchKernelGGL(whs_power_kernel, dim3(F), dim3(256), 0, st, m->spec, m->pw);
    WH_LAUNCHED();
    {
        GemmArgs g = wg(m->pw, WHS_BINS_PAD, w.mel, WHS_BINS_PAD, nm, nullptr, m->lm, nm, F);
        g.epi = EPI_LOG10;
        WH_TRY(gemm(g, st));
    }
    hipLaunchKernelGGL(whs_mel_norm_kernel, dim3(1), dim3(1024), 0, st, m->lm, (long)F * nm);
    WH_LAUNCHED();
    m->mel_frames = F;
    if (mel_out &&
        hipMemcpyAsync(mel_out, m->lm, (size_t)F * nm * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return -2;
    return 0;
}

int whs_encode(whs_model* m, int32_t seek, int32_t seg_frames, float* feat_out, void* stream) {
    if (!m || seek < 0 || seg_frames < 0 || seg_frames > WHS_N_FRAMES || seek + seg_frames > m->mel_frames) return -1;
    hipStream_t st = (hipStream_t)stream;
    const whs_config& k = m->cfg;
    const whs_weights& w = m->w;
    const int C = k.n_audio_state, T = k.n_audio_ctx, nm = k.n_mels, H = k.n_audio_head;
    // conv stem: GELU(conv1(mel window)), GELU(conv2(.)) + positional embedding
    {
        const long n1 = (long)WHS_N_FRAMES * w.conv1_kpad;
        hipLaunchKernelGGL(whs_im2col_kernel, dim3((unsigned)((n1 + 255) / 256)), dim3(256), 0, st,
                           m->lm + (long)seek * nm, seg_frames, nm, 1, 1, m->col, WHS_N_FRAMES, w.conv1_kpad);
        WH_LAUNCHED();
        GemmArgs g = wg(m->col, w.conv1_kpad, w.conv1_w, w.conv1_kpad, C, w.conv1_b, m->h1, C, WHS_N_FRAMES);
        g.epi = EPI_GELU;
        WH_TRY(gemm(g, st));
        const long n2 = (long)T * w.conv2_kpad;
        hipLaunchKernelGGL(whs_im2col_kernel, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, st, m->h1,
                           WHS_N_FRAMES, C, 2, 1, m->col, T, w.conv2_kpad);
        WH_LAUNCHED();
        GemmArgs g2 = wg(m->col, w.conv2_kpad, w.conv2_w, w.conv2_kpad, C, w.conv2_b, m->x, C, T);
        g2.epi = EPI_GELU;
        g2.resid = w.enc_pos;
        WH_TRY(gemm(g2, st));
    }
    for (int l = 0; l < k.n_audio_layer; ++l) {
        const whs_block& L = w.enc[l];
        WH_TRY(whs_ln(m->x, m->xn, T, C, L.attn_ln_w, L.attn_ln_b, st));
        WH_TRY(gemm(wg(m->xn, C, L.attn.q_w, C, C, L.attn.q_b, m->qkv, 3 * C, T), st));
        WH_TRY(gemm(wg(m->xn, C, L.attn.k_w, C, C, nullptr, m->qkv + C, 3 * C, T), st));
        WH_TRY(gemm(wg(m->xn, C, L.attn.v_w, C, C, L.attn.v_b, m->qkv + 2 * C, 3 * C, T), st));
        WH_TRY(whs_attention(m->qkv, 3 * C, m->qkv + C, m->qkv + 2 * C, 3 * C, m->att, C, T, T, H, 0, 0, st));
        GemmArgs g = wg(m->att, C, L.attn.o_w, C, C, L.attn.o_b, m->x, C, T);
        g.resid = m->x;
        WH_TRY(gemm(g, st));
        WH_TRY(whs_mlp(L, m->x, m->xn, m->mid, T, C, st));
    }
    WH_TRY(whs_ln(m->x, m->xn, T, C, w.enc_ln_w, w.enc_ln_b, st));
    // every decoder layer's cross-attention K / V of this window
    for (int l = 0; l < k.n_text_layer; ++l) {
        const whs_attn& A = w.dec[l].cross;
        WH_TRY(gemm(wg(m->xn, C, A.k_w, C, C, nullptr, m->ck + (long)l * T * C, C, T), st));
        WH_TRY(gemm(wg(m->xn, C, A.v_w, C, C, A.v_b, m->cv + (long)l * T * C, C, T), st));
    }
    m->encoded = 1;
    if (feat_out &&
        hipMemcpyAsync(feat_out, m->xn, (size_t)T * C * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return -2;
    return 0;
}

int whs_decode(whs_model* m, const int32_t* tokens, int32_t n, int32_t offset, float* logits, void* stream) {
    if (!m || !tokens || !logits || n <= 0 || offset < 0 || offset + n > m->cfg.n_text_ctx || !m->encoded) return -1;
    hipStream_t st = (hipStream_t)stream;
    const whs_config& k = m->cfg;
    const whs_weights& w = m->w;
    const int C = k.n_text_state, T = k.n_audio_ctx, H = k.n_text_head, Lt = k.n_text_ctx;
    hipLaunchKernelGGL(whs_embed_kernel, dim3(n), dim3(256), 0, st, tokens, w.tok_emb, w.dec_pos, offset, C, k.n_vocab,
                       m->dx);
    WH_LAUNCHED();
    for (int l = 0; l < k.n_text_layer; ++l) {
        const whs_block& L = w.dec[l];
        float* kc = m->kc + (long)l * Lt * C;
        float* vc = m->vc + (long)l * Lt * C;
        // self attention: this call's K / V rows land at cache rows offset..offset+n-1
        WH_TRY(whs_ln(m->dx, m->dxn, n, C, L.attn_ln_w, L.attn_ln_b, st));
        WH_TRY(dgemm(wg(m->dxn, C, L.attn.q_w, C, C, L.attn.q_b, m->dq, C, n), st));
        {
            GemmArgs g = wg(m->dxn, C, L.attn.k_w, C, C, nullptr, kc, C, n);
            g.cm = RowMap{n, 0, offset};
            WH_TRY(dgemm(g, st));
            GemmArgs g2 = wg(m->dxn, C, L.attn.v_w, C, C, L.attn.v_b, vc, C, n);
            g2.cm = RowMap{n, 0, offset};
            WH_TRY(dgemm(g2, st));
        }
        WH_TRY(dec_attention(m, m->dq, kc, vc, C, m->datt, n, offset + n, H, 1, offset, st));
        {
            GemmArgs g = wg(m->datt, C, L.attn.o_w, C, C, L.attn.o_b, m->dx, C, n);
            g.resid = m->dx;
            WH_TRY(dgemm(g, st));
        }
        // cross attention over the encoded window
        WH_TRY(whs_ln(m->dx, m->dxn, n, C, L.cross_ln_w, L.cross_ln_b, st));
        WH_TRY(dgemm(wg(m->dxn, C, L.cross.q_w, C, C, L.cross.q_b, m->dq, C, n), st));
        WH_TRY(dec_attention(m, m->dq, m->ck + (long)l * T * C, m->cv + (long)l * T * C, C, m->datt, n, T, H, 0, 0,
                             st));
        {
            GemmArgs g = wg(m->datt, C, L.cross.o_w, C, C, L.cross.o_b, m->dx, C, n);
            g.resid = m->dx;
            WH_TRY(dgemm(g, st));
        }
        WH_TRY(whs_mlp(L, m->dx, m->dxn, m->dmid, n, C, st));
    }
    WH_TRY(whs_ln(m->dx, m->dxn, n, C, w.dec_ln_w, w.dec_ln_b, st));
    return dgemm(wg(m->dxn, C, w.tok_emb, C, k.n_vocab, nullptr, logits, k.n_vocab, n), st);
}

}  // extern "C"

// XCodec2 codec ENCODER (16 kHz waveform -> codec ids) for gfx950, fp32 end to end.
//
// Restates the encoder the reference reaches through AudioTokenizer.encode
// (data/tokenizer.py:105-115 -> pip xcodec2 encode_code); architecture per the
// transformers port ([tf] models/xcodec2/modeling_xcodec2.py Xcodec2Model.encode
// :974-1024) and its semantic model ([tf] models/wav2vec2_bert/modeling_wav2vec2_bert.py),
// fed by the Kaldi-style fbank of SeamlessM4TFeatureExtractor (the pip package's front
// end, [tf] models/seamless_m4t/feature_extraction_seamless_m4t.py:112-138, 256-292).
// See include/xc2.h for the data flow.
//
// HBM layout: every activation is time-major [T][width] fp32 for ONE utterance. Convs
// run as im2col (zero padding, stride, dilation; K padded to a multiple of 32) + the
// f32 MFMA GEMM; the FFT of the fbank is a DFT GEMM against a cos/sin basis. Kernels
// here are the row-wise / elementwise pieces between GEMMs.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "xc2.h"
#include "xc2_common.h"

namespace xc2 {
namespace {

constexpr int FB_WIN = 400, FB_SHIFT = 160, FB_FFT = 512, FB_BINS = 257, FB_POW_LD = 288, FB_SPEC_LD = 544,
              FB_MELS = 80;

// ---------------------------------------------------------------- fbank front end
// One frame per block (512 threads = FFT buffer slots): samples of the 16 kHz input
// scaled to int16 range, the n_pad-sample signal with 160 zeros either side
// (pip encode_code: F.pad(wav, (160, 160))), DC removal, pre-emphasis 0.97 (first
// sample x 0.03), povey window; slots >= 400 are the FFT zero padding
// (audio_utils.spectrogram, remove_dc_offset + preemphasis + window).
__global__ __launch_bounds__(512) void fbank_frames_kernel(const float* wav, int n, float* frames,
                                                           const float* window) {
    __shared__ float red[8];
    __shared__ float xs[FB_WIN];
    const int f = blockIdx.x, i = threadIdx.x;
    const long s = (long)f * FB_SHIFT + i - FB_SHIFT;
    const float x = (i < FB_WIN && s >= 0 && s < n) ? wav[s] * 32768.0f : 0.f;
    const float mean = bsum(x, red) / (float)FB_WIN;
    const float xc = x - mean;
    if (i < FB_WIN) xs[i] = xc;
    __syncthreads();
    float y = 0.f;
    if (i < FB_WIN) {
        y = i == 0 ? xc * (1.0f - 0.97f) : xc - 0.97f * xs[i - 1];
        y *= window[i];
    }
    frames[(long)f * FB_FFT + i] = y;
}

// |X_k|^2 from the DFT GEMM's interleaved (re, im) columns; bins >= 257 zero
__global__ void fbank_power_kernel(const float* spec, float* pw) {
    const int f = blockIdx.x;
    for (int k = threadIdx.x; k < FB_POW_LD; k += blockDim.x) {
        float v = 0.f;
        if (k < FB_BINS) {
            const float re = spec[(long)f * FB_SPEC_LD + 2 * k], im = spec[(long)f * FB_SPEC_LD + 2 * k + 1];
            v = re * re + im * im;
        }
        pw[(long)f * FB_POW_LD + k] = v;
    }
}

// per mel bin over the utterance's frames: (x - mean) / sqrt(unbiased var + 1e-7)
// (feature_extraction_seamless_m4t.py:256-260), in place on [F][80]
__global__ __launch_bounds__(256) void fbank_norm_kernel(float* lm, int F) {
    __shared__ float red[8];
    const int c = blockIdx.x;
    float s = 0.f;
    for (int r = threadIdx.x; r < F; r += blockDim.x) s += lm[(long)r * FB_MELS + c];
    const float mean = bsum(s, red) / (float)F;
    float ss = 0.f;
    for (int r = threadIdx.x; r < F; r += blockDim.x) {
        const float d = lm[(long)r * FB_MELS + c] - mean;
        ss += d * d;
    }
    const float var = bsum(ss, red) / (float)max(F - 1, 1);
    const float inv = 1.0f / sqrtf(var + 1e-7f);
    for (int r = threadIdx.x; r < F; r += blockDim.x) {
        const long o = (long)r * FB_MELS + c;
        lm[o] = (lm[o] - mean) * inv;
    }
}

// ------------------------------------------------------------------------- im2col
// out[t][k * cin + ci] = X[t * stride + k * dil - pad][ci] (0 outside [0, T_in)), columns
// k_taps * cin .. kpad - 1 zero: the A operand of a Conv1d as GEMM
__global__ void im2col_kernel(const float* X, int T_in, int cin, int k_taps, int stride, int dil, int pad, float* out,
                              int T_out, int kpad) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)T_out * kpad) return;
    const int t = (int)(idx / kpad), col = (int)(idx - (long)t * kpad);
    float v = 0.f;
    if (col < k_taps * cin) {
        const int k = col / cin, ci = col - k * cin;
        const int ti = t * stride + k * dil - pad;
        if (ti >= 0 && ti < T_in) v = X[(long)ti * cin + ci];
    }
    out[idx] = v;
}

// ------------------------------------------------- anti-aliased SnakeBeta activation
// [tf] Xcodec2AntiAliasedActivation1d :524-545: UpSample1d(2, 12 taps: replicate pad 5,
// conv_transpose stride 2, crop 15 / 15, x 2) -> SnakeBeta (x + 1/(e^beta + 1e-9)
// sin^2(x e^alpha)) -> DownSample1d(2, 12 taps: replicate pad 5 / 6, conv stride 2).
// One thread per (t, c); the 12 up-sampled values an output needs are rebuilt in place.
__global__ void aa_snake_kernel(const float* X, float* Y, int T, int C, const float* alpha_log,
                                const float* beta_log, const float* fu, const float* fd) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)T * C) return;
    const int t = (int)(idx / C), c = (int)(idx - (long)t * C);
    const float a = expf(alpha_log[c]);
    const float ib = 1.0f / (expf(beta_log[c]) + 1e-9f);
    const int T2 = 2 * T;
    float y = 0.f;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const int u = min(max(2 * t + k - 5, 0), T2 - 1);   // replicate pad of the down-sampler
        // up[u] = 2 * sum_i xp[i] fu[o - 2i], o = u + 15, xp[i] = X[clamp(i - 5)]
        const int o = u + 15;
        const int i_hi = o >> 1;
        float up = 0.f;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const int i = i_hi - j;
            const int kk = o - 2 * i;   // 0 or 1 for j = 0 ... up to 11
            if (kk < 12) {
                const int ts = min(max(i - 5, 0), T - 1);
                up += X[(long)ts * C + c] * fu[kk];
            }
        }
        up *= 2.0f;
        const float sn = sinf(up * a);
        const float z = up + ib * (sn * sn);
        y += fd[k] * z;
    }
    Y[idx] = y;
}

// Same activation, 4 consecutive outputs of one channel per thread: their 18 up-sampled
// values come from 14 input rows held in registers (the per-output form rebuilds 48 up
// values from 288 loads). Same operations in the same order, so bit-identical to
// aa_snake_kernel. Groups whose up-sample window reaches the replicate-padded edges
// (t0 < 3 or t0 > T - 7) take the per-output form. Needs T % 4 == 0.
__global__ void aa_snake4_kernel(const float* X, float* Y, int T, int C, const float* alpha_log,
                                 const float* beta_log, const float* fu, const float* fd) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)(T / 4) * C) return;
    const int tg = (int)(idx / C), c = (int)(idx - (long)tg * C);
    const int t0 = 4 * tg;
    const float a = expf(alpha_log[c]);
    const float ib = 1.0f / (expf(beta_log[c]) + 1e-9f);
    float fuv[12], fdv[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        fuv[k] = fu[k];
        fdv[k] = fd[k];
    }
    if (t0 >= 3 && t0 <= T - 7) {
        float x[14];
#pragma unroll
        for (int r = 0; r < 14; ++r) x[r] = X[(long)min(max(t0 + r - 5, 0), T - 1) * C + c];
        float z[18];
#pragma unroll
        for (int j = 0; j < 18; ++j) {
            // u = 2 t0 - 5 + j, o = u + 15: i = (o >> 1) - jj = t0 + 5 + (j >> 1) - jj,
            // tap kk = o - 2 i = (j & 1) + 2 jj, input row i - 5 -> x[(i - t0)]
            float up = 0.f;
#pragma unroll
            for (int jj = 0; jj < 6; ++jj) up += x[5 + (j >> 1) - jj] * fuv[(j & 1) + 2 * jj];
            up *= 2.0f;
            const float sn = sinf(up * a);
            z[j] = up + ib * (sn * sn);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float y = 0.f;
#pragma unroll
            for (int k = 0; k < 12; ++k) y += fdv[k] * z[2 * q + k];
            Y[(long)(t0 + q) * C + c] = y;
        }
        return;
    }
    const int T2 = 2 * T;
    for (int q = 0; q < 4; ++q) {
        const int t = t0 + q;
        float y = 0.f;
        for (int k = 0; k < 12; ++k) {
            const int u = min(max(2 * t + k - 5, 0), T2 - 1);
            const int o = u + 15;
            const int i_hi = o >> 1;
            float up = 0.f;
            for (int j = 0; j < 6; ++j) {
                const int i = i_hi - j;
                const int ts = min(max(i - 5, 0), T - 1);
                up += X[(long)ts * C + c] * fuv[o - 2 * i];
            }
            up *= 2.0f;
            const float sn = sinf(up * a);
            const float z = up + ib * (sn * sn);
            y += fdv[k] * z;
        }
        Y[(long)t * C + c] = y;
    }
}

// ------------------------------------------------- conformer convolution module middle
// [tf] Wav2Vec2BertConvolutionModule :196-227 between the two pointwise convs:
// GLU over the pointwise_conv1 output (a * sigmoid(b), a = first H channels), causal
// depthwise conv (kernel KW, left pad KW - 1), LayerNorm, swish. One block per frame,
// 4 channels per thread.
__global__ __launch_bounds__(256) void glu_dwconv_ln_swish_kernel(const float* P1, int H, int KW, const float* dw,
                                                                  const float* lw, const float* lb, float eps,
                                                                  float* out) {
    __shared__ float red[8];
    const int t = blockIdx.x;
    const int c = threadIdx.x * 4;
    const bool act = c < H;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (act) {
        for (int k = 0; k < KW; ++k) {
            const int r = t - (KW - 1) + k;
            if (r < 0) continue;
            const f32x4 av = *(const f32x4*)(P1 + (long)r * 2 * H + c);
            const f32x4 bv = *(const f32x4*)(P1 + (long)r * 2 * H + H + c);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] += dw[(long)(c + e) * KW + k] * (av[e] / (1.0f + expf(-bv[e])));
        }
    }
    const float mean = bsum(act ? (acc[0] + acc[1]) + (acc[2] + acc[3]) : 0.f, red) / (float)H;
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) ss += act ? (acc[e] - mean) * (acc[e] - mean) : 0.f;
    const float rstd = 1.0f / sqrtf(bsum(ss, red) / (float)H + eps);
    if (!act) return;
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const float v = (acc[e] - mean) * rstd * lw[c + e] + lb[c + e];
        y[e] = v / (1.0f + expf(-v));
    }
    *(f32x4*)(out + (long)t * H + c) = y;
}

// ------------------------------------------------------ relative-key self attention
// [tf] Wav2Vec2BertSelfAttention :263-330 with position_embeddings_type "relative_key":
// scores = (q.k + q.E[clamp(j - i, -L, R) + L]) / sqrt(64), softmax over all frames of
// the utterance (no mask), P.V. q.E comes precomputed (QE [T][heads][L + R + 1], one GEMM).
// Block = 4 waves x 32 queries of one head; K/V tiles of 64 frames in LDS; S^T = K Q^T so
// probabilities are the B operand of O^T = V^T P^T (the decoder's attn_f32_kernel scheme).
constexpr int AQ = 128, AK = 64, ALD = 68;

__global__ __launch_bounds__(256) void attn_relkey_kernel(const float* QKV, int ldq, int C, int heads, float* O, int T,
                                                          float scale, const float* QE, int L, int R) {
    __shared__ float sm[2 * AK * ALD];
    float* Ks = sm;
    float* Vs = sm + AK * ALD;
    const int h = blockIdx.y, q0 = blockIdx.x * AQ;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, hh = lane >> 5;
    const int nrel = L + R + 1;
    const int qi = q0 + w * 32 + li;
    const bool qv = qi < T;
    const float* qe = QE + ((long)min(qi, T - 1) * heads + h) * nrel;
    f32x4 qf[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (qv) v = *(const f32x4*)(QKV + (long)qi * ldq + h * 64 + 8 * g + 4 * hh);
        qf[g] = v * scale;
    }
    f32x16 oacc[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[0][r] = oacc[1][r] = 0.f;
    float mrun = -INFINITY, lrun = 0.f;
    for (int k0 = 0; k0 < T; k0 += AK) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (tid >> 4) + 16 * i, c4 = (tid & 15) * 4;
            const int kr = k0 + row;
            f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = kv;
            if (kr < T) {
                const float* src = QKV + (long)kr * ldq + h * 64 + c4;
                kv = *(const f32x4*)(src + C);
                vv = *(const f32x4*)(src + 2 * C);
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
                const int dist = min(max(key - qi, -L), R) + L;
                s[kt][r] = key < T ? s[kt][r] + qe[dist] * scale : -INFINITY;
                mx = fmaxf(mx, s[kt][r]);
            }
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
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
        if (q < T) *(f32x4*)(O + (long)q * C + h * 64 + c4) = *(const f32x4*)&slab[qq * ALD + c4];
    }
}

// ------------------------------------------------------------------------------ FSQ
// [tf] Xcodec2Quantizer.forward :811-818 + Xcodec2FiniteScalarQuantization :706-744:
// bound() applied twice (the quantizer bounds, then FSQ.forward bounds again), round
// half to even, digit = rounded + L/2, id = sum_j digit_j L^j.
__global__ void fsq_encode_kernel(const float* Pj, int T, int nl, int level, int* codes, float* latent) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const float half_range = (float)(level - 1) * (1.0f + 1e-3f) / 2.0f;
    const float offset = (level % 2 == 0) ? 0.5f : 0.0f;
    const float shift = atanhf(offset / half_range);
    const int half = level / 2;
    long id = 0, base = 1;
    for (int j = 0; j < nl; ++j) {
        float v = Pj[(long)t * nl + j];
        if (latent) latent[(long)t * nl + j] = v;
        v = tanhf(v + shift) * half_range - offset;
        v = tanhf(v + shift) * half_range - offset;
        const int digit = (int)rintf(v) + half;
        id += (long)digit * base;
        base *= level;
    }
    codes[t] = (int)id;
}

}  // namespace
}  // namespace xc2

using namespace xc2;

struct xc2_encoder {
    xc2e_config cfg;
    xc2e_weights w;
    int T_max, n_pad_max;
    // semantic
    float *frames, *spec, *pw, *lm, *fpn, *x, *xn, *mid, *qkv, *qe, *att, *p1, *dwo;
    // adapter / acoustic / head
    float *col, *a1, *a2, *cat, *fcout, *proj;
    float *ac0, *ac1, *ac_y, *ac_t;
    size_t bytes;
};

static int enc_alloc(xc2_encoder* e, float** p, long floats) {
    const size_t b = (size_t)max(floats, 1L) * sizeof(float);
    if (hipMalloc((void**)p, b) != hipSuccess) return -4;
    if (hipMemset(*p, 0, b) != hipSuccess) return -2;
    e->bytes += b;
    return 0;
}

static GemmArgs eg(const float* A, int lda, const float* W, int K, int N, const float* bias, float* Cp, int ldc, int M) {
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

#define XE_TRY(x)            \
    do {                     \
        int _rc = (x);       \
        if (_rc) return _rc; \
    } while (0)
#define XE_LAUNCHED() \
    do { if (hipGetLastError() != hipSuccess) return -2; } while (0)

static int conv_out_len(const xc2e_conv& c, int T_in) { return (T_in + 2 * c.pad - c.dil * (c.k - 1) - 1) / c.stride + 1; }

// Conv1d over [T_in][cin] -> [T_out][cout] (+ bias, + resid, epilogue) via im2col + GEMM
static int conv(xc2_encoder* e, const xc2e_conv& c, const float* X, int T_in, float* Y, int ldy, const float* resid,
                int epi, hipStream_t st, int* T_out_p = nullptr) {
    const int T_out = conv_out_len(c, T_in);
    if (T_out <= 0) return -1;
    const long n = (long)T_out * c.kpad;
    hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, T_in, c.cin, c.k,
                       c.stride, c.dil, c.pad, e->col, T_out, c.kpad);
    XE_LAUNCHED();
    GemmArgs g = eg(e->col, c.kpad, c.w, c.kpad, c.cout, c.b, Y, ldy, T_out);
    g.resid = resid;
    g.epi = epi;
    if (T_out_p) *T_out_p = T_out;
    return gemm(g, st);
}

static int snake(const float* X, float* Y, int T, int C, const xc2e_snake& s, const xc2e_weights& w, hipStream_t st) {
    if (T % 4 == 0 && T >= 8) {
        const long n = (long)(T / 4) * C;
        hipLaunchKernelGGL(aa_snake4_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, Y, T, C,
                           s.alpha, s.beta, w.aa_up, w.aa_down);
        XE_LAUNCHED();
        return 0;
    }
    const long n = (long)T * C;
    hipLaunchKernelGGL(aa_snake_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, X, Y, T, C, s.alpha,
                       s.beta, w.aa_up, w.aa_down);
    XE_LAUNCHED();
    return 0;
}

static int layer_norm(const float* X, float* Y, int T, int C, const float* lw, const float* lb, float eps,
                      hipStream_t st) {
    // whole waves (a partial wave's cross-lane sums would read inactive lanes)
    hipLaunchKernelGGL(rownorm_kernel, dim3(T), dim3(((C / 4 + 63) / 64) * 64), 0, st, X, Y, RowMap{T, 0, 0}, C, lw, lb,
                       eps, 1);
    XE_LAUNCHED();
    return 0;
}

extern "C" {

int xc2e_create(const xc2e_config* cfg, const xc2e_weights* w, xc2_encoder** out) {
    if (!cfg || !w || !out) return -1;
    const xc2e_config& k = *cfg;
    const int H = k.sem_hidden;
    if (H <= 0 || H % 128 || H > 1024 || k.sem_heads * 64 != H || k.sem_intermediate % 32 || k.sem_layers < 0 ||
        k.sem_layers > XC2E_MAX_LAYERS || k.feat_dim != 2 * FB_MELS || k.dw_kernel < 1 || k.rel_left < 0 ||
        k.rel_right < 0 || k.n_blocks < 1 || k.n_blocks > XC2E_MAX_BLOCKS || k.hidden % 32 || k.hidden > 4096 ||
        k.n_levels < 1 || k.n_levels > 16 || k.level < 2 || k.max_samples <= 0 || k.ac_channels0 <= 0)
        return -1;
    int hop = 1;
    for (int i = 0; i < k.n_blocks; ++i) {
        if (k.strides[i] < 1) return -1;
        hop *= k.strides[i];
    }
    if (hop != FB_SHIFT * 2) return -1;   // semantic frames (2 x 10 ms) must align with codes
    xc2_encoder* e = new xc2_encoder();
    memset(e, 0, sizeof(*e));
    e->cfg = k;
    e->w = *w;
    e->T_max = k.max_samples / hop + 1;
    e->n_pad_max = e->T_max * hop;
    const long T = e->T_max, F = 2 * T, I = k.sem_intermediate, nrel = k.rel_left + k.rel_right + 1;
    const long W2 = H + k.hidden;
    // acoustic activations: the widest (time x channels) stage, and the widest im2col
    long act = (long)e->n_pad_max * k.ac_channels0, col = (long)e->n_pad_max * w->ac_in.kpad;
    {
        long Tl = e->n_pad_max;
        for (int b = 0; b < k.n_blocks; ++b) {
            const xc2e_block& B = w->blocks[b];
            for (int r = 0; r < 3; ++r) {
                col = max(col, Tl * (long)B.ru[r].c1.kpad);
                col = max(col, Tl * (long)B.ru[r].c2.kpad);
            }
            act = max(act, Tl * (long)B.ru[0].c1.cin);
            Tl = Tl / k.strides[b];
            col = max(col, Tl * (long)B.down.kpad);
            act = max(act, Tl * (long)B.down.cout);
        }
        col = max(col, Tl * (long)w->ac_out.kpad);
        for (int i = 0; i < 4; ++i) col = max(col, T * (long)w->adapter[i].kpad);
    }
    int rc = 0;
    rc = rc ? rc : enc_alloc(e, &e->frames, F * FB_FFT);
    rc = rc ? rc : enc_alloc(e, &e->spec, F * FB_SPEC_LD);
    rc = rc ? rc : enc_alloc(e, &e->pw, F * FB_POW_LD);
    rc = rc ? rc : enc_alloc(e, &e->lm, F * FB_MELS);
    rc = rc ? rc : enc_alloc(e, &e->fpn, T * k.feat_dim);
    rc = rc ? rc : enc_alloc(e, &e->x, T * H);
    rc = rc ? rc : enc_alloc(e, &e->xn, T * H);
    rc = rc ? rc : enc_alloc(e, &e->mid, T * I);
    rc = rc ? rc : enc_alloc(e, &e->qkv, T * 3 * H);
    rc = rc ? rc : enc_alloc(e, &e->qe, T * k.sem_heads * nrel);
    rc = rc ? rc : enc_alloc(e, &e->att, T * H);
    rc = rc ? rc : enc_alloc(e, &e->p1, T * 2 * H);
    rc = rc ? rc : enc_alloc(e, &e->dwo, T * H);
    rc = rc ? rc : enc_alloc(e, &e->col, col);
    rc = rc ? rc : enc_alloc(e, &e->a1, T * H);
    rc = rc ? rc : enc_alloc(e, &e->a2, T * H);
    rc = rc ? rc : enc_alloc(e, &e->cat, T * W2);
    rc = rc ? rc : enc_alloc(e, &e->fcout, T * W2);
    rc = rc ? rc : enc_alloc(e, &e->proj, T * k.n_levels);
    rc = rc ? rc : enc_alloc(e, &e->ac0, act);
    rc = rc ? rc : enc_alloc(e, &e->ac1, act);
    rc = rc ? rc : enc_alloc(e, &e->ac_y, act);
    rc = rc ? rc : enc_alloc(e, &e->ac_t, act);
    if (rc) {
        xc2e_destroy(e);
        return rc;
    }
    *out = e;
    return 0;
}

int xc2e_destroy(xc2_encoder* e) {
    if (!e) return 0;
    float* bufs[] = {e->frames, e->spec, e->pw, e->lm, e->fpn, e->x, e->xn, e->mid, e->qkv, e->qe, e->att, e->p1,
                     e->dwo, e->col, e->a1, e->a2, e->cat, e->fcout, e->proj, e->ac0, e->ac1, e->ac_y, e->ac_t};
    for (float* b : bufs)
        if (b) (void)hipFree(b);
    delete e;
    return 0;
}

int64_t xc2e_workspace_bytes(const xc2_encoder* e) { return e ? (int64_t)e->bytes : 0; }

int32_t xc2e_num_codes(const xc2_encoder* e, int32_t n_samples) {
    if (!e || n_samples < 0) return -1;
    return n_samples / (2 * FB_SHIFT) + 1;
}

// fbank front end: [2T][80] normalised log-mel in e->lm (= the stacked [T][160] features)
static int fbank(xc2_encoder* e, const float* wav, int n, int T, hipStream_t st) {
    const xc2e_weights& w = e->w;
    const int F = 2 * T;
    hipLaunchKernelGGL(fbank_frames_kernel, dim3(F), dim3(512), 0, st, wav, n, e->frames, w.window);
    XE_LAUNCHED();
    XE_TRY(gemm(eg(e->frames, FB_FFT, w.dft, FB_FFT, 2 * FB_BINS, nullptr, e->spec, FB_SPEC_LD, F), st));
    hipLaunchKernelGGL(fbank_power_kernel, dim3(F), dim3(128), 0, st, e->spec, e->pw);
    XE_LAUNCHED();
    {
        GemmArgs g = eg(e->pw, FB_POW_LD, w.mel, FB_POW_LD, FB_MELS, nullptr, e->lm, FB_MELS, F);
        g.epi = EPI_LOG;
        XE_TRY(gemm(g, st));
    }
    hipLaunchKernelGGL(fbank_norm_kernel, dim3(FB_MELS), dim3(256), 0, st, e->lm, F);
    XE_LAUNCHED();
    return 0;
}

static int semantic(xc2_encoder* e, const float* wav, int n, int T, hipStream_t st) {
    const xc2e_config& k = e->cfg;
    const xc2e_weights& w = e->w;
    const int H = k.sem_hidden, I = k.sem_intermediate, nrel = k.rel_left + k.rel_right + 1;
    const float eps = k.sem_ln_eps;
    XE_TRY(fbank(e, wav, n, T, st));
    // [F][80] row-major is the stacked [T][160] feature matrix
    XE_TRY(layer_norm(e->lm, e->fpn, T, k.feat_dim, w.fp_ln_w, w.fp_ln_b, eps, st));
    XE_TRY(gemm(eg(e->fpn, k.feat_dim, w.fp_w, k.feat_dim, H, w.fp_b, e->x, H, T), st));
    for (int l = 0; l < k.sem_layers; ++l) {
        const xc2e_layer& L = w.layers[l];
        // half-step FFN 1
        XE_TRY(layer_norm(e->x, e->xn, T, H, L.ffn1_ln_w, L.ffn1_ln_b, eps, st));
        {
            GemmArgs g = eg(e->xn, H, L.ffn1_w1, H, I, L.ffn1_b1, e->mid, I, T);
            g.epi = EPI_SILU;
            XE_TRY(gemm(g, st));
            GemmArgs g2 = eg(e->mid, I, L.ffn1_w2, I, H, L.ffn1_b2, e->x, H, T);
            g2.alpha = 0.5f;
            g2.resid = e->x;
            XE_TRY(gemm(g2, st));
        }
        // relative-key self attention
        XE_TRY(layer_norm(e->x, e->xn, T, H, L.attn_ln_w, L.attn_ln_b, eps, st));
        XE_TRY(gemm(eg(e->xn, H, L.qkv_w, H, 3 * H, L.qkv_b, e->qkv, 3 * H, T), st));
        {
            // q . E for every (frame, head): the q block of head h is row t * (3H / 64) + h of
            // the qkv buffer viewed with 64-float rows
            GemmArgs g = eg(e->qkv, 64, L.dist_emb, 64, nrel, nullptr, e->qe, nrel, T * k.sem_heads);
            g.am = RowMap{k.sem_heads, 3 * H / 64, 0};
            XE_TRY(gemm(g, st));
        }
        hipLaunchKernelGGL(attn_relkey_kernel, dim3((T + AQ - 1) / AQ, k.sem_heads), dim3(256), 0, st, e->qkv, 3 * H,
                           H, k.sem_heads, e->att, T, 0.125f, e->qe, k.rel_left, k.rel_right);
        XE_LAUNCHED();
        {
            GemmArgs g = eg(e->att, H, L.o_w, H, H, L.o_b, e->x, H, T);
            g.resid = e->x;
            XE_TRY(gemm(g, st));
        }
        // convolution module
        XE_TRY(layer_norm(e->x, e->xn, T, H, L.conv_ln_w, L.conv_ln_b, eps, st));
        XE_TRY(gemm(eg(e->xn, H, L.pw1_w, H, 2 * H, nullptr, e->p1, 2 * H, T), st));
        hipLaunchKernelGGL(glu_dwconv_ln_swish_kernel, dim3(T), dim3(((H / 4 + 63) / 64) * 64), 0, st, e->p1, H, k.dw_kernel, L.dw_w,
                           L.dw_ln_w, L.dw_ln_b, eps, e->dwo);
        XE_LAUNCHED();
        {
            GemmArgs g = eg(e->dwo, H, L.pw2_w, H, H, nullptr, e->x, H, T);
            g.resid = e->x;
            XE_TRY(gemm(g, st));
        }
        // half-step FFN 2 + final LayerNorm
        XE_TRY(layer_norm(e->x, e->xn, T, H, L.ffn2_ln_w, L.ffn2_ln_b, eps, st));
        {
            GemmArgs g = eg(e->xn, H, L.ffn2_w1, H, I, L.ffn2_b1, e->mid, I, T);
            g.epi = EPI_SILU;
            XE_TRY(gemm(g, st));
            GemmArgs g2 = eg(e->mid, I, L.ffn2_w2, I, H, L.ffn2_b2, e->x, H, T);
            g2.alpha = 0.5f;
            g2.resid = e->x;
            XE_TRY(gemm(g2, st));
        }
        XE_TRY(layer_norm(e->x, e->x, T, H, L.final_ln_w, L.final_ln_b, eps, st));
    }
    // adapter: conv1 -> ReLU (= residual) -> conv2 -> ReLU -> conv3 (+ residual) -> conv4
    const int W2 = H + k.hidden;
    XE_TRY(conv(e, w.adapter[0], e->x, T, e->a1, H, nullptr, EPI_RELU, st));
    XE_TRY(conv(e, w.adapter[1], e->a1, T, e->a2, H, nullptr, EPI_RELU, st));
    XE_TRY(conv(e, w.adapter[2], e->a2, T, e->a2, H, e->a1, EPI_NONE, st));
    return conv(e, w.adapter[3], e->a2, T, e->cat, W2, nullptr, EPI_NONE, st);
}

static int acoustic(xc2_encoder* e, const float* wav, int n, int n_pad, int T, hipStream_t st) {
    const xc2e_config& k = e->cfg;
    const xc2e_weights& w = e->w;
    // zero-padded input [n_pad][1] (ac_y holds it; the encoder never reads past n_pad)
    if (hipMemsetAsync(e->ac_y, 0, (size_t)n_pad * sizeof(float), st) != hipSuccess) return -2;
    if (hipMemcpyAsync(e->ac_y, wav, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess) return -2;
    float* a = e->ac0;
    float* b = e->ac1;
    int Tl = n_pad, C = k.ac_channels0;
    XE_TRY(conv(e, w.ac_in, e->ac_y, Tl, a, C, nullptr, EPI_NONE, st));
    for (int bi = 0; bi < k.n_blocks; ++bi) {
        const xc2e_block& B = w.blocks[bi];
        for (int r = 0; r < 3; ++r) {
            const xc2e_resunit& U = B.ru[r];
            XE_TRY(snake(a, e->ac_y, Tl, C, U.s1, w, st));
            XE_TRY(conv(e, U.c1, e->ac_y, Tl, e->ac_t, C, nullptr, EPI_NONE, st));
            XE_TRY(snake(e->ac_t, e->ac_y, Tl, C, U.s2, w, st));
            XE_TRY(conv(e, U.c2, e->ac_y, Tl, a, C, a, EPI_NONE, st));
        }
        XE_TRY(snake(a, e->ac_y, Tl, C, B.s, w, st));
        int To = 0;
        XE_TRY(conv(e, B.down, e->ac_y, Tl, b, B.down.cout, nullptr, EPI_NONE, st, &To));
        Tl = To;
        C = B.down.cout;
        float* tmp = a;
        a = b;
        b = tmp;
    }
    if (Tl != T) return -1;
    XE_TRY(snake(a, e->ac_y, Tl, C, w.ac_snake, w, st));
    return conv(e, w.ac_out, e->ac_y, Tl, e->cat + k.sem_hidden, k.sem_hidden + k.hidden, nullptr, EPI_NONE, st);
}

int xc2e_encode(xc2_encoder* e, const float* wav, int32_t n, int32_t* codes, float* latent, void* stream) {
    if (!e || !wav || !codes || n < 0) return -1;
    const xc2e_config& k = e->cfg;
    if (n > k.max_samples) return -5;
    hipStream_t st = (hipStream_t)stream;
    const int T = n / (2 * FB_SHIFT) + 1, n_pad = T * 2 * FB_SHIFT;
    const int W2 = k.sem_hidden + k.hidden;
    XE_TRY(semantic(e, wav, n, T, st));
    XE_TRY(acoustic(e, wav, n, n_pad, T, st));
    XE_TRY(gemm(eg(e->cat, W2, e->w.fc_w, W2, W2, e->w.fc_b, e->fcout, W2, T), st));
    XE_TRY(gemm(eg(e->fcout, W2, e->w.pin_w, W2, k.n_levels, e->w.pin_b, e->proj, k.n_levels, T), st));
    hipLaunchKernelGGL(fsq_encode_kernel, dim3((T + 127) / 128), dim3(128), 0, st, e->proj, T, k.n_levels, k.level,
                       codes, latent);
    XE_LAUNCHED();
    return 0;
}

int xc2e_features(xc2_encoder* e, const float* wav, int32_t n, float* feat, void* stream) {
    if (!e || !wav || !feat || n < 0) return -1;
    if (n > e->cfg.max_samples) return -5;
    hipStream_t st = (hipStream_t)stream;
    const int T = n / (2 * FB_SHIFT) + 1;
    XE_TRY(fbank(e, wav, n, T, st));
    return hipMemcpyAsync(feat, e->lm, (size_t)T * 2 * FB_MELS * sizeof(float), hipMemcpyDeviceToDevice, st) ==
                   hipSuccess ? 0 : -2;
}

}  // extern "C"

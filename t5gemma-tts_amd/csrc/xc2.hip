// XCodec2 codec decoder (codes -> waveform) for gfx950, fp32 end to end.
//
// Restates the decoder the reference reaches through AudioTokenizer.decode
// (data/tokenizer.py:117-123 -> pip xcodec2 decode_code; architecture per the
// transformers port [tf] models/xcodec2/modeling_xcodec2.py):
//   FSQ digits (:692-700) -> project_out Linear (:806-809) -> fc Linear (:839)
//   -> Conv1d k7 (:841) -> 2 x ResNet[GN32+SiLU+Conv k3]x2 (:650-661)
//   -> 12 x [RMSNorm -> MHA(RoPE over the HEAD axis :855-857) -> +res
//            -> RMSNorm -> SiLU MLP -> +res] (:344-373)
//   -> 2 x ResNet -> LayerNorm -> ISTFT head (:763-796: Linear, exp/clamp, polar,
//   irfft, Hann, overlap-add, envelope divide).
//
// HBM layout: every activation is time-major [B][P][width] fp32 with P =
// max_frames + 6 rows per sequence and 3 zero halo rows in front, so a Conv1d of
// kernel k over a sequence is a plain GEMM whose A rows overlap (row t starts at
// halo row t - k/2, K = k * width, weights tap-major). Rows t >= len of a conv input
// are written as zeros by their producer, which makes the conv's right edge see the
// same zero padding as the reference.
//
// Every contraction runs on v_mfma_f32_32x32x2_f32 (exact f32 products, f32
// accumulate), so results track the fp32 CPU reference to ~1e-6 relative.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "xc2.h"
#include <vector>
#include "xc2_common.h"

namespace xc2 {

// ------------------------------------------------------------- FSQ + project_out
// [tf] Xcodec2FiniteScalarQuantization._indices_to_codes :692-700 and
// Xcodec2Quantizer.from_codes :806-809. Ids reduce mod level^n_levels (digit formula).
__global__ void fsq_project_kernel(const int* codes, int T, RowMap om, float* out, int ld, const float* W,
                                   const float* bias, int qd, int nl, int level) {
    const int m = blockIdx.x;
    const int b = m / T, t = m - b * T;
    const unsigned id = (unsigned)codes[b * T + t];
    float c[16];
    const int half = level / 2;
    unsigned base = 1;
    for (int j = 0; j < nl; ++j) {
        const int digit = (int)((id / base) % (unsigned)level);
        c[j] = (float)(digit - half) / (float)half;
        base *= (unsigned)level;
    }
    float* o = out + rowaddr(om, m) * ld;
    for (int n = threadIdx.x; n < qd; n += blockDim.x) {
        const float* wr = W + (long)n * nl;
        float s = 0.f;
        for (int j = 0; j < nl; ++j) s = fmaf(c[j], wr[j], s);
        o[n] = s + bias[n];
    }
}

// ---------------------------------------------------------------- polar spectrum
// [tf] Xcodec2ISTFTHead.forward :765-772: magnitude = clamp(exp(mag), max=100),
// spectrum = polar(magnitude, phase). In place on interleaved (mag_k, phase_k) pairs.
__global__ void polar_kernel(float* S, RowMap rm, int ld, int nbins) {
    const long row = rowaddr(rm, blockIdx.x);
    const int k = blockIdx.y * blockDim.x + threadIdx.x;
    if (k >= nbins) return;
    float* p = S + row * ld + 2 * k;
    const float mag = fminf(expf(p[0]), 100.0f);
    float sn, cs;
    sincosf(p[1], &sn, &cs);
    p[0] = mag * cs;
    p[1] = mag * sn;
}

// -------------------------------------------------- GroupNorm(32) + SiLU producer
// [tf] Xcodec2ResNetBlock :650-661 (nn.GroupNorm eps 1e-6, affine; nn.SiLU). One block
// per (sequence, group); two-pass mean / biased variance over len x (C/G) values.
// Writes rows [0, T + 3): zeros for t >= len (the next conv's right padding).
__global__ __launch_bounds__(256) void groupnorm_silu_kernel(const float* X, float* Y, int seq, int C, int G,
                                                             const float* w, const float* bsh, const int* lens,
                                                             int T, float eps) {
    __shared__ float red[8];
    const int b = blockIdx.x / G, g = blockIdx.x - b * G;
    const int cpg = C / G, nq = cpg / 4;
    const int len = lens ? min(lens[b], T) : T;
    const long base = ((long)b * seq + 3) * C + g * cpg;
    const int total = len * nq;
    float s = 0.f;
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
        const int t = i / nq, q = i - t * nq;
        const f32x4 x = *(const f32x4*)(X + base + (long)t * C + 4 * q);
        s += (x[0] + x[1]) + (x[2] + x[3]);
    }
    const float cnt = (float)(len * cpg);
    const float mean = bsum(s, red) / cnt;
    float ss = 0.f;
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
        const int t = i / nq, q = i - t * nq;
        const f32x4 x = *(const f32x4*)(X + base + (long)t * C + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) ss += (x[e] - mean) * (x[e] - mean);
    }
    const float var = bsum(ss, red) / cnt;
    const float rstd = 1.0f / sqrtf(var + eps);
    const int tot2 = (T + 3) * nq;
    for (int i = threadIdx.x; i < tot2; i += blockDim.x) {
        const int t = i / nq, q = i - t * nq;
        f32x4 y = {0.f, 0.f, 0.f, 0.f};
        if (t < len) {
            const f32x4 x = *(const f32x4*)(X + base + (long)t * C + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int c = g * cpg + 4 * q + e;
                y[e] = silu((x[e] - mean) * rstd * w[c] + bsh[c]);
            }
        }
        *(f32x4*)(Y + base + (long)t * C + 4 * q) = y;
    }
}

// ------------------------------------------------------------ RoPE over the heads
// [tf] Xcodec2Decoder.forward :855-857 + apply_rotary_pos_emb(unsqueeze_dim=2): the
// rotation angle of head h is h * inv_freq (constant over time). In place on q, k.
__global__ void rope_heads_kernel(float* QKV, RowMap rm, int ldq, int C, int H, const float* cs,
                                  const float* sn) {
    const long row = rowaddr(rm, blockIdx.x);
    for (int i = threadIdx.x; i < 2 * H * 32; i += blockDim.x) {
        const int which = i / (H * 32), h = (i / 32) % H, d = i & 31;
        float* p = QKV + row * ldq + which * C + h * 64;
        const float x1 = p[d], x2 = p[d + 32];
        const float c = cs[h * 32 + d], s = sn[h * 32 + d];
        p[d] = __fadd_rn(__fmul_rn(x1, c), __fmul_rn(-x2, s));
        p[d + 32] = __fadd_rn(__fmul_rn(x2, c), __fmul_rn(x1, s));
    }
}

// ------------------------------------------------------------------ attention
// Bidirectional MHA over the frames of one sequence, head_dim 64, fp32 online softmax
// ([tf] Xcodec2Attention :268-310, no mask, scale head_dim^-0.5). Block = 4 waves x 32
// queries of one (sequence, head); K/V tiles of 64 keys in LDS. Scores are computed
// transposed (S^T = K Q^T: keys on the MFMA rows, queries on lanes) so that the
// probabilities are already the B operand of O^T = V^T P^T, no lane movement.
constexpr int AQ = 128, AK = 64, ALD = 68;

__global__ __launch_bounds__(256) void attn_f32_kernel(const float* QKV, int seq, int ldq, int C, float* O,
                                                       const int* lens, int T, float scale) {
    __shared__ float sm[2 * AK * ALD];
    float* Ks = sm;
    float* Vs = sm + AK * ALD;
    const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * AQ;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 31, hh = lane >> 5;
    const int len = lens ? min(lens[b], T) : T;
    if (q0 >= len) return;
    const long rbase = (long)b * seq + 3;
    const int qi = q0 + w * 32 + li;
    const bool qv = qi < len;
    f32x4 qf[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (qv) v = *(const f32x4*)(QKV + (rbase + qi) * ldq + h * 64 + 8 * g + 4 * hh);
        qf[g] = v * scale;
    }
    f32x16 oacc[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) oacc[0][r] = oacc[1][r] = 0.f;
    float mrun = -INFINITY, lrun = 0.f;
    for (int k0 = 0; k0 < len; k0 += AK) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = (tid >> 4) + 16 * i, c4 = (tid & 15) * 4;
            const int kr = k0 + row;
            f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = kv;
            if (kr < len) {
                const float* src = QKV + (rbase + kr) * ldq + h * 64 + c4;
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
                if (key >= len) s[kt][r] = -INFINITY;
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
    // transpose O^T through LDS (wave-private 32 x 68 slab) and write rows of 64
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
        if (q < len) *(f32x4*)(O + (rbase + q) * C + h * 64 + c4) = *(const f32x4*)&slab[qq * ALD + c4];
    }
}

// ------------------------------------------------------------ overlap-add + norm
// [tf] Xcodec2ISTFTHead.forward :780-795: fold with stride hop, crop (n_fft-hop)/2 on
// both sides, divide by the folded window^2 envelope (clamped at 1e-11).
__global__ void ola_kernel(const float* FR, int seq, int nfft, float* wav, const int* lens, int T, int hop,
                           const float* win) {
    const int b = blockIdx.y;
    const long s = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long total = (long)T * hop;
    if (s >= total) return;
    const int len = lens ? min(lens[b], T) : T;
    float* out = wav + (long)b * total;
    if (s >= (long)len * hop) {
        out[s] = 0.f;
        return;
    }
    const long sp = s + (nfft - hop) / 2;
    const int fhi = (int)min((long)len - 1, sp / hop);
    const int flo = sp >= nfft ? (int)((sp - nfft) / hop + 1) : 0;
    float acc = 0.f, env = 0.f;
    for (int f = flo; f <= fhi; ++f) {
        const int n = (int)(sp - (long)f * hop);
        acc += FR[((long)b * seq + 3 + f) * nfft + n];
        env += win[n] * win[n];
    }
    out[s] = acc / fmaxf(env, 1e-11f);
}

}  // namespace xc2

using namespace xc2;

struct xc2_codec {
    xc2_config cfg;
    xc2_weights w;
    int P;   // rows per sequence incl. halo
    float *lat, *fx, *x, *hbuf, *hn, *qkv, *mid, *spec, *fr;
    size_t bytes;
};

static int alloc(xc2_codec* c, float** p, long floats) {
    size_t b = (size_t)floats * sizeof(float);
    if (hipMalloc((void**)p, b) != hipSuccess) return -4;
    if (hipMemset(*p, 0, b) != hipSuccess) return -2;
    c->bytes += b;
    return 0;
}

extern "C" {

int xc2_create(const xc2_config* cfg, const xc2_weights* w, xc2_codec** out) {
    if (!cfg || !w || !out) return -1;
    const xc2_config& k = *cfg;
    if (k.head_dim != 64 || k.hidden != k.n_heads * 64 || k.hidden % 128 || k.n_layers < 0 ||
        k.n_layers > XC2_MAX_LAYERS || k.n_groups <= 0 || k.hidden % (4 * k.n_groups) || k.quant_dim % 32 ||
        k.intermediate % 32 || k.n_levels < 1 || k.n_levels > 16 || k.level < 2 || k.hop <= 0 ||
        k.n_fft < k.hop || (k.n_fft - k.hop) % 2 || k.spec_ld < k.n_fft + 2 || k.spec_ld % 32 ||
        k.max_batch <= 0 || k.max_frames <= 0 || k.hidden > 1024 * 4)
        return -1;
    xc2_codec* c = new xc2_codec();
    memset(c, 0, sizeof(*c));
    c->cfg = k;
    c->w = *w;
    c->P = k.max_frames + 6;
    const long rows = (long)k.max_batch * c->P;
    int rc = 0;
    rc = rc ? rc : alloc(c, &c->lat, rows * k.quant_dim);
    rc = rc ? rc : alloc(c, &c->fx, rows * k.hidden);
    rc = rc ? rc : alloc(c, &c->x, rows * k.hidden);
    rc = rc ? rc : alloc(c, &c->hbuf, rows * k.hidden);
    rc = rc ? rc : alloc(c, &c->hn, rows * k.hidden);
    rc = rc ? rc : alloc(c, &c->qkv, rows * 3 * k.hidden);
    rc = rc ? rc : alloc(c, &c->mid, rows * k.intermediate);
    rc = rc ? rc : alloc(c, &c->spec, rows * k.spec_ld);
    rc = rc ? rc : alloc(c, &c->fr, rows * k.n_fft);
    if (rc) {
        xc2_destroy(c);
        return rc;
    }
    *out = c;
    return 0;
}

int xc2_destroy(xc2_codec* c) {
    if (!c) return 0;
    float* bufs[] = {c->lat, c->fx, c->x, c->hbuf, c->hn, c->qkv, c->mid, c->spec, c->fr};
    for (float* b : bufs)
        if (b) (void)hipFree(b);
    delete c;
    return 0;
}

int64_t xc2_workspace_bytes(const xc2_codec* c) { return c ? (int64_t)c->bytes : 0; }

static GemmArgs gargs(const float* A, int lda, RowMap am, const float* W, int K, int N, const float* bias, float* Cp,
                      int ldc, RowMap cm, int M) {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A = A;
    g.lda = lda;
    g.am = am;
    g.W = W;
    g.ldw = K;
    g.bias = bias;
    g.C = Cp;
    g.ldc = ldc;
    g.cm = cm;
    g.M = M;
    g.N = N;
    g.K = K;
    return g;
}

#define XC2_TRY(x)              \
    do {                        \
        int _rc = (x);          \
        if (_rc) return _rc;    \
    } while (0)
#define XC2_LAUNCHED() \
    do { if (hipGetLastError() != hipSuccess) return -2; } while (0)

static int resblock(xc2_codec* c, const xc2_resblock& rb, const int* lens, int B, int T, hipStream_t st) {
    const xc2_config& k = c->cfg;
    const int C = k.hidden, P = c->P, M = B * T;
    const RowMap R{T, P, 3}, Rc{T, P, 2};
    hipLaunchKernelGGL(groupnorm_silu_kernel, dim3(B * k.n_groups), dim3(256), 0, st, c->x, c->fx, P, C, k.n_groups,
                       rb.gn1_w, rb.gn1_b, lens, T, k.gn_eps);
    XC2_LAUNCHED();
    XC2_TRY(gemm(gargs(c->fx, C, Rc, rb.conv1_w, 3 * C, C, rb.conv1_b, c->hbuf, C, R, M), st));
    hipLaunchKernelGGL(groupnorm_silu_kernel, dim3(B * k.n_groups), dim3(256), 0, st, c->hbuf, c->fx, P, C,
                       k.n_groups, rb.gn2_w, rb.gn2_b, lens, T, k.gn_eps);
    XC2_LAUNCHED();
    GemmArgs g = gargs(c->fx, C, Rc, rb.conv2_w, 3 * C, C, rb.conv2_b, c->x, C, R, M);
    g.resid = c->x;
    return gemm(g, st);
}

int xc2_decode(xc2_codec* c, const int32_t* codes, const int32_t* lens, int32_t B, int32_t T, float* wav,
               void* stream) {
    if (!c || !codes || !wav) return -1;
    const xc2_config& k = c->cfg;
    if (B <= 0 || T <= 0) return -1;
    if (B > k.max_batch || T > k.max_frames) return -5;
    hipStream_t st = (hipStream_t)stream;
    const xc2_weights& w = c->w;
    const int C = k.hidden, P = c->P, M = B * T;
    const RowMap R{T, P, 3}, R3{T + 3, P, 3};
    // FSQ digits -> project_out (rows [0, T + 3) so the fc GEMM can zero the conv tail)
    hipLaunchKernelGGL(fsq_project_kernel, dim3(M), dim3(256), 0, st, codes, T, R, c->lat, k.quant_dim,
                       w.project_out_w, w.project_out_b, k.quant_dim, k.n_levels, k.level);
    XC2_LAUNCHED();
    {   // fc over T + 3 rows per sequence; rows t >= len written as 0
        GemmArgs g = gargs(c->lat, k.quant_dim, R3, w.fc_w, k.quant_dim, C, w.fc_b, c->fx, C, R3, B * (T + 3));
        g.lens = lens;
        g.mask_T = T;
        XC2_TRY(gemm(g, st));
    }
    // Conv1d k7, padding 3: A row t starts at halo row t - 3
    XC2_TRY(gemm(gargs(c->fx, C, RowMap{T, P, 0}, w.embed_w, 7 * C, C, w.embed_b, c->x, C, R, M), st));
    for (int i = 0; i < 2; ++i) XC2_TRY(resblock(c, w.prior[i], lens, B, T, st));
    for (int l = 0; l < k.n_layers; ++l) {
        const xc2_layer& L = w.layers[l];
        hipLaunchKernelGGL(rownorm_kernel, dim3(M), dim3(C / 4), 0, st, c->x, c->hn, R, C, L.attn_norm,
                           (const float*)nullptr, k.rms_eps, 0);
        XC2_LAUNCHED();
        XC2_TRY(gemm(gargs(c->hn, C, R, L.qkv, C, 3 * C, nullptr, c->qkv, 3 * C, R, M), st));
        hipLaunchKernelGGL(rope_heads_kernel, dim3(M), dim3(256), 0, st, c->qkv, R, 3 * C, C, k.n_heads, w.rope_cos,
                           w.rope_sin);
        XC2_LAUNCHED();
        hipLaunchKernelGGL(attn_f32_kernel, dim3((T + AQ - 1) / AQ, k.n_heads, B), dim3(256), 0, st, c->qkv, P, 3 * C,
                           C, c->hbuf, lens, T, k.attn_scale);
        XC2_LAUNCHED();
        {
            GemmArgs g = gargs(c->hbuf, C, R, L.o, C, C, nullptr, c->x, C, R, M);
            g.resid = c->x;
            XC2_TRY(gemm(g, st));
        }
        hipLaunchKernelGGL(rownorm_kernel, dim3(M), dim3(C / 4), 0, st, c->x, c->hn, R, C, L.mlp_norm,
                           (const float*)nullptr, k.rms_eps, 0);
        XC2_LAUNCHED();
        {
            GemmArgs g = gargs(c->hn, C, R, L.fc1, C, k.intermediate, nullptr, c->mid, k.intermediate, R, M);
            g.epi = EPI_SILU;
            XC2_TRY(gemm(g, st));
        }
        {
            GemmArgs g = gargs(c->mid, k.intermediate, R, L.fc2, k.intermediate, C, nullptr, c->x, C, R, M);
            g.resid = c->x;
            XC2_TRY(gemm(g, st));
        }
    }
    for (int i = 0; i < 2; ++i) XC2_TRY(resblock(c, w.post[i], lens, B, T, st));
    hipLaunchKernelGGL(rownorm_kernel, dim3(M), dim3(C / 4), 0, st, c->x, c->hn, R, C, w.ln_w, w.ln_b, k.ln_eps, 1);
    XC2_LAUNCHED();
    {
        XC2_TRY(gemm(gargs(c->hn, C, R, w.head_w, C, k.n_fft + 2, w.head_b, c->spec, k.spec_ld, R, M), st));
        const int nbins = k.n_fft / 2 + 1;
        hipLaunchKernelGGL(polar_kernel, dim3(M, (nbins + 127) / 128), dim3(128), 0, st, c->spec, R, k.spec_ld, nbins);
        XC2_LAUNCHED();
    }
    XC2_TRY(gemm(gargs(c->spec, k.spec_ld, R, w.dft, k.spec_ld, k.n_fft, nullptr, c->fr, k.n_fft, R, M), st));
    const long total = (long)T * k.hop;
    hipLaunchKernelGGL(ola_kernel, dim3((unsigned)((total + 255) / 256), B), dim3(256), 0, st, c->fr, P, k.n_fft, wav,
                       lens, T, k.hop, w.window);
    XC2_LAUNCHED();
    return 0;
}

int xc2_gemm(const float* X, int32_t ldx, int32_t M, const float* W, int32_t N, int32_t K, const float* bias,
             float* Y, int32_t ldy, int32_t epi, void* stream) {
    if (!X || !W || !Y || M <= 0 || N <= 0 || K <= 0 || epi < 0 || epi > 1) return -1;
    GemmArgs g = gargs(X, ldx, RowMap{M, 0, 0}, W, K, N, bias, Y, ldy, RowMap{M, 0, 0}, M);
    g.epi = epi;
    return gemm(g, (hipStream_t)stream);
}

int xc2_time_decode(xc2_codec* c, const int32_t* codes, int32_t B, int32_t T, float* wav, int32_t iters,
                    void* stream, float* avg_us) {
    if (!c || !avg_us || iters <= 0) return -1;
    hipStream_t st = (hipStream_t)stream;
    XC2_TRY(xc2_decode(c, codes, nullptr, B, T, wav, st));
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -2;
    (void)hipEventRecord(e0, st);
    int rc = 0;
    for (int i = 0; i < iters && !rc; ++i) rc = xc2_decode(c, codes, nullptr, B, T, wav, st);
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *avg_us = ms * 1000.f / (float)iters;
    return rc;
}

// gemm_f32_kernel alone over whole decodes (the codec roofline, bench.py --e2e): each GEMM
// launch of `iters` decodes between its own pair of events. *gemm_us = summed GEMM device
// time per decode, *flops = 2 M N K summed over one decode's GEMMs, *launches per decode.
int xc2_time_gemms(xc2_codec* c, const int32_t* codes, int32_t B, int32_t T, float* wav, int32_t iters,
                   void* stream, float* gemm_us, double* flops, int32_t* launches) {
    if (!c || !gemm_us || !flops || !launches || iters <= 0 || iters > 64) return -1;
    hipStream_t st = (hipStream_t)stream;
    XC2_TRY(xc2_decode(c, codes, nullptr, B, T, wav, st));   // warm
    const int cap = 256 * iters;
    std::vector<hipEvent_t> ev(2 * cap);
    for (auto& e : ev)
        if (hipEventCreate(&e) != hipSuccess) return -2;
    GemmTimer t{ev.data(), cap, 0, 0.0};
    g_gemm_timer = &t;
    int rc = 0;
    for (int i = 0; i < iters && !rc; ++i) rc = xc2_decode(c, codes, nullptr, B, T, wav, st);
    g_gemm_timer = nullptr;
    (void)hipStreamSynchronize(st);
    double us = 0.0;
    for (int i = 0; i < t.n; ++i) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
        us += ms * 1000.0;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    if (rc) return rc;
    *gemm_us = (float)(us / iters);
    *flops = t.flops / iters;
    *launches = t.n / iters;
    return 0;
}

}  // extern "C"

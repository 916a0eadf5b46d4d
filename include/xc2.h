/* XCodec2 codec DECODER (codes -> waveform) on MI355X (gfx950): C ABI.
 *
 * Replaces the reference's `AudioTokenizer.decode(frames)` (data/tokenizer.py:117-123),
 * which calls the pip `xcodec2==0.1.7` package's `XCodec2Model.decode_code` (absent
 * from the reference tree; architecture restated from the in-container transformers
 * port, [tf] models/xcodec2/modeling_xcodec2.py:799-862 Quantizer/Decoder, :746-796
 * ISTFT head, :639-661 ResNet block, :333-373 transformer layer). Called by
 * inference_tts_utils.py:359 and :363 after generate().
 *
 * Arithmetic is fp32 end to end (the reference runs the codec in fp32): every dense
 * contraction (Linear, Conv1d as an implicit GEMM over halo-padded rows, attention,
 * the irfft as a windowed DFT GEMM) runs on the exact-f32 MFMA
 * v_mfma_f32_32x32x2_f32.
 *
 * Conventions (same as t5gtts.h): status codes 0 ok, -1 invalid argument, -2 HIP
 * error, -4 out of memory, -5 capacity exceeded. All pointers named *_dev are device
 * pointers; the codec object keeps (does not copy) the weight pointers, which must
 * stay alive until xc2_destroy. Stream-ordered; one host thread per codec object.
 */
#ifndef XC2_H
#define XC2_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define XC2_MAX_LAYERS 32

typedef struct xc2_config {
    int32_t hidden;         /* 1024 */
    int32_t intermediate;   /* 4096 (SiLU MLP) */
    int32_t n_layers;       /* 12 */
    int32_t n_heads;        /* 16 */
    int32_t head_dim;       /* 64 (only 64 is supported) */
    int32_t n_groups;       /* 32 (GroupNorm) */
    int32_t quant_dim;      /* 2048 (project_out width = fc input width) */
    int32_t n_levels;       /* 8 FSQ dimensions */
    int32_t level;          /* 4 levels per dimension (codebook 4^8 = 65536) */
    int32_t hop;            /* 320 (16 kHz) / 882 (Anime-XCodec2 44.1 kHz) */
    int32_t n_fft;          /* 4 * hop */
    int32_t spec_ld;        /* padded spectrum row length: round_up(n_fft + 2, 32) */
    float attn_scale;       /* head_dim ** -0.5 */
    float rms_eps;          /* 1e-6 */
    float gn_eps;           /* 1e-6 */
    float ln_eps;           /* 1e-6 */
    int32_t max_batch;
    int32_t max_frames;
} xc2_config;

typedef struct xc2_resblock {     /* [tf] Xcodec2ResNetBlock :639-661 */
    const float *gn1_w, *gn1_b;   /* [hidden] */
    const float *conv1_w;         /* [hidden][3*hidden], tap-major: w[co][k*hidden + ci] */
    const float *conv1_b;
    const float *gn2_w, *gn2_b;
    const float *conv2_w, *conv2_b;
} xc2_resblock;

typedef struct xc2_layer {        /* [tf] Xcodec2DecoderLayer :333-373 */
    const float* attn_norm;       /* RMSNorm weight [hidden] */
    const float* qkv;             /* [3*hidden][hidden] = cat(q_proj, k_proj, v_proj) */
    const float* o;               /* [hidden][hidden] */
    const float* mlp_norm;        /* [hidden] */
    const float* fc1;             /* [intermediate][hidden] */
    const float* fc2;             /* [hidden][intermediate] */
} xc2_layer;

typedef struct xc2_weights {
    const float *project_out_w, *project_out_b;   /* [quant_dim][n_levels], [quant_dim] */
    const float *fc_w, *fc_b;                     /* [hidden][quant_dim], [hidden] */
    const float *embed_w, *embed_b;               /* Conv1d k7: [hidden][7*hidden] tap-major */
    xc2_resblock prior[2];
    xc2_layer layers[XC2_MAX_LAYERS];
    xc2_resblock post[2];
    const float *ln_w, *ln_b;                     /* final LayerNorm */
    const float *head_w, *head_b;                 /* [n_fft+2][hidden]: rows interleaved (mag_k, phase_k) */
    const float* dft;                             /* [n_fft][spec_ld] windowed irfft basis (zero pad cols) */
    const float* window;                          /* [n_fft] hann (periodic) */
    const float *rope_cos, *rope_sin;             /* [n_heads][head_dim/2]: RoPE over the HEAD axis */
} xc2_weights;

typedef struct xc2_codec xc2_codec;

int xc2_create(const xc2_config* cfg, const xc2_weights* w, xc2_codec** out);
int xc2_destroy(xc2_codec* c);
int64_t xc2_workspace_bytes(const xc2_codec* c);

/* codes_dev: int32 [B][T] codec token ids (row b valid for t < lens[b]); lens_dev:
 * int32 [B] or NULL (= all T). Ids are reduced mod level^n_levels (the FSQ digit
 * formula, as the pip package's indices_to_codes does; the HF port's codebook[idx]
 * would raise for the special ids 65536..65538). wav_dev: fp32 [B][T*hop]; samples
 * past lens[b]*hop are written as 0. */
int xc2_decode(xc2_codec* c, const int32_t* codes_dev, const int32_t* lens_dev, int32_t B, int32_t T,
               float* wav_dev, void* stream);

/* Diagnostics / measurement. xc2_gemm: Y[M][N] = X[M][K] . W[N][K]^T (+bias) on the f32
 * MFMA GEMM (rows dense, K % 32 == 0); epi 0 none, 1 SiLU. */
int xc2_gemm(const float* X_dev, int32_t ldx, int32_t M, const float* W_dev, int32_t N, int32_t K,
             const float* bias_dev, float* Y_dev, int32_t ldy, int32_t epi, void* stream);
int xc2_time_decode(xc2_codec* c, const int32_t* codes_dev, int32_t B, int32_t T, float* wav_dev,
                    int32_t iters, void* stream, float* avg_us);

#ifdef __cplusplus
}
#endif
#endif /* XC2_H */

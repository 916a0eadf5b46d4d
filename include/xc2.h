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
/* gemm_f32_kernel alone inside `iters` (<= 64) whole decodes of B x T frames, each GEMM launch
 * between its own event pair: *gemm_us = GEMM device time per decode, *flops = 2 M N K per
 * decode, *launches = GEMM launches per decode (the codec's roofline leg in bench.py --e2e). */
int xc2_time_gemms(xc2_codec* c, const int32_t* codes_dev, int32_t B, int32_t T, float* wav_dev,
                   int32_t iters, void* stream, float* gemm_us, double* flops, int32_t* launches);


/* ===================================================================================
 * XCodec2 codec ENCODER (16 kHz waveform -> codec ids) on MI355X (gfx950): C ABI.
 *
 * Replaces the reference's `AudioTokenizer.encode(wav)` (data/tokenizer.py:105-115;
 * called by tokenize_audio :125-143 from inference_tts_utils.py:182-188), which calls the
 * pip `xcodec2` package's `encode_code` (absent from the reference tree; architecture
 * restated from the in-container transformers port, [tf] models/xcodec2/modeling_xcodec2.py
 * :974-1024 Xcodec2Model.encode, :548-636 acoustic encoder, :663-745 FSQ, :865-909
 * semantic adapter; [tf] models/wav2vec2_bert/modeling_wav2vec2_bert.py :119-550 the
 * w2v-BERT 2.0 semantic encoder; [tf] models/seamless_m4t/feature_extraction_seamless_m4t.py
 * :112-138, :256-292 the Kaldi-style fbank front end the pip package feeds it).
 *
 *   wav (n samples, 16 kHz) -> zero-pad to n_pad = (n / 320 + 1) * 320
 *   semantic: fbank(80 mel, 25 ms / 10 ms, povey window, pre-emphasis 0.97, DC removal,
 *             512-point power spectrum, log) of the n_pad samples with 160 zeros either
 *             side, per-bin mean / unbiased-variance normalisation, 2-frame stacking
 *             -> LayerNorm + Linear(160 -> H) -> L conformer layers (half-step FFNs,
 *             relative-key MHA, GLU + causal depthwise conv module) -> 4-conv adapter
 *   acoustic: Conv1d(1 -> c0, k7) -> blocks of [3 dilated residual units (anti-aliased
 *             SnakeBeta) + anti-aliased SnakeBeta + strided Conv1d] -> SnakeBeta ->
 *             Conv1d(k3 -> hidden)
 *   concat(semantic, acoustic) -> Linear fc -> Linear project_in (-> n_levels) ->
 *   FSQ bound (twice, as the port does) -> round -> id = sum_j digit_j * level^j
 *
 * fp32 end to end (the reference runs the codec in fp32); dense contractions on the
 * exact-f32 MFMA GEMM of the decoder. One utterance per call (the reference encodes one
 * prompt at a time). Status codes as above.
 * =================================================================================== */
#define XC2E_MAX_LAYERS 32
#define XC2E_MAX_BLOCKS 8

typedef struct xc2e_config {
    int32_t sem_hidden;        /* 1024 */
    int32_t sem_heads;         /* 16 (head size 64 only) */
    int32_t sem_intermediate;  /* 4096 */
    int32_t sem_layers;        /* 16 */
    int32_t feat_dim;          /* 160 = 80 mel bins x 2 stacked frames */
    int32_t dw_kernel;         /* 31 (causal depthwise conv) */
    int32_t rel_left;          /* 64 left / 8 right relative-key distance clamp */
    int32_t rel_right;
    float sem_ln_eps;          /* 1e-5 */
    int32_t ac_channels0;      /* 48: first acoustic conv width */
    int32_t n_blocks;          /* 5 */
    int32_t strides[XC2E_MAX_BLOCKS];   /* 2, 2, 4, 4, 5 (product = hop 320) */
    int32_t hidden;            /* 1024: acoustic output width */
    int32_t n_levels;          /* 8 FSQ dimensions */
    int32_t level;             /* 4 levels per dimension */
    int32_t max_samples;       /* capacity: 16 kHz samples per call */
} xc2e_config;

typedef struct xc2e_conv {        /* Conv1d / Linear: weights tap-major [cout][kpad], */
    const float* w;               /* w[co][k * cin + ci], zero-padded to kpad (% 32 == 0) */
    const float* b;               /* [cout] or NULL */
    int32_t cin, cout, k, stride, dil, pad, kpad;
} xc2e_conv;

typedef struct xc2e_snake {       /* SnakeBeta log-parameters [C] (the kernel takes exp) */
    const float *alpha, *beta;
} xc2e_snake;

typedef struct xc2e_resunit {     /* [tf] Xcodec2ResidualUnit :548-581 */
    xc2e_snake s1;
    xc2e_conv c1;                 /* k7, dilation 1 / 3 / 9 */
    xc2e_snake s2;
    xc2e_conv c2;                 /* k1 */
} xc2e_resunit;

typedef struct xc2e_block {       /* [tf] Xcodec2EncoderBlock :584-604 */
    xc2e_resunit ru[3];
    xc2e_snake s;
    xc2e_conv down;               /* k = 2 * stride, pad = ceil(stride / 2) */
} xc2e_block;

typedef struct xc2e_layer {       /* [tf] Wav2Vec2BertEncoderLayer :398-461 */
    const float *ffn1_ln_w, *ffn1_ln_b, *ffn1_w1, *ffn1_b1, *ffn1_w2, *ffn1_b2;
    const float *attn_ln_w, *attn_ln_b;
    const float *qkv_w, *qkv_b;   /* [3H][H], [3H]: cat(linear_q, linear_k, linear_v) */
    const float *o_w, *o_b;
    const float* dist_emb;        /* [rel_left + rel_right + 1][64] */
    const float *conv_ln_w, *conv_ln_b;
    const float* pw1_w;           /* [2H][H] (no bias) */
    const float* dw_w;            /* [H][dw_kernel] */
    const float *dw_ln_w, *dw_ln_b;
    const float* pw2_w;           /* [H][H] (no bias) */
    const float *ffn2_ln_w, *ffn2_ln_b, *ffn2_w1, *ffn2_b1, *ffn2_w2, *ffn2_b2;
    const float *final_ln_w, *final_ln_b;
} xc2e_layer;

typedef struct xc2e_weights {
    const float* dft;             /* [544][512]: row 2k = cos, 2k+1 = -sin of bin k < 257, rest 0 */
    const float* mel;             /* [80][288]: Kaldi mel filters over the 257 power bins, 0-padded */
    const float* window;          /* [400] povey window */
    const float *fp_ln_w, *fp_ln_b, *fp_w, *fp_b;   /* feature projection LayerNorm(160) + Linear */
    xc2e_layer layers[XC2E_MAX_LAYERS];
    xc2e_conv adapter[4];         /* [tf] Xcodec2SemanticAdapter :865-909 (k3, pad 1) */
    xc2e_conv ac_in;              /* Conv1d(1 -> c0, k7, pad 3) */
    xc2e_block blocks[XC2E_MAX_BLOCKS];
    xc2e_snake ac_snake;
    xc2e_conv ac_out;             /* Conv1d(c0 * 2^n_blocks -> hidden, k3, pad 1) */
    const float *fc_w, *fc_b;     /* [sem_hidden + hidden] square */
    const float *pin_w, *pin_b;   /* project_in [n_levels][sem_hidden + hidden] */
    const float *aa_up, *aa_down; /* [12] Kaiser-sinc filters of the anti-aliased activations */
} xc2e_weights;

typedef struct xc2_encoder xc2_encoder;

int xc2e_create(const xc2e_config* cfg, const xc2e_weights* w, xc2_encoder** out);
int xc2e_destroy(xc2_encoder* e);
int64_t xc2e_workspace_bytes(const xc2_encoder* e);
/* codes the encoder emits for n samples: n / 320 + 1 (hop = product of strides) */
int32_t xc2e_num_codes(const xc2_encoder* e, int32_t n_samples);
/* wav_dev: fp32 [n_samples] at 16 kHz (device); codes_dev: int32 [xc2e_num_codes];
 * latent_dev (optional, NULL ok): fp32 [num_codes][n_levels] project_in outputs before
 * the FSQ bound. -5 if n_samples > max_samples. */
int xc2e_encode(xc2_encoder* e, const float* wav_dev, int32_t n_samples, int32_t* codes_dev, float* latent_dev,
                void* stream);
/* Diagnostics: the semantic model's input features alone (fbank front end), fp32
 * [num_codes][160] into feat_dev. */
int xc2e_features(xc2_encoder* e, const float* wav_dev, int32_t n_samples, float* feat_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* XC2_H */

/* Whisper speech recognizer: the auto-transcription that gives a voice-clone prompt its
 * text when the caller passes reference audio without reference text.
 *
 * Replaces:
 *   inference_commandline_hf.py:144-150
 *     wh_model = whisper.load_model("large-v3-turbo")
 *     prefix_transcript = wh_model.transcribe(reference_speech)["text"]
 * The model arithmetic runs here on gfx950 (fp32, f32 MFMA). The host side
 * (t5gemma-tts_amd/whisper_asr.py) keeps openai-whisper's transcribe/decode control flow
 * (language detection, logit filters, temperature fallback, seeking by timestamps).
 *
 * Data flow for one utterance (batch 1; the reference transcribes one file per call):
 *   whs_log_mel : 16 kHz samples + 30 s of zeros -> log-mel [frames][n_mels] (STFT 400/160,
 *                 periodic Hann, reflect pad, last frame dropped, log10, max - 8, (x + 4) / 4)
 *   whs_encode  : mel rows [seek, seek + seg) then zeros to 3000 frames -> conv stem ->
 *                 n_audio_layer pre-LN blocks -> ln_post; then every decoder layer's
 *                 cross-attention K / V from those features
 *   whs_decode  : n tokens at positions [offset, offset + n) through the text decoder with
 *                 its self-attention cache -> logits [n][n_vocab]
 * All pointers are device pointers, fp32 unless noted; calls are stream-ordered.
 * stream is a hipStream_t (null: the default stream).
 * Return codes: 0 ok, -1 bad argument, -2 HIP error, -4 out of device memory, -5 audio
 * longer than max_samples. */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WHS_MAX_LAYERS 64
#define WHS_SAMPLE_RATE 16000
#define WHS_HOP 160
#define WHS_N_FFT 400
#define WHS_N_FRAMES 3000   /* 30 s window */
#define WHS_FFT_K 416       /* n_fft padded to the GEMM's 32-wide K step */
#define WHS_BINS 201        /* n_fft / 2 + 1 */
#define WHS_BINS_PAD 224

/* openai-whisper ModelDimensions (whisper/model.py); n_audio_state == n_text_state and
 * both == 64 x heads are required. max_samples bounds the audio one call may pass. */
typedef struct whs_config {
    int32_t n_mels, n_audio_ctx, n_audio_state, n_audio_head, n_audio_layer;
    int32_t n_vocab, n_text_ctx, n_text_state, n_text_head, n_text_layer;
    int32_t max_samples;
} whs_config;

/* MultiHeadAttention: query / value / out have biases, key has none. [out][in] row-major. */
typedef struct whs_attn {
    const float *q_w, *q_b, *k_w, *v_w, *v_b, *o_w, *o_b;
} whs_attn;

/* ResidualAttentionBlock (cross_* only in the decoder); mlp = Linear(C, 4C), GELU, Linear. */
typedef struct whs_block {
    const float *attn_ln_w, *attn_ln_b;
    whs_attn attn;
    const float *cross_ln_w, *cross_ln_b;
    whs_attn cross;
    const float *mlp_ln_w, *mlp_ln_b;
    const float *fc1_w, *fc1_b, *fc2_w, *fc2_b;
} whs_block;

typedef struct whs_weights {
    const float* window;   /* [400] periodic Hann */
    const float* dft;      /* [2 * 201][416]: rows 2k / 2k+1 = cos / -sin of bin k, K zero padded */
    const float* mel;      /* [n_mels][224]: mel filters over the 201 bins, zero padded */
    const float *conv1_w, *conv1_b;   /* [C][k * n_mels + ci], K padded to a multiple of 32 */
    const float *conv2_w, *conv2_b;   /* [C][k * C + ci] */
    int32_t conv1_kpad, conv2_kpad;
    const float* enc_pos;             /* [n_audio_ctx][C] sinusoids */
    whs_block enc[WHS_MAX_LAYERS];
    const float *enc_ln_w, *enc_ln_b; /* ln_post */
    const float* tok_emb;             /* [n_vocab][C]; also the logit projection */
    const float* dec_pos;             /* [n_text_ctx][C] */
    whs_block dec[WHS_MAX_LAYERS];
    const float *dec_ln_w, *dec_ln_b;
} whs_weights;

typedef struct whs_model whs_model;

int whs_create(const whs_config* cfg, const whs_weights* w, whs_model** out);
int whs_destroy(whs_model* m);
int64_t whs_workspace_bytes(const whs_model* m);
/* frames of whs_log_mel for n samples: n / 160 + 3000 (the 30 s of padding included) */
int32_t whs_mel_frames(const whs_model* m, int32_t n_samples);
/* log-mel of wav[n] (+ 30 s of zeros) into the model's mel buffer; mel_out (optional)
 * receives a copy [frames][n_mels] */
int whs_log_mel(whs_model* m, const float* wav, int32_t n, float* mel_out, void* stream);
/* encode the 3000-frame window: mel rows [seek, seek + seg_frames) of the last
 * whs_log_mel, zero beyond; feat_out (optional) receives [n_audio_ctx][C] */
int whs_encode(whs_model* m, int32_t seek, int32_t seg_frames, float* feat_out, void* stream);
/* decode n tokens (device int32) at positions offset..offset+n-1 against the last
 * whs_encode; logits [n][n_vocab]. offset 0 starts a new sequence (cache reset). */
int whs_decode(whs_model* m, const int32_t* tokens, int32_t n, int32_t offset, float* logits, void* stream);

#ifdef __cplusplus
}
#endif

/*
 * t5gtts.h -- C ABI of the MI355X-native T5Gemma-TTS generate() engine (libt5gtts.so).
 *
 * This is the drop-in boundary for the reference's generate() hot path
 * (tori29umai0123/T5Gemma-TTS @ 2025-12-26). The reference is pure Python, so
 * there is no native FFI to mirror; each entry point replaces the Python/torch
 * call sequence named beside it. The Python host mirror
 * (t5gemma_tts_amd/engine.py: T5GemmaVoiceForConditionalGeneration.inference_tts,
 * same signature as hf_export/modeling_t5gemma_voice.py:565-580) drives it via
 * ctypes; INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions: plain pointers and sizes only (no torch types). "dev" pointers are
 * device (HBM) addresses owned by the caller unless stated; `stream` is a
 * hipStream_t passed as void*. All calls are stream-ordered and asynchronous
 * unless documented as synchronous. Return 0 on success, negative T5G_E* on error
 * (the Python shim maps them to ValueError / RuntimeError, like the reference's
 * asserts at :581-594). One host thread per engine; no global state.
 */
#ifndef T5GTTS_H
#define T5GTTS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define T5G_OK 0
#define T5G_EINVAL (-1)      /* bad shape / argument   -> ValueError  */
#define T5G_EHIP (-2)        /* HIP runtime failure    -> RuntimeError */
#define T5G_EUNSUPPORTED (-3)
#define T5G_ENOMEM (-4)
#define T5G_ECAPACITY (-5)   /* exceeds engine capacity (max_batch / max_text / max_audio) */
#define T5G_EHANDOFF (-6)    /* a fused decode launch's in-launch hand-off gave up waiting (not all of its
                              * workgroups were resident, e.g. another process shares the GPU): that
                              * call's outputs are invalid; the counters are cleared, rerun with
                              * t5g_engine_set_fused(e, 0) -> FusedHandoffError */

#define T5G_MAX_LAYERS 64

typedef struct t5g_engine t5g_engine;

/* Shapes + sampler constants. Mirrors T5GemmaVoiceConfig
 * (hf_export/configuration_t5gemma_voice.py:54-144) and the T5Gemma backbone
 * config ([tf] configuration_t5gemma.py). */
typedef struct {
    int32_t hidden, intermediate, n_enc_layers, n_dec_layers;
    int32_t n_heads, n_kv_heads, head_dim;
    int32_t text_vocab, n_audio_tokens;
    float attn_scale;      /* query_pre_attn_scalar ** -0.5 */
    float softcap;         /* 0: sdpa numerics (no softcap); >0: eager + tanh softcap */
    float rms_eps;
    float normalizer;      /* bf16(sqrt(hidden)) */
    int32_t sliding_window;
    uint8_t enc_sliding[T5G_MAX_LAYERS]; /* 1 = "sliding_attention" layer */
    uint8_t dec_sliding[T5G_MAX_LAYERS];
    int32_t max_batch;     /* utterance rows per call */
    int32_t max_text;      /* text tokens per row (encoder length capacity) */
    int32_t max_audio;     /* decoder cache length per row: BOS + prompt + generated (<= 12 288: a 100 s prompt + the 120 s duration cap) */
    int32_t max_gen;       /* generated-token capacity per row */
    /* sampler / stop constants (:590-592, :727, :773-777) */
    int32_t eos;           /* eog_inference */
    int32_t eos_guard;     /* encodec_sr // 5 */
    float budget_extra;    /* int(encodec_sr) * extra_cutoff */
    int32_t text_guard;    /* text_guard_frames_per_token */
    float progress_scale;
} t5g_config;

/* Device pointers to bf16 weights. "packed" = P16 layout built by t5g_pack_weight. */
typedef struct {
    const void* qkv;       /* packed [q_dim + 2 kv_dim][hidden]: q_proj | k_proj | v_proj rows */
    const void* o;         /* packed [hidden][q_dim] */
    const void* gate_up;   /* packed [2 inter][hidden]: 16-row groups of 8 gate + the same 8 up rows */
    const void* down;      /* packed [hidden][inter] */
    const void* cross_q;   /* decoder only: packed [q_dim][hidden] */
    const void* cross_kv;  /* decoder only: packed [2 kv_dim][hidden]: k_proj | v_proj */
    const void* cross_o;   /* decoder only: packed [hidden][q_dim] */
    const void* norms[6];  /* bf16 [hidden]: pre_self, post_self, pre_cross, post_cross, pre_ff, post_ff */
} t5g_layer_weights;

typedef struct {
    const void* enc_embed;       /* bf16 [text_vocab][hidden] row-major */
    const void* audio_embed;     /* bf16 [n_audio_tokens][hidden] row-major */
    const void* enc_final_norm;  /* bf16 [hidden] */
    const void* dec_final_norm;
    const void* head1;           /* packed [hidden][hidden]     predict_layer.0.0 */
    const void* head1_bias;      /* bf16 [hidden] */
    const void* head2;           /* packed [n_audio_tokens][hidden] predict_layer.0.2 */
    const void* head2_bias;      /* bf16 [n_audio_tokens] */
    const float* inv_freq;       /* fp32 [head_dim/2] RoPE inverse frequencies */
    const t5g_layer_weights* enc_layers;  /* host array [n_enc_layers] */
    const t5g_layer_weights* dec_layers;  /* host array [n_dec_layers] */
} t5g_weights;

/* Per-utterance sampler parameters (topk_sampling args, :744-750). */
typedef struct {
    int32_t top_k;           /* <= 0 disabled */
    int32_t top_k_list_len;  /* > 0: per-step list (top_k given as a list, :722-723) */
    int32_t top_k_list_off;
    float top_p, min_p, temperature;
    int32_t stop_repetition;
    int32_t n_silence;
    int32_t silence_off;
    int32_t eos_disabled;    /* throughput mode: EOS logit -> -inf (never accepted before the budget) */
    uint32_t seed_lo, seed_hi;  /* production noise (Philox4x32-10) */
} t5g_sampler_row;

/* Per-utterance AR state (the locals of inference_tts, :696-700, :717). */
typedef struct {
    int32_t cur_num_gen;
    int32_t current_length;
    int32_t prompt_offset;
    int32_t target_total;    /* < 0: none */
    int32_t est_total;
    int32_t prev_token;
    int32_t consec_silence;
    int32_t first_input_len;
    int32_t done;
    int32_t ambiguous_steps;
    int32_t last_token;
    float next_pos;
} t5g_sampler_state;

/* --- weights ------------------------------------------------------------- */
/* Bytes of the P16-packed image of an [N][K] bf16 matrix (K % 32 == 0). */
int64_t t5g_packed_bytes(int32_t N, int32_t K);
/* Pack src_dev [N][K] (row stride ld elements) into dst_dev (t5g_packed_bytes(N,K) bytes). */
int t5g_pack_weight(const void* src_dev, int32_t N, int32_t K, int64_t ld, void* dst_dev, void* stream);

/* --- engine lifetime --------------------------------------------------------- */
/* Replaces T5GemmaVoiceForConditionalGeneration.__init__ (:343-479) for the
 * inference path: binds caller-owned device weights, allocates the KV arena and
 * scratch in HBM (sized by cfg->max_*). */
int t5g_engine_create(const t5g_config* cfg, const t5g_weights* w, t5g_engine** out);
int t5g_engine_destroy(t5g_engine* e);
int64_t t5g_engine_workspace_bytes(const t5g_engine* e);

/* --- generate() phases --------------------------------------------------------
 * Token batches are PACKED: ntok tokens of B rows, with per-token row index
 * tok_row[ntok] and in-row position tok_t[ntok] (device int32). */

/* Encoder (:596-615 -> [tf] T5GemmaEncoder.forward :648-702) over text ids with
 * float PM positions pos[ntok] (:516-531), then every decoder layer's
 * PM-RoPE'd cross-attention K/V (:198-230) into the engine's cross cache.
 * text_len_dev[B] = x_lens. */
int t5g_encode(t5g_engine* e, int32_t B, int32_t ntok, const int32_t* ids_dev, const int32_t* tok_row_dev,
               const int32_t* tok_t_dev, const float* pos_dev, const int32_t* text_len_dev, void* stream);

/* Decoder prefill (:630-694): audio ids (BOS + prompt) with float PM positions
 * (:669-681); fills the self KV cache; writes the logits of each row's last token
 * (last_index_dev[B] = packed index) into the engine logits buffer.
 * kv_len_dev[B] = BOS + prompt length per row. */
int t5g_prefill(t5g_engine* e, int32_t B, int32_t ntok, const int32_t* ids_dev, const int32_t* tok_row_dev,
                const int32_t* tok_t_dev, const float* pos_dev, const int32_t* kv_len_dev,
                const int32_t* last_index_dev, void* stream);

/* Sampler setup (host arrays, copied): rows[B], init state[B], shared top-k list
 * and silence-token buffers. noise_dev: NULL for on-device Philox noise, else
 * bf16 [B][noise_steps][n_audio_tokens] -- the exact exponential draws of
 * torch.multinomial (parity mode). */
int t5g_sampler_setup(t5g_engine* e, int32_t B, const t5g_sampler_row* rows, const t5g_sampler_state* init,
                      const int32_t* top_k_list, int32_t n_top_k_list, const int32_t* silence, int32_t n_silence,
                      const void* noise_dev, int32_t noise_steps, void* stream);

/* n_steps iterations of the AR loop (:788-848): sample the current logits
 * (on-device stop rules), then run the single-token decoder step + predict head
 * for every row that is not done. use_graph != 0 replays a captured hipGraph of
 * one iteration. Asynchronous. */
int t5g_decode(t5g_engine* e, int32_t n_steps, int32_t use_graph, void* stream);

/* Synchronous readback: state[B] and tokens [B][max_gen] (host buffers). */
int t5g_read_state(t5g_engine* e, t5g_sampler_state* state_out, int32_t B, void* stream);
int t5g_read_tokens(t5g_engine* e, int32_t* tokens_out, int32_t B, void* stream);
/* Host write of one row's state (parity-mode correction of an ambiguous step). */
int t5g_write_state(t5g_engine* e, const t5g_sampler_state* state, int32_t row, int32_t token_slot,
                    int32_t token, void* stream);

/* Parity-mode pieces of one AR iteration: sample only (flags readable), then
 * the decoder step + head only (replayed from a graph captured on first use per
 * batch size). t5g_read_flags: bit0 = ambiguous top-p tie cut, bit1 = argmax was
 * EOS (synchronous); t5g_read_step: the row states and the flags in one sync. */
int t5g_step_only(t5g_engine* e, void* stream);
int t5g_read_flags(t5g_engine* e, int32_t* flags_out, int32_t B, void* stream);
int t5g_read_step(t5g_engine* e, t5g_sampler_state* state_out, int32_t* flags_out, int32_t B, void* stream);
/* Host re-run of one sampler step with torch.sort's exact std::sort tie order
 * (resolves ambiguous steps; see csrc/host_sampler.cpp). Pure host function.
 * max_gen / max_len: the engine's generated-token and self-attention cache capacity
 * (EOS is forced at the last generated slot or when the cache has no room left). */
int t5g_host_sample(const uint16_t* logits_bf16, int32_t V, const t5g_sampler_row* row,
                    const int32_t* top_k_list, const int32_t* silence, const t5g_sampler_state* state_in,
                    const uint16_t* noise_bf16, int32_t eos, int32_t eos_guard, float budget_extra,
                    int32_t text_guard, float progress_scale, int32_t max_gen, int32_t max_len,
                    t5g_sampler_state* state_out, int32_t* token_out);

/* Device pointer of the logits buffer bf16 [max_batch][logits_ld] (debug / parity). */
void* t5g_logits_ptr(t5g_engine* e, int32_t* logits_ld);
/* Stream-ordered device copy of the first B logits rows into dst_dev [B][logits_ld]. */
/* Parity mode: the RoPE cos / sin exception table (data/rope_trig_exc.bin: n sorted
 * (fp32 angle bits, cos_bf16 | sin_bf16 << 16) pairs, host memory; copied). Angles in it
 * take the reference host's MKL values, all others the correctly rounded ones. */
int t5g_engine_set_rope_exc(t5g_engine* e, const uint32_t* tab, int32_t n);
/* Diagnostics: device pointer of decoder layer `layer`'s cache (which: 0 self K, 1 self V,
 * 2 cross K, 3 cross V), bf16 [max_batch][n_kv_heads][cap][head_dim]; strides in elements. */
void* t5g_engine_cache_ptr(t5g_engine* e, int32_t layer, int32_t which, int64_t* head_stride,
                           int64_t* row_stride);
int t5g_copy_logits(t5g_engine* e, void* dst_dev, int32_t B, void* stream);

/* --- single-op entry points (parity tests, kernel benchmarks) ------------------ */
/* One sampler step on caller logits (bf16 [B][ld]) using the engine's sampler state. */
int t5g_sample_only(t5g_engine* e, int32_t B, const void* logits_dev, int32_t ld, void* stream);
/* Y = X . W^T on a packed W; epi: 0 bf16, 1 +bias bf16, 2 +bias GELU(erf) bf16, 3 GeGLU(tanh), 4 fp32 slabs;
 * epi | T5G_GEMM_PREFILL selects the many-token (encoder / prefill) kernel the engine uses for those phases */
#define T5G_GEMM_PREFILL 0x100
/* with T5G_GEMM_PREFILL: the register-ring many-token kernel instead of the LDS-staged one
 * (A/B probes only; the two are bitwise equal) */
#define T5G_GEMM_PREFILL_REG 0x200
int t5g_gemm(const void* X_dev, int32_t ldx, int32_t M, const void* Wp_dev, int32_t N, int32_t K, int32_t splits,
             const void* bias_dev, void* Y_dev, int32_t ldy, int32_t epi, void* stream);
/* Time `iters` launches of one GEMM shape with hipEvents on `stream`; launch i uses packed
 * weights Wp_list[i % n_w] (rotate over more bytes than the 256 MiB Infinity Cache to time
 * HBM-cold streaming as in a real decode step); average microseconds per launch in *avg_us. */
int t5g_time_gemm(const void* X_dev, int32_t ldx, int32_t M, const void* const* Wp_list, int32_t n_w, int32_t N,
                  int32_t K, int32_t splits, void* Y_dev, int32_t ldy, int32_t epi, int32_t iters, void* stream,
                  float* avg_us);
int t5g_time_decode_step(t5g_engine* e, int32_t iters, void* stream, float* avg_us);

/* Decode-step GEMV (csrc/gemv.hip): Y = X . W^T on a packed W with epilogue epi (as
 * t5g_gemm: 0 bf16, 1 +bias bf16, 3 GeGLU(tanh), 4 fp32 split-K slabs), at most one
 * workgroup per CU per k-slice -- the kernels the decode step runs its gate/up and down
 * projections ([tf] T5GemmaMLP :81-97), attention output projections ([tf] :264-304,
 * PMCrossAttention :167-253) and 65 541-row head (predict_layer :469-478) on. Fields
 * marked "reserved" must be 0 / NULL (the fused-prologue variants measured slower in
 * round 1 were removed). */
typedef struct {
    int32_t M, K, N;
    int32_t epi, pro, nw;     /* pro: reserved (0); nw: waves per block -- layout 0: 4 / 8 / 16
                                 (GeGLU 4 / 8); layout 1: 4 / 6 / 8 / 9 / 12 (others: 8) */
    const void* W;            /* packed [N][K] */
    const void* bias;         /* bf16 [N] (epi 1) */
    void* Y;                  /* bf16 or fp32 [M][ldy] */
    int32_t ldy, ldx;
    const void* X;            /* bf16 [M][ldx] */
    const void* v;            /* reserved */
    const void* h_in;         /* reserved */
    const int32_t* ids;       /* reserved */
    const void* table;        /* reserved */
    float scale, eps;         /* reserved */
    const void* post_w;       /* reserved */
    const void* pre_w;        /* reserved */
    void* h_out;              /* reserved */
    void* x_out;              /* reserved */
    int32_t un;               /* tuning: fragments in flight per wave (8 / 16), 0 = default; layout 1:
                                 -1 = every unit's weights requested before the first MFMA */
    int32_t max_grid;         /* tuning: blocks per launch cap, 0 = one per CU */
    int32_t splits;           /* split-K (epi 4): fp32 slabs [splits][M][ldy]; 0/1 = none */
    int32_t layout;           /* 0: the LDS-staged-X GEMV (M <= 16); 1: the register-resident-X
                                 GEMV (M <= 32; K / 32 k-steps per slice = 72 unsplit, or epi 4
                                 with 8 / 16 / 18 / 32 / 36 per slice, nw dividing it); W packed
                                 P16 either way; -1 for any other shape */
} t5g_gemv_args;
int t5g_gemv(const t5g_gemv_args* args, void* stream);
/* The decode step's residual + RMSNorm pair on caller buffers (norm.hip, [tf] T5GemmaRMSNorm
 * :61-78 wired as PMDecoderLayer :285-323): resid_out = bf16(resid + RMSNorm(1+post_w)(delta)),
 * normed_out = RMSNorm(1+pre_w)(resid_out); bf16 [M][d] rows. For parity tests. */
int t5g_resid_norm(int32_t M, int32_t d, const void* delta, const void* resid, const void* post_w,
                   const void* pre_w, float eps, void* resid_out, void* normed_out, void* stream);
/* hipEvent-timed `iters` launches rotating over packed weights Wp_list[i % n_w]
 * (see t5g_time_gemm); average microseconds per launch in *avg_us. */
int t5g_time_gemv(const t5g_gemv_args* args, const void* const* Wp_list, int32_t n_w, int32_t iters, void* stream,
                  float* avg_us);

/* Decode attention on caller buffers (single-query rows, sdpa numerics): the kernels the
 * engine's decode step runs for self / cross attention ([tf] T5GemmaSelfAttention
 * :264-304 with the KV cache of cache_utils.py:127-144; PMCrossAttention :167-253) --
 * keys split in chunks of <= 64 over workgroups, exp values rounded to bf16 before P.V
 * like torch's CPU SDPA, then one P.V + combine launch over 32-dimension slices of the
 * output for rows of > 64 keys. For parity tests. */
typedef struct {
    int32_t B, n_heads, n_kv_heads, head_dim;
    const void* q;            /* bf16 [B][n_heads * head_dim], PM-RoPE already applied */
    const void* k_cache;      /* bf16 [B][n_kv_heads][cap][head_dim] */
    const void* v_cache;
    int32_t cap;              /* key slots per (row, kv head) */
    const int32_t* kv_len;    /* device [B]: keys of each row (query = key kv_len - 1) */
    int32_t causal;           /* 1: self attention (keys <= query), 0: cross attention */
    int32_t window;           /* sliding window (0: none) */
    float scale;
    void* out;                /* bf16 [B][n_heads * head_dim] */
    void* work;               /* fp32 scores + chunk maxima, t5g_attention_decode_work_bytes() */
} t5g_attn_decode_args;
int64_t t5g_attention_decode_work_bytes(int32_t B, int32_t n_heads, int32_t n_kv_heads, int32_t head_dim,
                                        int32_t cap);
int t5g_attention_decode(const t5g_attn_decode_args* args, void* stream);
/* The fast path's form of the same attention (the engine's default decode self attention
 * in fast mode, t5g_engine_set_attn_flash): rows of > 64 keys finish in ONE launch -- each
 * 64-key chunk's workgroup computes an online-softmax partial (chunk max, sum of exp,
 * unnormalised bf16(p).V), the last to arrive for a (row, kv head) combines them. Not
 * aten's 512-key block order (fast-mode numerics); rows of <= 64 keys as
 * t5g_attention_decode. `work` as t5g_attention_decode_work_bytes(); its last
 * B * n_kv_heads words are arrival tickets that must be zero before the first call (each
 * call leaves them zero). */
int t5g_attention_decode_flash(const t5g_attn_decode_args* args, void* stream);
/* Decode self attention in fast mode: 1 (default) the one-launch flash form above, 0 the
 * two-launch aten-order form (scores, then P.V / combine). Reference: [tf]
 * T5GemmaSelfAttention :264-304; no reference-side equivalent switch. */
int t5g_engine_set_attn_flash(t5g_engine* e, int32_t enable);

/* Fast-path decode self attention inside the persistent layer launch (needs the flash form and
 * t5g_engine_set_fused). mode 0: its own flash launch between the layers; 1: stage S in front of
 * the launch's o-projection (the flash launch's arithmetic on the launch's workgroups, three
 * 64-key chunks each, att_self handed to the o-projection in-launch); 2 (default): stage S at
 * the END of the previous layer's launch -- after its q|k|v stage, with the K / V requested
 * before the N3 wait -- followed by that layer's o-projection, whose slabs the next launch's
 * norm reads (layer 0's attention and o-projection stay the step's own launches). Every mode
 * is bitwise equal to mode 0. A call whose rows x kv heads x chunks exceed 2 chunk slots per
 * worker takes mode 1 instead of 2; mode 1 runs up to 2 passes of 3 slots per workgroup (8
 * rows: rows of up to 3 072 keys); past that the separate launch.
 * Replaces the reference's per-layer self-attention call inside PMDecoderLayer
 * (hf_export/modeling_t5gemma_voice.py:256-323, [tf] modeling_t5gemma.py:264-304).
 * t5g_engine_attn_in_block_launches: layer launches issued with S (captured ones once).
 * t5g_engine_attn_in_block_mode: where the last decode step ran S (2, 1, or 0 = its own
 * launch). */
int t5g_engine_set_attn_in_block(t5g_engine* e, int32_t mode);
int t5g_engine_attn_in_block_launches(t5g_engine* e, int64_t* n);
int t5g_engine_attn_in_block_mode(t5g_engine* e, int32_t* mode);

/* Sampler launch shape: 0 (default) the 16-slice multi-block kernel, falling back per row to
 * the single-block kernel when a row's top-k / survivor set exceeds it; 1 the single-block
 * kernel only. Both pick the same tokens (tests/test_gpu_sampler.py). */
int t5g_engine_set_sampler_path(t5g_engine* e, int32_t single_block);
/* Decode step layout (fast path; parity mode runs the exact-order kernels): each decoder
 * layer after its self attention -- o-projection, norm, cross-q, PM cross attention,
 * cross-o, norm, gate/up GeGLU, down, norm, the next layer's q|k|v -- as ONE persistent
 * launch with in-launch hand-offs (fused.hip; 1-16 rows; 17-32 rows fuse the MLP half) or as
 * per-op launches; bitwise equal. Default on. Computes the reference's PMDecoderLayer
 * (hf_export/modeling_t5gemma_voice.py:256-323, [tf] modeling_t5gemma.py:81-97); no
 * reference-side equivalent switch. The switch also selects parity mode's persistent layer
 * (xlayer.hip: the same stages in the reference's CPU order, 1-8 decode rows of <= 64 text
 * keys each; bitwise equal to parity mode's per-op launches). */
int t5g_engine_set_fused(t5g_engine* e, int32_t enable);
/* Test / bench hook: parity-mode persistent layer launches issued so far (a launch captured
 * into a graph counts once, at capture). No reference-side equivalent. */
int t5g_engine_xlayer_launches(t5g_engine* e, int64_t* n);
/* Bench hook: average duration (us, HIP events on `stream`) of parity mode's persistent layer
 * launch at B decode rows, layers rotated as a step runs them, on the engine's current decode
 * state (call after a parity-mode generate). T5G_EUNSUPPORTED when the launch does not serve
 * B rows / this model. Like every t5g_time_* hook that runs engine launches, it leaves the
 * decode state invalid: t5g_decode returns T5G_EINVAL until the next t5g_sampler_setup.
 * No reference-side equivalent. */
int t5g_time_xlayer(t5g_engine* e, int32_t B, int32_t iters, void* stream, float* avg_us);
/* Host hint: the longest text (encoder length) of the batch the next t5g_encode / t5g_decode
 * calls run (0: assume max_text). The persistent decode launch reads at most 64 cross keys
 * per row, so it is chosen when the batch's texts fit, whatever the engine's max_text. */
int t5g_engine_set_text_max(t5g_engine* e, int32_t n);
/* Host hint: a bound on every row's self-attention keys in the next t5g_sampler_setup /
 * t5g_decode calls (0: max_audio) -- the largest prompt + time budget of the batch. The
 * decode attention grids cover that many keys, not the cache capacity, and the sampler
 * force-stops a row there (its capacity rule, :773-779 budget semantics unchanged when the
 * bound is at or above every row's prompt + budget). Replaces no reference interface: the
 * reference's DynamicCache grows per call ([tf] cache_utils.py:127-144). */
int t5g_engine_set_audio_max(t5g_engine* e, int32_t n);
/* Test hook: store `code` (non-zero) in the fused launch's sticky timeout word, as a
 * hand-off that gave up waiting would: every later in-launch wait gives up at once, the next
 * t5g_read_tokens returns T5G_EHANDOFF and clears the counters (tests/test_gpu_fused.py:
 * engine.generate then reruns the call on the per-op launches, same tokens). */
int t5g_engine_poison_handoff(t5g_engine* e, uint32_t code);
/* Average device time (us, hipEvents on `stream`) of the fused decode-MLP launch at B rows,
 * rotating over the decoder layers (bench.py roofline leg; no reference equivalent). */
int t5g_time_decode_mlp(t5g_engine* e, int32_t B, int32_t iters, void* stream, float* avg_us);
/* The same for the persistent layer launch WITH the self-attention stage S (the fast decode
 * step's launch; T5G_EUNSUPPORTED when the call would not take it), at the cache lengths the
 * last call left; *keys = keys one launch reads per kv head, summed over the rows and
 * averaged over the layers (bench.py prices the K / V stream with it). */
int t5g_time_decode_layer(t5g_engine* e, int32_t B, int32_t iters, void* stream, float* avg_us, float* keys);
/* Parity mode (after t5g_engine_set_exact(e, 1, ...) and one parity call): average device time
 * (us, hipEvents on `stream`) of one decoder layer's six exact decode Linear launches at B
 * rows (q|k|v, o, cross-q, cross-o, gate/up + GeGLU, down in the reference's K parts), layers
 * rotated (bench.py's parity roofline; no reference equivalent). */
int t5g_time_exact_linears(t5g_engine* e, int32_t B, int32_t iters, void* stream, float* avg_us);

/* --- parity mode (csrc/exact.hip) ------------------------------------------------
 * Switch an engine to the exact-order kernels: every Linear, RMSNorm mean, q.k / P.V of
 * attention and GELU computed in the accumulation order of the reference's own CPU run
 * (torch 2.10 CPU bf16: oneDNN AMX F.linear, aten SDPA + oneDNN gemv / gemm, aten AVX2
 * sum; measured on the machine the golden vectors come from), so that
 * logits -- and with the reference's noise stream, token ids -- are the reference's bit
 * for bit. Replaces the bf16 linears of modeling_t5gemma_voice.py:469-478 / [tf]
 * modeling_t5gemma.py:81-97, 264-304, PMCrossAttention :167-253 and the RMSNorm of [tf]
 * :61-78 inside t5g_encode / t5g_prefill / t5g_decode. gelu_lut: bf16 -> bf16 nn.GELU()
 * (erf) of the reference host, 65 536 entries indexed by the input bits (NULL: the
 * exact-erf form, equal except on 24 inputs in [-5.4, -3.1]); threads: the reference
 * host's torch thread count (8, the only measured K-split table; others -> EUNSUPPORTED).
 * enable = 0 returns to the fast kernels. Per-utterance token counts (text, prompt + 1)
 * must not exceed 5001 in parity mode (the measured table, csrc/ref_ksplit.h). Synchronous. */
int t5g_engine_set_exact(t5g_engine* e, int32_t enable, const uint16_t* gelu_lut, int32_t threads);
/* Single exact-order Linear on caller buffers (parity tests): Y = X . W^T on a packed W in
 * the reference's order (32-element E/O chunk chains, chunk sums folded; K split into
 * parts of kb32 * 32 elements, kb32 = 0: no split; bias last). epi as t5g_gemm
 * (0 bf16, 1 +bias bf16, 2 +bias GELU(erf) via gelu_lut, 3 GeGLU(tanh), 4 fp32 unrounded). */
int t5g_exact_linear(const void* X_dev, int32_t ldx, int32_t M, const void* Wp_dev, int32_t N, int32_t K,
                     int32_t kb32, const void* bias_dev, const void* gelu_lut_dev, void* Y_dev, int32_t ldy,
                     int32_t epi, void* stream);
/* The same exact-order Linear on the f32-input MFMA kernels the engine's parity mode runs
 * (csrc/xmm.hip: v_mfma_f32_16x16x4_f32 chains = the reference's E/O chunk chains); same
 * arguments and results as t5g_exact_linear, bit for bit. epi | 0x2000 (M <= 32, kb32 <
 * K / 32): the decode part mode -- Y receives each K part's fp32 fold, [parts][M][N]. */
int t5g_xmm_linear(const void* X_dev, int32_t ldx, int32_t M, const void* Wp_dev, int32_t N, int32_t K,
                   int32_t kb32, const void* bias_dev, const void* gelu_lut_dev, void* Y_dev, int32_t ldy,
                   int32_t epi, void* stream);
/* The parity Linears' operand layouts (csrc/xmm.hip): the E16 image of a P16-packed weight
 * (bytes = t5g_packed_bytes(N, K)), the X16 image of bf16 rows X [M][ldx] (K columns,
 * ceil(M / 16) * 16 * K elements). */
int t5g_pack_e16(const void* p16_dev, void* e16_dev, int64_t bytes, void* stream);
int t5g_to_x16(const void* X_dev, int32_t ldx, int32_t M, int32_t K, void* Y16_dev, void* stream);
/* hipEvent-timed f32-MFMA Linear launches on E16 weights W16_list[i % n_w] (rotated to
 * stream from HBM as in a decode step); epi as t5g_gemm, | 0x1000: Y is an X16 output.
 * Average microseconds per launch in *avg_us (kernel probes, bench roofline). */
int t5g_time_xmm(const void* X16_dev, int32_t M, const void* const* W16_list, int32_t n_w, int32_t N, int32_t K,
                 int32_t epi, const void* bias_dev, void* Y_dev, int32_t ldy, int32_t iters, void* stream,
                 float* avg_us);
/* Single exact-order SDPA call on caller buffers (parity tests): one reference call per row b
 * with q_len[b] queries (q rows packed, q_row / q_pos per query) over kv_len[b] keys of a
 * [B][n_kv_heads][cap][head_dim] cache, torch 2.10 CPU flash-attention numerics incl. its
 * GEMM selection (gemv / unpacked / packed, threads = the reference thread count).
 * q_pos = q_len = null: one query per row at its last key, on the decode launches the
 * engine runs (scores + P.V, csrc/xattn.hip). */
int t5g_exact_attention(const void* q_dev, int32_t Mq, const int32_t* q_row_dev, const int32_t* q_pos_dev,
                        const int32_t* q_len_dev, const void* k_cache_dev, const void* v_cache_dev, int32_t cap,
                        const int32_t* kv_len_dev, int32_t n_heads, int32_t n_kv_heads, int32_t head_dim,
                        int32_t causal, int32_t window, float scale, int32_t threads, void* out_dev, void* stream);
/* The same call for eager attention (attn_implementation="eager", the reference default;
 * [tf] eager_attention_forward modeling_t5gemma.py:199-230): bf16 q.k^T, x scale, tanh
 * softcap (tanh from tanh_lut_dev: the reference host's bf16 tanh, 65 536 entries),
 * masked fp32 softmax, bf16 P.V, in the reference host's orders (csrc/eager.hip; restated
 * for n_heads = 8, head_dim = 256 -- the reference model's call shape -- else
 * T5G_EUNSUPPORTED). Replaces the eager branch of the reference's attention interface. */
int t5g_eager_attention(const void* q_dev, int32_t Mq, const int32_t* q_row_dev, const int32_t* q_pos_dev,
                        const int32_t* q_len_dev, const void* k_cache_dev, const void* v_cache_dev, int32_t cap,
                        const int32_t* kv_len_dev, int32_t n_heads, int32_t n_kv_heads, int32_t head_dim,
                        int32_t causal, int32_t window, float scale, float softcap, const uint16_t* tanh_lut_dev,
                        void* out_dev, void* stream);
/* Parity mode for an eager-attention checkpoint: the reference host's bf16 tanh table
 * (data/tanh_bf16.bin), required before t5g_engine_set_exact on such a config. */
int t5g_engine_set_tanh_lut(t5g_engine* e, const uint16_t* lut_host);

/* --- parity-mode noise on the device (csrc/noise.hip) --------------------------------
 * The reference's torch.multinomial draws V exponential variates per step from torch's CPU
 * generator (MT19937; hf_export/modeling_t5gemma_voice.py:133-138, SURVEY a14' 6). Replaces
 * drawing them with torch on the host (engine.reference_noise):
 * t5g_mt_stream: one MT19937 stream per row from init_dev [B][625] (624 state words + the
 * outputs of that state already consumed, 1..624 -- torch's `left` = 625 - pos), outputs
 * [0, n_out) of row b to out_dev[b * out_stride ...] (uint32), and if snap_dev != NULL the
 * generator after every snap_every outputs (s < n_snap) to snap_dev [B][n_snap][625].
 * Step s of a row uses outputs [2 V s, 2 V (s + 1)): draw i = (out[2i] << 32 | out[2i+1]).
 * t5g_mt_exponential: q = bf16(float(-log1p(-u))) of n draws (raw pairs) into bf16 q_dev
 * (tests: equal to torch's exponential_). t5g_engine_set_noise_mt: the engine's parity
 * sampler reads its draws from raw_dev [max_batch][steps][2 V] (NULL: off). */
int t5g_mt_stream(const uint32_t* init_dev, int32_t B, int64_t n_out, int64_t out_stride, uint32_t* out_dev,
                  int64_t snap_every, int32_t n_snap, uint32_t* snap_dev, void* stream);
int t5g_mt_exponential(const uint32_t* raw_dev, int64_t n, void* q_dev, void* stream);
/* Test hook: y_dev[i] = std::exp(x_dev[i]) as the exact attention kernels evaluate it -- the
 * reference host's glibc 2.35 expf (aten's flash-attention rescale exp(m_old - m) and block
 * tails), restated in csrc/common.h sdpa_expf; fp32 device arrays of n values. */
int t5g_sdpa_expf(const float* x_dev, float* y_dev, int64_t n, void* stream);
int t5g_engine_set_noise_mt(t5g_engine* e, const uint32_t* raw_dev, int32_t steps);
/* Host build of the sampler's sparse emulation of torch.sort's tie order (csrc/sort_emu.h;
 * replaces the reference's torch.sort in top_k_top_p_filtering, :107-108, for the order of
 * the survivors only): S survivors at ascending slots pos[] with values val[] in an array of
 * n otherwise -inf entries; on return the three arrays are ordered by final slot (pos[] the
 * final slots). T5G_EUNSUPPORTED where the emulation does not follow std::sort (heapsort
 * fallback, NaN); pure host function. */
int t5g_sort_emu(int32_t n, int32_t S, int32_t* pos, float* val, int32_t* tag);
/* The same replay on one GPU wave (the sampler's path for <= 63 survivors), device arrays;
 * the fail code (0 = reproduced) is written to fail_dev[0]. Tests. */
int t5g_sort_emu_wave(int32_t n, int32_t S, int32_t* pos_dev, float* val_dev, int32_t* tag_dev,
                      int32_t* fail_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* T5GTTS_H */

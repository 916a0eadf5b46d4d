// Internal launcher interface of the gfx950 kernels (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace t5g {
typedef uint16_t bf16_t;

enum { EPI_BF16 = 0, EPI_BIAS_BF16 = 1, EPI_BIAS_GELU = 2, EPI_GEGLU = 3, EPI_F32 = 4 };

struct GemmArgs {
    const bf16_t* X;  // [M][ldx] activations
    int ldx;
    int M;
    const bf16_t* W;  // packed P16, NG row groups x KB fragments
    int N;            // real output rows of W (GEGLU: 2*F interleaved gate/up groups)
    int NG;           // padded row groups (multiple of 4)
    int KB;           // K / 32
    int splits;       // split-K over blockIdx.y (EPI_F32 only)
    const bf16_t* bias;
    void* Y;          // bf16 [M][ldy] or f32 [splits][M][ldy]
    int ldy;
    int dbg_seq;      // diagnostic timeline slot (T5G_DBG_TS builds only)
    int prefill;      // 1: many-token phase (encoder / prefill) -> register-tiled MFMA kernel
};
int pack_p16(const bf16_t* src, int N, int K, long ld, bf16_t* dst, int NGpad, hipStream_t st);
int gemm_p16(const GemmArgs& a, int epi, hipStream_t st);

// ---- decode-step GEMV (M <= 16 rows, gemv.hip) ----------------------------------
struct DecGemmArgs {
    int M, K;                 // rows (<= 16), reduction length (= X row width)
    const bf16_t* W;          // packed P16
    int N, NG, KB;
    const bf16_t* bias;
    void* Y;                  // bf16 or fp32 [M][ldy] (EPI_F32 split-K: [splits][M][ldy])
    int ldy;
    const bf16_t* X;          // [M][ldx], staged through LDS
    int ldx;
    int nw;                   // waves per block (4, 8 or 16)
    int un;                   // fragments in flight per wave (8 / 16), 0 = default
    int max_grid;             // blocks per launch cap, 0 = one per CU
    int splits;               // split-K over blockIdx.y (EPI_F32 only)
    int layout_rx;            // 1: register-resident-X kernel (1..32 rows, K = 2304)
};
int gemv_dec(const DecGemmArgs& a, int epi, hipStream_t st);
size_t gemv_dec_lds_bytes(const DecGemmArgs& a, int rg);

// decode MLP half in one persistent launch (fused.hip): norm of the cross-o slabs ->
// gate/up GeGLU -> down slabs, hand-offs in-launch
struct FusedMlpArgs {
    int M, d, f;              // rows (<= 32), hidden (2304), intermediate (9216)
    const float* part_in;     // cross-o fp32 slabs [4][M][d]
    const bf16_t* post_w;     // RMSNorm(1+w) of the cross-attention output
    const bf16_t* pre_w;      // RMSNorm(1+w) in front of the MLP
    float eps;
    bf16_t* h;                // residual [M][d], updated in place
    bf16_t* xn;               // normed rows [M][d] (handed off in-launch)
    const bf16_t* Wgu;        // packed P16 gate/up (interleaved), NGgu row groups, K = d
    int NGgu;
    bf16_t* act;              // [M][f] (handed off in-launch)
    const bf16_t* Wd;         // packed P16 down, NGd row groups, K = f
    int NGd;
    float* part_out;          // down fp32 slabs [8][M][d] (may alias part_in: written only after
                              // every norm workgroup has consumed part_in)
    unsigned* sync;           // this launch's FM_SET_WORDS counter words (zero when it starts)
    unsigned* sync_next;      // the next launch's set: zeroed by this launch (its last user is done)
    unsigned* timeout;        // sticky: a wait that gave up stores its code here
    int grid;                 // 0: one workgroup per CU
    int norm_b0;              // set by fused_mlp: first norm workgroup
    int dbg_seq;              // diagnostic timeline slot (T5G_DBG_TS builds only)
    // ---- cross-attention chain in front (xattn = 1: fused.hip fused_block_kernel):
    //   N1: h1 = h + RMSNorm_post1(o-proj slabs), xn1 = RMSNorm_pre1(h1)
    //   Q:  cross-q fp32 slabs [2][M][q_dim] = xn1 . Wq^T (2 k-slices of 36 k-steps)
    //   A:  att = PMCrossAttention(q slabs, cross K/V) per (row, q head)
    //   O:  cross-o fp32 slabs [4][M][d] = att . Wo^T; then part_in := those slabs
    int xattn;
    const float* o_slabs;     // self-attention o-projection slabs [4][M][d] (previous launch)
    const bf16_t* post1_w;    // post_self_attn_layernorm
    const bf16_t* pre1_w;     // pre_cross_attn_layernorm
    bf16_t* xn1;              // [M][d] handed off in-launch
    const bf16_t* Wq;         // packed cross q_proj, NGq row groups, K = d
    int NGq;
    float* qslab;             // [2][M][q_dim] handed off in-launch
    const bf16_t* ck;         // cross K / V cache of the layer [B][Hkv][kv_cap][D]
    const bf16_t* cv;
    int kv_cap;
    const int* enc_len;       // [B] text lengths (keys of each row)
    int text_max;             // the batch's longest text (the cross-attention stage reads <= 64 keys)
    const float* rope_tab;    // [B][D] this step's PM-RoPE cos | sin
    int q_dim, Hq, Hkv, D;
    float scale;
    float softcap;            // eager checkpoints: the tanh logit softcap (0: none)
    bf16_t* att;              // [M][q_dim] handed off in-launch
    const bf16_t* Wo;         // packed cross o_proj, NGo row groups, K = q_dim
    int NGo;
    float* oslab;             // [4][M][d] handed off in-launch (the N2 norm's input)
    // ---- the layer's last norm and the next layer's q|k|v projection at the end (xattn):
    //   D writes its slabs to dslab (in-launch), N3: h = h + RMSNorm_post3(down slabs),
    //   xn = RMSNorm_pre3(h) (the next layer's pre_self_attn or the final norm), then, unless
    //   Wqkv is null (last layer), QKV: fp32 slabs [2][M][qkv_dim] -> qkv_out (next launch)
    float* dslab;             // [8][M][d]
    const bf16_t* post3_w;    // post_feedforward_layernorm
    const bf16_t* pre3_w;     // next layer's pre_self_attn_layernorm, or the final norm
    const bf16_t* Wqkv;       // next layer's packed q|k|v (NGqkv row groups, K = d), or null
    int NGqkv, qkv_dim;
    float* qkv_out;           // [2][M][qkv_dim]
    // ---- the self-attention o-projection in front (Wo1 non-null): O1 = att_self . Wo1^T as
    //   fp32 slabs [4][M][d] in o1slab (in-launch), the N1 norm's input instead of o_slabs
    const bf16_t* att_self;   // [M][q_dim] self-attention output (previous launch, or stage S)
    const bf16_t* Wo1;        // packed self o_proj, NGo row groups, K = q_dim
    float* o1slab;
    // ---- the layer's decode self-attention in front of O1 (self_attn = 1, needs Wo1): stage
    //   S = attn.hip attn_decode_kernel<256, 2, true, true>'s arithmetic (q / new-key PM-RoPE
    //   from the q|k|v slabs, the key and value appended to the cache, flash-form 64-key chunk
    //   partials, the last chunk of a (row, kv head) combining), writing att_self in-launch
    int self_attn;
    const float* qkv_in;      // [2][M][qkv_dim] this layer's q|k|v slabs (previous launch)
    bf16_t* sk;               // self K / V cache of the layer [B][Hkv][s_cap][D]
    bf16_t* sv;
    int s_cap;                // cache capacity (keys)
    int s_nsplit;             // 64-key chunk records per (row, kv head) in fpart / fstat
    const int* kv_len;        // [B] keys of each row, the appended one included
    int window;               // sliding window (0: none)
    float* fpart;             // [M][Hkv][s_nsplit][G][D] chunk partials
    float* fstat;             // [M][Hkv][s_nsplit][G][2] chunk max / sum
    unsigned* fticket;        // [M][Hkv] arrival tickets (zero between launches)
    // ---- stage S at the END instead (self_tail = 1, needs Wqkv, no Wo1): the S fields above
    //   describe the NEXT layer, whose q|k|v this launch projects; then that layer's O1 into
    //   o1n ([4][M][d], the next launch's o_slabs: its N1 reads them, Wo1 null there)
    int self_tail;
    const bf16_t* Wo1n;       // the next layer's packed self o_proj
    float* o1n;
};
int fused_mlp(const FusedMlpArgs& a, hipStream_t st);
int fused_mlp_check(const FusedMlpArgs& a);   // 0: fused_mlp would launch these args; -1: not built for them
// counter words of one fused launch, each on its own 128-byte line (arrivals on one line
// serialise at ~12 ns each): N1, 8 cross-q heads, 8 attention heads, 8 cross-o groups,
// N2, 8 down slices, 8 down groups, N3, 8 o-projection groups, 8 self-attention kv heads, 8
// q|k|v groups (the tail's in-launch hand-off).
// The engine keeps one set per decoder layer after one line for the timeout word.
constexpr int FM_LINE = 32, FM_SET_LINES = 67, FM_SET_WORDS = FM_SET_LINES * FM_LINE;

// parity mode's decode layer after the self attention as one persistent launch (xlayer.hip):
// O1 self o-proj, N1, cross q, PM cross attention, cross o, N2, gate/up + GeGLU, down in the
// reference's two K parts, N3, the next layer's q|k|v -- the per-op launches' arithmetic,
// bitwise. Decode rows M <= 8, the 2b-2b shapes (hidden 2304, q_dim 2048, head_dim 256, 8 q
// heads over 4 kv heads, intermediate 9216), <= 64 text keys per row.
struct XLayerArgs {
    int M;
    // E16 weights of the layer (Wqkv: the next layer's; null on the last layer)
    const bf16_t *Wo, *Wq, *Wco, *Wgu, *Wd, *Wqkv;
    // RMSNorm(1 + w) weights: N1 post_self / pre_cross, N2 post_cross / pre_ff, N3 post_ff /
    // the next layer's pre_self (or the final norm)
    const bf16_t *n1_post, *n1_pre, *n2_post, *n2_pre, *n3_post, *n3_pre;
    float eps;
    const bf16_t* att16_self;   // X16 self-attention output (previous launch)
    bf16_t* h;                  // residual rows [M][hidden] (read at N1, written at N3)
    bf16_t* xn;                 // normed rows [M][hidden] (row-major copy)
    bf16_t* xn16;               // normed rows, X16 (handed off in-launch)
    bf16_t* tmp;                // o-projection outputs [M][hidden] (in-launch)
    bf16_t* q;                  // cross q [M][q_dim] un-rotated (in-launch)
    bf16_t* att;                // cross attention output [M][q_dim] (row-major copy)
    bf16_t* att16;              // cross attention output, X16 (in-launch)
    bf16_t* act16;              // GeGLU act, X16 (in-launch)
    float* dpart;               // down projection K parts [2][M][hidden] fp32 (in-launch)
    bf16_t* qkv;                // next layer's q|k|v [M][qkv_dim] (next launch)
    int qkv_dim;
    const bf16_t *ck, *cv;      // the layer's cross K / V cache [B][Hkv][kv_cap][D]
    long kv_bstride, kv_hstride;
    const int* enc_len;         // [B] text lengths
    const float* rope_tab;      // [B][D] this step's PM-RoPE cos | sin
    float scale;
    unsigned* sync;             // this launch's XL_SET_LINES counter lines (zero when it starts)
    unsigned* sync_next;        // the next launch's set: zeroed by this launch
    unsigned* timeout;          // sticky timeout word (fused.hip's)
};
constexpr int XL_SET_LINES = 56, XL_SET_WORDS = XL_SET_LINES * FM_LINE;
int xlayer_launch(const XLayerArgs& a, hipStream_t st);   // -1: not built for these args / this device

// ---- row-wise residual / RMSNorm / embedding -------------------------------
struct NormArgs {
    int M, d;
    const int* ids;          // optional: v = bf16(table[ids[m]] * scale)
    const bf16_t* table;
    int n_table;             // rows of table: ids are clamped into [0, n_table) (no OOB read)
    float scale;
    const bf16_t* delta;     // [M][d] bf16 (if ids == null and part == null)
    const float* part;       // fp32 partial slabs [nsplit][M][ldp]
    int nsplit, ldp;
    const bf16_t* post_w;    // RMSNorm(1+w) applied to v before the residual add
    const bf16_t* resid;     // [M][d] or null
    const bf16_t* pre_w;     // RMSNorm(1+w) producing normed_out
    float eps;
    bf16_t* resid_out;       // [M][d] or null
    bf16_t* normed_out;      // [M][d] or null
    const int* out_rows;     // optional: process only rows out_rows[i] (i < M), write compact
    int dbg_seq;             // diagnostic timeline slot (T5G_DBG_TS builds only)
    // optional: each row block also writes that row's RoPE cos/sin table
    const float* rope_pos;   // [M] positions
    const float* rope_inv_freq;
    float* rope_tab;         // [M][rope_D]
    int rope_D;
    int exact;               // parity mode: the reference's CPU sum order (delta / ids sources)
    const uint32_t* trig_exc;   // parity mode: the RoPE cos / sin exception table (exact_math.h rope_trig)
    int n_trig_exc;
    bf16_t* normed_x16;      // optional: normed_out again in the X16 layout (xmm.hip)
};
int resid_norm(const NormArgs& a, hipStream_t st);

// ---- RoPE + KV-cache store --------------------------------------------------
struct RopeArgs {
    const bf16_t* X;         // [M][ldx]: q heads | k heads | v heads
    const float* Xpart;      // alternatively fp32 split-K slabs [nsplit][M][ldx] (summed, rounded)
    int nsplit;
    int ldx, M, D;
    int nq, nk, nv;          // head counts present in X (column blocks of D, from column col0)
    int col0;
    int rope_q, rope_k;
    const float* pos;        // [M] float PM positions (or pos_dev_row when decode)
    const float* inv_freq;   // [D/2]
    const int* tok_row;      // [M] batch row of each token (null: row = m)
    const int* tok_t;        // [M] cache slot (null: slot = kv_len[row] - 1)
    const int* kv_len;
    bf16_t* Qout;            // [M][ldq] (may alias X)
    int ldq;
    bf16_t* Kc;              // cache [B][Hkv][Lmax][D]
    bf16_t* Vc;
    long c_bstride, c_hstride;
    const float* rope_tab;   // optional [rows][D]: bf16-rounded cos (D/2) | sin (D/2) per row
    int exact_trig;          // parity mode: cos / sin as the reference host rounds them (exact_math.h)
    const uint32_t* trig_exc;   // with the exception table of rope_trig
    int n_trig_exc;
};
int rope_store(const RopeArgs& a, hipStream_t st);
// (the decode step's per-row table tab[r][i] = bf16(cos(inv_freq[i] * pos[r])),
// tab[r][D/2 + i] = bf16(sin(...)) is written by layer 0's embedding-norm launch: NormArgs.rope_*)

// ---- attention ----------------------------------------------------------------
struct AttnArgs {
    const bf16_t* Q;         // [Mq][ldq] rope applied
    int ldq, Mq;
    const int* q_row;        // [Mq] batch row (null: row = query index)
    const int* q_pos;        // [Mq] query position t (null: t = kv_len[row] - 1)
    const bf16_t* K;         // cache [B][Hkv][Lmax][D]
    const bf16_t* V;
    long kv_bstride, kv_hstride;
    const int* kv_len;       // [B] valid keys per row
    int Hkv, D, G;           // kv heads, head dim, q heads per kv head
    int causal;              // 1: keys [0, t]; 0: keys [0, len)
    int window;              // 0 none; causal: k > t-W; bidirectional: |t-k| <= W
    float scale, softcap;
    int eager;               // eager numerics (bf16 scores, normalised bf16 probs)
    int nsplit, chunk;       // decode: 64-key chunks (nsplit = ceil(kv_cap / 64)); packed: 1, chunk = Lmax
    bf16_t* O;               // [Mq][ldo]
    int ldo;
    // decode extras: q straight from the projection's fp32 split-K slabs, PM-RoPE'd in-kernel
    const float* Qpart;      // [q_nsplit][Mq][ldqp] or null (then Q is used)
    int q_nsplit, ldqp;
    const float* pos;        // [rows] float PM positions for the q rotation
    const float* inv_freq;   // [D/2]
    float* sbuf;             // decode, rows of > 64 keys: scores [Mq][Hkv*G][kv_cap] fp32
    float* mbuf;             // decode: per-chunk score maxima [Mq][Hkv][nsplit][G]
    const float* rope_tab;   // optional per-row cos/sin table (written with layer 0's embedding norm)
    int kv_cap;              // allocated keys per (row, head): speculative loads stay below it
    // decode self-attention: the block holding key t = kv_len-1 builds it from the
    // projection slabs (k rotated by PM-RoPE, v as is), uses it and appends it to K/V
    int append, k_col0, v_col0;
    int dbg_seq;             // diagnostic timeline slot (T5G_DBG_TS builds only)
    int head_split;          // set by the decode launcher: q heads run one per workgroup
    // flash form (fast path): rows of > 64 keys in ONE launch -- each 64-key chunk's
    // workgroup writes its online-softmax partial (max, sum, unnormalised P.V), the last to
    // arrive for a (row, kv head) combines them. Tickets start (and are left) at zero.
    int flash;
    float* fpart;            // [Mq][Hkv][nsplit][G][D]
    float* fstat;            // [Mq][Hkv][nsplit][G][2] (chunk max, chunk sum)
    unsigned* fticket;       // [Mq][Hkv]
};
int attention(const AttnArgs& a, hipStream_t st);
// decode-shaped (64-key chunks over blockIdx.z + one P.V / combine launch, sdpa numerics)
int attention_decode(const AttnArgs& a, hipStream_t st);

// ---- exact-order (parity mode) kernels, exact.hip ------------------------------------
struct ExactLinArgs {
    const bf16_t* X;          // [M][ldx] bf16
    int ldx, M;
    const bf16_t* W;          // packed P16
    int N, NG, KB;            // real output rows, padded row groups (multiple of 4), K / 32
    const bf16_t* bias;
    void* Y;                  // fp32 / bf16 [M][ldy] (GEGLU: bf16 [M][N/2])
    int ldy;
    // the reference call's row count of each X row: row_len[tok_row[m]] (tok_row null:
    // row_len[m]; row_len null: 1) selects the K split kb_a[M_ref - 1] (columns >= nsplit_col:
    // kb_b) in 32-element chunks; null tables: no split
    const int* tok_row;
    const int* row_len;
    const uint16_t* kb_a;
    const uint16_t* kb_b;
    int nsplit_col, kb_len;
    int kb_fixed;             // > 0: every row splits K into parts of kb_fixed chunks (no tables)
    const uint16_t* gelu_lut; // EPI_BIAS_GELU: bf16 -> bf16 nn.GELU() table (null: exact_math.h)
};
int exact_linear(const ExactLinArgs& a, int epi, hipStream_t st);

// exact-order Linear on the f32 MFMA (xmm.hip): X and Y16 in the X16 layout, W in E16
struct XmmArgs {
    const bf16_t* X16;        // [ceil(M / 16)][KB][16][4][8] bf16 (xmm_to_x16 / producers)
    int M;
    const bf16_t* W;          // E16 packed, NG row groups x KB fragments
    int N, NG, KB;
    const bf16_t* bias;
    void* Y;                  // row-major bf16 / fp32 [M][ldy] (GEGLU: bf16 [M][N/2]) or null
    int ldy;
    bf16_t* Y16;              // optional: the bf16 output again in the X16 layout (next Linear's X)
    const int* tok_row;       // K split as ExactLinArgs
    const int* row_len;
    const uint16_t* kb_a;
    const uint16_t* kb_b;
    int nsplit_col, kb_len;
    int kb_fixed;             // > 0: every row splits K into parts of kb_fixed chunks (no tables)
    const uint16_t* gelu_lut;
    // decode rows whose K parts are all part_kbc chunks: one workgroup per (group, part),
    // each writes its part's fp32 fold to part_out[part][M][N] (the consumer adds them in
    // order from 0, as the reference's fold of parts; resid_norm's part source)
    float* part_out;
    int part_kbc;
    int timing_var;           // t5g_time_xmm only: 1 decode kernel without the fold, 2 without the MFMA
};
int xmm(const XmmArgs& a, int epi, hipStream_t st);
int pack_e16(const bf16_t* p16, bf16_t* e16, long bytes, hipStream_t st);
int to_x16(const bf16_t* X, int ldx, int M, int K, bf16_t* Y, hipStream_t st);
// X16 element offset of (row m, column k) of a matrix with KB chunks of 32 per row: per
// 16-row tile and chunk a 1 KiB block in the B-operand lane order of v_mfma_f32_16x16x4_f32
// (lane l = 16 q + j, j = row in the tile), lane l's 16 bytes the element pairs 4t + q,
// t = 0..3, of row j
__host__ __device__ inline long x16_off(long m, int k, int KB) {
    const int kb = k >> 5, e = k & 31, p = e >> 1, t = p >> 2, q = p & 3;
    return ((((m >> 4) * KB + kb) * 4 + q) * 16 + (m & 15)) * 8 + t * 2 + (e & 1);
}
// torch CPU SDPA kv blocks (common.h sdpa_*): keys per block, blocks per row. 24 blocks =
// 12 288 keys: the reference's longest call -- a 100 s prompt (5 003 prefill tokens,
// inference_commandline_hf.py:91) plus the 120 s duration cap (duration_estimator.py:79)
constexpr int SDPA_KV_BLOCK = 512;
constexpr int SDPA_MAX_BLOCKS = 24;   // 12 288 keys
constexpr int DEC_MAX_CHUNKS = SDPA_KV_BLOCK * SDPA_MAX_BLOCKS / 64;   // 64-key decode chunks per row

struct ExactAttnArgs {
    const bf16_t* Q;          // [Mq][ldq] RoPE'd queries
    int ldq, Mq;
    const int* q_row;         // [Mq] batch row (null: query index)
    const int* q_pos;         // [Mq] query index within its row's call (null: Tq - 1)
    const int* q_len;         // [B] queries of each row's reference call (null: 1)
    const bf16_t* K;          // cache [B][Hkv][cap][D]
    const bf16_t* V;
    long kv_bstride, kv_hstride;
    const int* kv_len;        // [B] keys of each row's call
    int Hq, Hkv, D;
    int causal, window;       // window > 0: sliding-window layer (explicit mask once keys >= window)
    float scale;
    int threads;              // the reference host's torch thread count (aten need_pack)
    bf16_t* O;
    int ldo;
    bf16_t* O16;              // optional: the output again in the X16 layout (K = ldo)
    // decode only (exact_attention_decode): RoPE fused into the scores launch
    const float* rope_tab;    // non-null: Q holds the UN-rotated queries; rotate them with
                              // rope_tab[row] (bf16 cos | sin, engine rope table)
    const bf16_t* kv_new;     // non-null: the step's un-rotated key / value rows of row r at
    int ld_new, k_col0, v_col0;   // kv_new[r * ld_new + k_col0 / v_col0 + head * D]: rotated,
                                  // appended at slot kv_len[row] - 1 of K / V (written) and used
    int span_max;             // decode: no row attends to more keys (0: cap); <= 64 without
                              // kv_new runs the one-launch form (xattn_single_kernel)
    float softcap;            // eager attention (eager.hip): > 0 the tanh logit softcap
    const uint16_t* tanh_lut; // eager: the reference host's bf16 tanh [65536]
};
int exact_attention(const ExactAttnArgs& a, hipStream_t st);
// decode (one query per row, at its last key): scores + P.V launches (xattn.hip) on the
// scratch sbuf [Mq][Hq][cap] / mbuf [Mq][Hkv][ceil(cap / 64)][G]
int exact_attention_decode(const ExactAttnArgs& a, float* sbuf, float* mbuf, int cap, hipStream_t st);
int sdpa_expf_array(const float* x, float* y, long n, hipStream_t st);
bool exact_attention_decode_supported(int G, int D);   // head shapes the decode launches are built for
// eager attention (attn_implementation="eager") in the reference host's order, eager.hip:
// scores + softmax/P.V launches on the scratch sbuf [Mq][Hq][cap]; -3: not the measured shape
int eager_attention(const ExactAttnArgs& a, float* sbuf, int cap, hipStream_t st);
int sort_emu_wave(int n, int S, int* pos, float* val, int* tag, int* out, hipStream_t st);   // sampler.hip test entry

// ---- sampler -------------------------------------------------------------------
struct SamplerRow {           // per-utterance parameters (device)
    int top_k;                // <= 0 disabled
    int top_k_list_len;       // > 0: top_k_list[min(len-1, cur_num_gen)]
    int top_k_list_off;       // offset into the shared top-k list buffer
    float top_p, min_p, temperature;
    int stop_repetition;
    int n_silence;
    int silence_off;          // offset into the shared silence-token buffer
    int eos_disabled;
    uint32_t seed_lo, seed_hi;
};
struct SamplerState {         // per-utterance AR state (device), see inference_tts locals
    int cur_num_gen;
    int current_length;       // == self-attention keys in cache after the current input
    int prompt_offset;
    int target_total;         // < 0: none
    int est_total;
    int prev_token;
    int consec_silence;
    int first_input_len;
    int done;
    int ambiguous_steps;      // top-p tie groups straddling the cut (parity info)
    int last_token;
    float next_pos;           // PM position of the next decoder input
};
struct SamplerArgs {
    const bf16_t* logits;     // [B][ldl]
    int ldl, V, B;
    const SamplerRow* rows;
    SamplerState* state;
    const int* top_k_list;
    const int* silence;
    const bf16_t* noise;      // parity mode: [B][noise_steps][V] bf16 or null (Philox)
    int noise_steps;
    const uint32_t* noise_mt; // parity mode: raw MT19937 outputs [B][noise_mt_steps][2 V] (noise.hip)
    int noise_mt_steps;
    int eos, eos_guard;       // eos id, encodec_sr // 5
    float budget_extra;       // int(encodec_sr) * extra_cutoff
    int text_guard;           // text_guard_frames_per_token
    float progress_scale;
    int* out_tokens;          // [B][max_gen]
    int max_gen;
    int max_len;              // self-attention cache slots per row (engine max_audio)
    int* kv_len;              // [B] self-attention keys (advanced with current_length)
    float* next_pos;          // [B] float PM position for the next step
    int* next_token;          // [B] token fed to the next decoder step
    int* flags;               // [B] per-step debug: bit0 ambiguous
    unsigned* hist;           // scratch [B][65536] (top-p histogram walk)
    // multi-block fast path (top-k <= FS_KMAX, no min_p): per-slice candidates
    float* fs_val;            // [B][FS_NB][FS_CAP] temperature-scaled candidate values
    int* fs_idx;              // [B][FS_NB][FS_CAP]
    int* fs_cnt;              // [B][FS_NB] candidates written (-1: overflow)
    float* fs_amv;            // [B][FS_NB] slice argmax value (edited logits)
    int* fs_ami;              // [B][FS_NB] slice argmax index
    unsigned* fs_ticket;      // [B] arrival counters (reset by the last block)
    int* fs_slow;             // [B] 1: row left to the single-block kernel this step
    int dbg_seq;             // diagnostic timeline slot (T5G_DBG_TS builds only)
};
constexpr int FS_NB = 16;     // slices (blocks) per row
constexpr int FS_CAP = 128;   // candidates per slice
constexpr int FS_KMAX = 64;   // largest top-k the fast path takes
constexpr int FS_SMAX = 256;  // largest top-k survivor set (ties) the fast path takes
size_t sampler_fast_ws_bytes(int B);

// ---- parity-mode noise (noise.hip) ------------------------------------------------
// init [B][625]: MT19937 words + consumed position; raw outputs [B][out_stride] (n_out per
// row); optional snapshots of the generator every snap_every outputs [B][n_snap][625]
int mt_stream(const uint32_t* init, int B, long n_out, long out_stride, uint32_t* out, long snap_every, int n_snap,
              uint32_t* snap, hipStream_t st);
int mt_exponential(const uint32_t* raw, long n, bf16_t* q, hipStream_t st);
int sample(const SamplerArgs& a, hipStream_t st);
}  // namespace t5g

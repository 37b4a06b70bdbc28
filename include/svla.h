/*
 * svla.h — C-ABI of the MI355X (gfx950) SpatialVLA hot-path kernels (libsvla.so).
 *
 * Drop-in boundary.  Every entry point replaces one op of the reference's
 * eager PyTorch/flash-attn/DeepSpeed path; the reference interface each one replaces is cited
 * next to it.  Conventions (all entry points):
 *   - plain pointers + sizes, no torch types; caller owns every buffer (incl. workspace),
 *     kernels never allocate or free;
 *   - bf16 tensors are raw 16-bit bit patterns (uint16_t), row-major unless stated;
 *   - launches are asynchronous and stream-ordered on `stream` (a hipStream_t), no host sync;
 *   - return 0 on success, SVLA_ERR_ARG on a rejected argument, SVLA_ERR_HIP on a launch
 *     failure; svla_last_error() returns the thread-local message of the last failure;
 *   - deterministic: no float atomics anywhere, so results are bitwise run-to-run stable.
 */
#ifndef SVLA_H_
#define SVLA_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { SVLA_OK = 0, SVLA_ERR_ARG = 1, SVLA_ERR_HIP = 2 };

/* Last error message of the calling thread ("" if none). */
const char* svla_last_error(void);
/* Library version string and the gfx target it was built for. */
const char* svla_version(void);

/* ------------------------------------------------------------------------------------------
 * GEMM  C[M,N] (op)= epilogue( sum_k A(m,k) * B(n,k) ), bf16 in, fp32 accumulate (MFMA 16x16x32).
 * Replaces every nn.Linear / torch.matmul of the hot path: Gemma2 q/k/v/o and gate/up/down
 * (reference model/modeling_gemma2.py:86-92, 351-354, 376-408), lm_head (:895, :993),
 * SigLIP q/k/v/out/fc1/fc2 and patch-embed conv (transformers siglip [3p]), projector
 * (model/modeling_spatialvla.py:124), Ego3D MLP (:59-64) — forward and both backward GEMMs.
 * ---------------------------------------------------------------------------------------- */
enum { SVLA_LAYOUT_KC = 0, /* element (r,k) at ptr[r*ld + k]  (reduction dim contiguous) */
       SVLA_LAYOUT_RC = 1  /* element (r,k) at ptr[k*ld + r]  (outer dim contiguous)     */ };
enum { SVLA_SEG_OUTER = 0, SVLA_SEG_K = 1, SVLA_SEG_GEGLU = 2 };

/* One GEMM operand.  r = outer index (m for A, n for B), k = reduction index.
 * Up to 4 segments along `seg_dim`: segment s covers [seg_start[s], seg_start[s+1]) of that
 * index and reads ptr[s] with the index rebased to seg_start[s] (lets q/k/v or gate/up weights
 * that live in separate tensors act as one operand).  Segment starts must be tile aligned
 * (128 on the outer dim, 64 on k).  SVLA_SEG_GEGLU (B only): outer row n of tile t=n/128 reads
 * ptr[0] row 64t+(n%128) if n%128<64 else ptr[1] row 64t+(n%128)-64 (gate/up interleave). */
typedef struct {
  const void* ptr[4];
  int64_t seg_start[5];
  int32_t nseg;
  int32_t seg_dim;
  int32_t layout;
  int32_t _pad;
  int64_t ld;
  int64_t r_valid;   /* readable extent of the outer index (0 = M or N); beyond it the operand reads as 0 */
  int64_t k_valid;   /* readable extent of the reduction index (0 = K); beyond it the operand reads as 0 */
} svla_operand;

enum {
  SVLA_EPI_STORE = 0,      /* C = alpha*acc                                                  */
  SVLA_EPI_BIAS = 1,       /* C = alpha*acc + bias[n]                                        */
  SVLA_EPI_BIAS_GELU = 2,  /* pre = bf16(acc+bias) -> out1;  C = gelu_tanh(pre)               */
  SVLA_EPI_BIAS_RESID = 3, /* C = bf16(acc+bias) + in0[m,n]   (bias optional)                 */
  SVLA_EPI_GEGLU = 4,      /* B uses SVLA_SEG_GEGLU; g->out1, u->out2, C = gelu_tanh(g)*u     */
  SVLA_EPI_GEGLU_BWD = 5,  /* acc = dH; in0=g, in1=u: out1 = dH*u*gelu'(g), out2 = dH*gelu(g) */
  SVLA_EPI_GELU_BWD = 6,   /* acc = dAct; in0 = pre-activation: C = dAct*gelu'(pre)           */
  SVLA_EPI_SOFTCAP_CE = 7, /* C = cap*tanh(acc/cap); row_stats[m, tile_n] = {max,sumexp,argmax} */
  SVLA_EPI_ROPE = 8,       /* C = bf16(acc), then Gemma2 rotate_half RoPE on columns < rope_cols (heads of
                              rope_D, position m % rope_L, tables [rope_L][rope_D/2]) with the reference's bf16
                              rounding: bf16(bf16(x*cos) + bf16(rotate_half(x)*sin))
                              (model/modeling_gemma2.py:123-154) — q/k leave the QKV GEMM rotated */
  SVLA_EPI_BIAS_GELU_ERF = 9,    /* C = bf16(gelu_erf(bf16(acc + bias[n])))  (BEiT MLP fc1 + exact GELU, no
                                    pre-activation output: the ZoeDepth backbone is frozen) */
  SVLA_EPI_BIAS_SCALE_RESID = 10 /* C = bf16(bf16(colscale[n] * bf16(acc + bias[n])) + in0[m,n])  (BEiT layer
                                    scale lambda * sublayer + residual; bias optional) */
};

typedef struct {
  int32_t kind;
  int32_t accumulate;        /* 1: C += result (STORE only) */
  float alpha;
  float cap;
  const void* bias;          /* [N] bf16 */
  const void* in0; int64_t ld_in0;
  const void* in1; int64_t ld_in1;
  void* out1; int64_t ld_out1;
  void* out2; int64_t ld_out2;
  float* row_stats;          /* [M][ceil(N/128)][3] fp32 (SOFTCAP_CE) */
  const void* rope_cos;      /* ROPE: bf16 [rope_L][rope_D/2] tables, row stride rope_ld */
  const void* rope_sin;
  int64_t rope_ld;
  int64_t rope_cols;         /* columns [0, rope_cols) are rotated (q and k heads), the rest (v) plain */
  int32_t rope_L;            /* sequence length: row m is position m % rope_L */
  int32_t rope_D;            /* head dim; the GEMM tile width must be a multiple of it */
  const void* colscale;      /* [N] bf16 (BIAS_SCALE_RESID) */
  void* mx_q;                /* GEGLU on the fp8 GEMMs (svla_gemm_mxfp8 / svla_gemm_fp8) only, else NULL: also the
                                OCP MX e4m3 copy of C (h) -- [M][mx_ldq] bytes, E8M0 scales in svla_quant_mx_rows'
                                layout (mx_sld >= 4 M), bitwise svla_quant_mx_rows of the stored bf16 h; N/2 % 128 == 0 */
  int64_t mx_ldq;
  void* mx_scales;
  int64_t mx_sld;
} svla_epilogue;

/* C: up to 4 row segments (c_seg_start tile-aligned to 128) — lets dW of q/k/v (or gate/up)
 * land directly in separate gradient tensors.  c_nseg = 1 for a plain matrix.
 * Requirements: ld of every operand and of C a multiple of 8 elements; pointers 16-B aligned; the
 * reduction extent of a KC operand (k_valid, default K) a multiple of 8 (zero-pad: e.g. the lm_head
 * dlogits rows are zero beyond V up to their padded ld). */
/* workspace: caller-owned stream-K / split-K workspace (fp32 partial slabs + arrival counters of the 256x256
 * kernels' stream-K and of the short-M split-K tiles; 256-B aligned, zero-filled once before its first use, at
 * least svla_gemm_workspace_bytes() for the current device; the kernels leave the counters zeroed).  NULL = every
 * output tile runs whole.  GEMMs that run concurrently (other streams, other threads) must use distinct
 * workspaces; nothing else is shared between calls, so the entry point is re-entrant. */
int svla_gemm_bf16(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B,
                   void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                   const svla_epilogue* epi, void* workspace, size_t ws_bytes, void* stream);
/* Cap (this host thread) on the persistent grid of the stream-K GEMM schedules: the GEMMs it launches next use at
 * most `cap` workgroups a persistent wave (0 = every CU).  Set around a GEMM queued on a side stream so the main
 * stream's kernels find free CUs beside it; results stay deterministic (a fixed cap fixes the split). */
void svla_gemm_set_cu_cap(int cap);
size_t svla_gemm_workspace_bytes(void);
/* svla_gemm_bf16 with an explicit kernel choice (tests / tuning tools, not a reference interface): 0 = auto (as
 * svla_gemm_bf16), 1 = two-barrier tiles, 2 = 8-phase without stream-K, 3 = 4-wave kernel for every 256x256 case,
 * 4 = never the 4-wave kernel, 5 = auto without the small-M GEMV path, 6 = small-M GEMVs without the prefetching
 * kernel, 7 = the prefetching GEMV with two rows per wave, 8 = 8-phase + stream-K for every sub-wave grid, 9 = the
 * 64x64 two-stage tiles for sub-wave grids, 10 / 11 / 12 / 16 = the deep-pipelined 64x64 / 64x128 / 128x128 /
 * 128x256 tiles (both operands KC), 13 / 14 / 15 / 17 = the same with split-K. */
int svla_gemm_bf16_ex(int64_t M, int64_t N, int64_t K, const svla_operand* A, const svla_operand* B,
                      void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                      const svla_epilogue* epi, void* workspace, size_t ws_bytes, int32_t variant, void* stream);

/* ------------------------------------------------------------------------------------------
 * fp8 projections (BASELINE configs[4]; OCP e4m3 on v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulate).
 * Replaces the bf16 nn.Linear of Gemma2 q/k/v/o and gate/up/down (model/modeling_gemma2.py:86-92, 351-354,
 * 376-408) in the forward and the input-gradient (dgrad) GEMMs when fp8 projections are enabled.  Two scalings:
 * OCP MX block scales (svla_quant_mx_rows + svla_gemm_mxfp8: one E8M0 scale per 32 consecutive k of a row, fed to
 * the MFMA; the product path) and per-row fp32 scales (svla_quant_fp8_rows + svla_gemm_fp8: unit MFMA block
 * scales, row scales applied in the epilogue).
 * ---------------------------------------------------------------------------------------- */
/* OCP MX (Microscaling spec v1.0) e4m3 quantisation of rows: for each block of 32 consecutive k of row r,
 * X = clamp(floor(log2(amax)) - 8, -127, 127), q[r,k] = e4m3(clamp(x[r,k] * 2^-X, +-448)) (RNE), scale byte
 * E8M0 = 127 + X.  Scales are tile-major: the 4 bytes of row r in 128-k tile t at scales[t * sld + 4 r]
 * (sld >= 4 rows, a multiple of 4), so a k-tile's scales of 256 consecutive rows are contiguous.  x bf16
 * [rows][ldx], q bytes [rows][ldq]; K % 128 == 0. */
int svla_quant_mx_rows(int64_t rows, int64_t K, const void* x, int64_t ldx, void* q, int64_t ldq, void* scales,
                       int64_t sld, void* stream);
/* The same quantisation of the rows of W^T, read from W [N][ldw] bf16 without a transposed copy: q[k][n] bytes
 * [K][ldq], blocks of 32 consecutive n, scales in svla_quant_mx_rows' layout for a [K]-row matrix (the dgrad
 * operand of svla_gemm_mxfp8); bitwise svla_quant_mx_rows(W^T).  N % 128 == 0, K % 64 == 0, ldq % 16 == 0. */
int svla_quant_mx_cols(int64_t N, int64_t K, const void* w, int64_t ldw, void* q, int64_t ldq, void* scales,
                       int64_t sld, void* stream);
/* Both MX layouts of W [R][ldw] bf16 from one read: q_rows [R][C] (blocks along C) = svla_quant_mx_rows(W) and
 * q_cols [C][R] (blocks along R) = svla_quant_mx_rows(W^T), each with its scales in that layout (the fp8 weight
 * copies of the forward and the dgrad GEMMs).  R % 128 == 0, C % 128 == 0, ldq_cols % 16 == 0. */
int svla_quant_mx_both(int64_t R, int64_t C, const void* w, int64_t ldw, void* q_rows, int64_t ldq_rows, void* sc_rows,
                       int64_t sld_rows, void* q_cols, int64_t ldq_cols, void* sc_cols, int64_t sld_cols,
                       void* stream);
/* C[M,N] = epilogue( sum_k 2^(Xa(m,k/32) + Xb(n,k/32)) A(m,k) B(n,k) ): A, B e4m3 KC operands as svla_gemm_fp8
 * with their MX block scales in svla_quant_mx_rows' layout (a_mx: M rows, b_mx: N rows -- GEGLU: the gate rows then
 * the up rows of one [N] scale matrix; *_ld the per-k-tile stride, *_bytes the buffer size); K and k_valid
 * multiples of 128.  Epilogues and workspace as svla_gemm_fp8. */
int svla_gemm_mxfp8(int64_t M, int64_t N, int64_t K, const svla_operand* A, const void* a_mx, int64_t a_mx_ld,
                    int64_t a_mx_bytes, const svla_operand* B, const void* b_mx, int64_t b_mx_ld, int64_t b_mx_bytes,
                    void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                    const svla_epilogue* epi, void* workspace, size_t ws_bytes, void* stream);
/* Row-wise quantisation: x'[r,k] = x[r,k] * colscale[k] (colscale fp32 [K], 16-B aligned, or NULL = 1);
 * scale[r] = amax_r(x')/448, q[r,k] = e4m3(clamp(x'[r,k]*448/amax_r, +-448)) (RNE; a zero row gives q = 0,
 * scale 0).  x bf16 [rows][ldx], q bytes [rows][ldq]; K % 8 == 0 (the dgrad GEMMs quantise dY with
 * colscale = the row scales of the forward fp8 weight, so the weight's transposed e4m3 copy is reused as is). */
int svla_quant_fp8_rows(int64_t rows, int64_t K, const void* x, int64_t ldx, const float* colscale, void* q,
                        int64_t ldq, float* scale, void* stream);
/* Byte transpose out[c][r] = in[r][c] of an R x C matrix (the e4m3 weight copies for the dgrad GEMMs).
 * ldi % 16 == 0, ldo % 4 == 0, 16-B aligned input. */
int svla_transpose_u8(int64_t R, int64_t C, const void* in, int64_t ldi, void* out, int64_t ldo, void* stream);
/* C[M,N] = epilogue( a_scale[m] * b_scale[n] * sum_k A(m,k) B(n,k) ) with A, B e4m3 KC operands (ld in bytes, a
 * multiple of 16; K and k_valid multiples of 16; A one segment; B one segment, or two SVLA_SEG_GEGLU segments of
 * N/2 rows with SVLA_EPI_GEGLU, b_scale then [N]: gate rows then up rows).  Scales fp32, 16-B aligned.  Epilogues
 * STORE (alpha 1), BIAS, BIAS_RESID, GEGLU, ROPE as svla_gemm_bf16; workspace as svla_gemm_bf16. */
int svla_gemm_fp8(int64_t M, int64_t N, int64_t K, const svla_operand* A, const float* a_scale, const svla_operand* B,
                  const float* b_scale, void* const* c_ptr, const int64_t* c_seg_start, int32_t c_nseg, int64_t ldc,
                  const svla_epilogue* epi, void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Attention.  Reference: eager_attention_forward (model/modeling_gemma2.py:169-195) selected via
 * GEMMA2_ATTENTION_FUNCTION (:317-322) with the prefix-LM additive mask of
 * _update_causal_mask (model/modeling_spatialvla.py:258-306) and Gemma2 RoPE
 * (modeling_gemma2.py:95-154); SigLIP eager attention (transformers siglip [3p], no mask).
 * The [B,1,L,L] mask is never materialised: kv_class[b, j] (uint8) classifies key j:
 *   0 = visible to every query, 1 = visible to queries i >= j, 2 = never visible;
 * plus an optional sliding window (key j masked for query i when i - j >= window, 0 = off).
 * Masked scores take the bf16 minimum (-3.3895e38) exactly as the reference's additive mask.
 * q/k/v are read in place from projection outputs: element (b, t, h, d) at
 *   base + (b*L + t)*ld + h*D + d.
 * q and k arrive already rotated (Gemma2 RoPE is applied in the QKV GEMM epilogue, SVLA_EPI_ROPE).
 * rope_cos/rope_sin ([L][D/2] bf16, row stride rope_ld) are for svla_attn_bwd only: with them dq/dk are
 * returned w.r.t. the pre-rotation q/k (the transpose of rotate_half RoPE applied to the gradients);
 * svla_attn_fwd rejects them.
 * bias (optional, forward only): an additive score bias shared by the batch, element (h, i, j) at
 * bias + (h*L + i)*bias_ld + j (bf16; bias_ld >= round8(L), a multiple of 8) — BEiT's relative position bias (transformers beit BeitLayer [3p], the
 * ZoeDepth backbone called at model/modeling_spatialvla.py:314-323); not combined with softcap or kv_class.
 * head_dim D in {256, 72, 64}; L <= 8192.  lse: [B, Hq, L] fp32 (natural log of the softmax denominator).
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  int32_t B, L, Hq, Hkv, D;
  int32_t sliding_window;
  float scale;      /* query_pre_attn_scalar^-0.5 (Gemma2) or D^-0.5 (SigLIP) */
  float softcap;    /* 0 = off */
  const void* q; int64_t ldq;
  const void* k; int64_t ldk;
  const void* v; int64_t ldv;
  const uint8_t* kv_class;   /* [B, L] or NULL (= all visible) */
  const void* rope_cos;      /* [L][D/2] bf16 or NULL (backward only) */
  const void* rope_sin;
  int64_t rope_ld;
  const void* bias;          /* [Hq][L][bias_ld] bf16 additive score bias or NULL (forward only) */
  int64_t bias_ld;
} svla_attn_args;

int svla_attn_fwd(const svla_attn_args* a, void* out, int64_t ldo, float* lse, void* stream);
/* KV-cached decode attention.  Replaces the HybridCache decode step of
 * SpatialVLAForConditionalGeneration.generate / predict_action (model/modeling_spatialvla.py:440-492) through
 * eager_attention_forward (model/modeling_gemma2.py:169-195, cache update :387-395).
 * Lq new queries per sequence sit at absolute positions Lk-Lq .. Lk-1 and attend to the first Lk cached keys:
 *   q   (b, t, h, d) at q + (b*Lq + t)*ldq + h*D + d              (already rotated)
 *   k/v (b, j, h, d) at k + b*bsk + j*ldk + h*D + d               (cache rows, keys already rotated)
 *   out (b, t, h, d) at out + (b*Lq + t)*ldo + h*D + d
 * kv_class[b*ldc + j] as svla_attn_fwd (0 prompt key, 1 causal, 2 never visible); sliding window as there.
 * D in {64,128,256}; Hq/Hkv in {1,2,4}; any Lk (keys are split into 64-key chunks across workgroups).
 * workspace: >= svla_attn_decode_workspace_bytes(B, Lq, Hq, Lk, D) bytes (fp32 chunk partials). */
typedef struct {
  int32_t B, Lq, Lk, Hq, Hkv, D;
  int32_t sliding_window;
  float scale;
  float softcap;
  const void* q; int64_t ldq;
  const void* k; int64_t ldk; int64_t bsk;
  const void* v; int64_t ldv; int64_t bsv;
  const uint8_t* kv_class; int64_t ldc;
} svla_attn_decode_args;

size_t svla_attn_decode_workspace_bytes(int32_t B, int32_t Lq, int32_t Hq, int32_t Lk, int32_t D);
int svla_attn_decode(const svla_attn_decode_args* a, void* out, int64_t ldo, float* workspace, size_t ws_bytes,
                     void* stream);

/* The decode step's attention in ONE launch: svla_qkv_rope_append + svla_attn_decode fused (same results, bitwise).
 * a->q / a->ldq point at the raw q|k|v projection rows (row b*Lq+t: Hq q heads, Hkv k heads, Hkv v heads, not yet
 * rotated); the new tokens sit at cache rows p0 = Lk-Lq .. Lk-1 and token row b*Lq+t uses RoPE table row b*Lq+t
 * (rope_cos/rope_sin [B*Lq, >=D/2], rope_ld): per-sequence positions, as the reference's generate derives them
 * from attention_mask.cumsum(-1) for padded prompts (modeling_gemma2.py:1039-1042).  The rotated k and the v rows are appended to cache rows p0+t; q is not written back.
 * workspace: >= svla_attn_decode_rope_workspace_bytes(...) bytes, 256-B aligned, ZEROED ONCE by the caller (its
 * head holds arrival counters that every launch returns to zero; one workspace per stream).
 * Replaces modeling_gemma2.py:123-154 (RoPE), :387-395 (HybridCache update) and :169-195 (eager attention). */
size_t svla_attn_decode_rope_workspace_bytes(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t Lk, int32_t D);
int svla_attn_decode_rope(const svla_attn_decode_args* a, const void* rope_cos, const void* rope_sin, int64_t rope_ld,
                          void* out, int64_t ldo, void* workspace, size_t ws_bytes, void* stream);

/* Decode-step q|k|v epilogue: rotate_half RoPE on q in place (rows b*Lq+t of qkv, position table row b*Lq+t) and on
 * k, rotated k and plain v written to cache rows p0+t (k/v cache element (b, j, h, d) at base + b*bs + j*ld + h*D + d).
 * Replaces apply_rotary_pos_emb + the HybridCache update (model/modeling_gemma2.py:123-154, :387-395). */
int svla_qkv_rope_append(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t D, void* qkv, int64_t ld,
                         const void* rope_cos, const void* rope_sin, int64_t rope_ld, void* k_cache, int64_t ldk,
                         int64_t bsk, void* v_cache, int64_t ldv, int64_t bsv, int32_t p0, void* stream);

/* The prefill's form of svla_qkv_rope_append (same arguments and rounding): q AND k rotated in place in the projection
 * rows (where the prompt's flash attention reads them), rotated k and plain v also written to cache rows p0+t -- one
 * launch instead of a RoPE pass and two cache copies (model/modeling_gemma2.py:123-154, :387-395). */
int svla_qkv_rope_fill(int32_t B, int32_t Lq, int32_t Hq, int32_t Hkv, int32_t D, void* qkv, int64_t ld,
                       const void* rope_cos, const void* rope_sin, int64_t rope_ld, void* k_cache, int64_t ldk,
                       int64_t bsk, void* v_cache, int64_t ldv, int64_t bsv, int32_t p0, void* stream);

/* dq/dk/dv use the same in-place layout convention as q/k/v (ld_dq, ld_dk, ld_dv).
 * workspace: B*Hq*L fp32 (row dot(dO, O), formed by the dQ kernel and read by the dK/dV kernel). */
int svla_attn_bwd(const svla_attn_args* a, const void* out, int64_t ldo, const void* dout, int64_t lddo,
                  const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv,
                  float* workspace, void* stream);
/* The same backward for head_dim 256 (Gemma2, modeling_gemma2.py:169-195) with dS stored instead of recomputed:
 * delta = rowsum(dO * O) -> dK/dV (which also writes dS^T, bf16 [B][Hq][round64(L)][round64(L)]) -> dQ = dS K.
 * workspace: >= svla_attn_bwd_ds_workspace_bytes(B, L, Hq) bytes, 256-B aligned (delta, then dS^T). */
size_t svla_attn_bwd_ds_workspace_bytes(int32_t B, int32_t L, int32_t Hq);
int svla_attn_bwd_ds(const svla_attn_args* a, const void* out, int64_t ldo, const void* dout, int64_t lddo,
                     const float* lse, void* dq, int64_t lddq, void* dk, int64_t lddk, void* dv, int64_t lddv,
                     void* workspace, size_t ws_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Norms.  Gemma2RMSNorm (modeling_gemma2.py:60-77): y = bf16(x*rsqrt(mean(x^2)+eps)*(1+w)) in fp32.
 * Residual form (decoder layer :489-496): h = bf16(res + bf16(rms(y_in; w))).
 * LayerNorm (SigLIP layer_norm1/2/post, Ego3D head.1): y = bf16((x-mu)*rstd*w + b).
 * rows of length N (ld = N).  rstd/mean saved per row (fp32) for backward.
 * ---------------------------------------------------------------------------------------- */
int svla_rmsnorm_fwd(int64_t rows, int64_t N, const void* x, const void* w, float eps, void* y,
                     float* rstd, void* stream);
/* dw_partial: [ceil(rows/rows_per_block)] x N fp32 partial sums, reduced by svla_colsum_f32. */
int svla_rmsnorm_bwd(int64_t rows, int64_t N, const void* x, const void* w, const float* rstd,
                     const void* dy, const void* dres, void* dx, float* dw_partial, int64_t* n_partial,
                     void* stream);
int svla_add_rmsnorm_fwd(int64_t rows, int64_t N, const void* res, const void* yin, const void* w, float eps,
                         void* h, float* rstd, void* stream);
/* Backward of the training pair svla_add_rmsnorm2_fwd_train (h = res + rms(y; w1), x = rms(h; w2)) in one pass:
 * dh_out = bf16(bf16(rms_bwd(h; dx)) + dres) (dres may be NULL), dy_out = bf16(rms_bwd(y; dh_out)); dw_partial: two
 * planes [2][ceil(rows/8)][N] fp32 (w2's partials, then w1's) for svla_colsum2_f32.  dh_out / dy_out are bitwise
 * two svla_rmsnorm_bwd calls; dw is the same sum over 8-row instead of 16-row partials. */
int svla_rmsnorm2_bwd(int64_t rows, int64_t N, const void* h, const void* w2, const float* rstd2, const void* dx,
                      const void* dres, const void* y, const void* w1, const float* rstd1, void* dh_out, void* dy_out,
                      float* dw_partial, int64_t* n_partial, void* stream);
/* svla_rmsnorm_bwd / svla_rmsnorm2_bwd that also write the OCP MX e4m3 copy of the input gradient they store (dx,
 * resp. dy) -- q [rows][ldq] bytes, E8M0 scales in svla_quant_mx_rows' layout (sld >= 4 rows), bitwise
 * svla_quant_mx_rows of it: the fp8 dgrad operands of the down and o projections, without a separate pass.
 * N % 128 == 0 (svla_rmsnorm_bwd_mx: N > 1536, the block-per-row kernel). */
int svla_rmsnorm_bwd_mx(int64_t rows, int64_t N, const void* x, const void* w, const float* rstd, const void* dy,
                        const void* dres, void* dx, float* dw_partial, int64_t* n_partial, void* q, int64_t ldq,
                        void* scales, int64_t sld, void* stream);
int svla_rmsnorm2_bwd_mx(int64_t rows, int64_t N, const void* h, const void* w2, const float* rstd2, const void* dx,
                         const void* dres, const void* y, const void* w1, const float* rstd1, void* dh_out,
                         void* dy_out, float* dw_partial, int64_t* n_partial, void* q, int64_t ldq, void* scales,
                         int64_t sld, void* stream);
/* h = res + rmsnorm(yin; w1), x = rmsnorm(h; w2) in one pass (inference; bitwise the two separate calls):
 * Gemma2 post-attention + pre-feedforward norms, or post-feedforward + next input norm (modeling_gemma2.py:487-496). */
int svla_add_rmsnorm2_fwd(int64_t rows, int64_t N, const void* res, const void* yin, const void* w1, const void* w2,
                          float eps1, float eps2, void* h, void* x, void* stream);
/* The same pair in the training forward: also writes the per-row rstd of both norms (fp32 [rows] each) for the two
 * svla_rmsnorm_bwd calls of the backward.  Decoder layer post-attention + pre-feedforward norms
 * (modeling_gemma2.py:487-490); bitwise svla_add_rmsnorm_fwd followed by svla_rmsnorm_fwd. */
int svla_add_rmsnorm2_fwd_train(int64_t rows, int64_t N, const void* res, const void* yin, const void* w1,
                                const void* w2, float eps1, float eps2, void* h, void* x, float* rstd1, float* rstd2,
                                void* stream);
/* The training forwards of svla_rmsnorm_fwd and svla_add_rmsnorm2_fwd_train that also write the OCP MX e4m3 copy of
 * the normalised output (y, resp. x): q [rows][ldq] bytes with E8M0 scales in svla_quant_mx_rows' layout (sld >= 4
 * rows) -- bitwise svla_quant_mx_rows of the bf16 output, the fp8 q|k|v / gate|up operand without a separate
 * pass.  N % 128 == 0. */
int svla_rmsnorm_fwd_mx(int64_t rows, int64_t N, const void* x, const void* w, float eps, void* y, float* rstd,
                        void* q, int64_t ldq, void* scales, int64_t sld, void* stream);
int svla_add_rmsnorm2_fwd_train_mx(int64_t rows, int64_t N, const void* res, const void* yin, const void* w1,
                                   const void* w2, float eps1, float eps2, void* h, void* x, float* rstd1,
                                   float* rstd2, void* q, int64_t ldq, void* scales, int64_t sld, void* stream);
int svla_layernorm_fwd(int64_t rows, int64_t N, const void* x, const void* w, const void* b, float eps,
                       void* y, float* mean, float* rstd, void* stream);
/* dwb_partial: two planes [2][ceil(rows/rows_per_block)][N] fp32 (dw partials, then db partials), reduced by
 * svla_colsum2_f32. */
int svla_layernorm_bwd(int64_t rows, int64_t N, const void* x, const void* w, const float* mean,
                       const float* rstd, const void* dy, const void* dres, void* dx, float* dwb_partial,
                       int64_t* n_partial, void* stream);
/* out[n] = bf16(sum_p in[p, n]) (+ existing out if accumulate): reduces partial sums in one launch, fixed order
 * (the weight-gradient reduction autograd does for Gemma2RMSNorm.weight / nn.LayerNorm, modeling_gemma2.py:60-77).
 * N % 8 == 0; workspace unused (may be NULL). */
int svla_colsum_f32(int64_t P, int64_t N, const float* in, void* out_bf16, int32_t accumulate, float* workspace,
                    void* stream);
/* The two planes [2][P][N] of svla_layernorm_bwd in one launch: out0 = bf16(sum_p in[0][p]), out1 = plane 1. */
int svla_colsum2_f32(int64_t P, int64_t N, const float* in, void* out0_bf16, void* out1_bf16, int32_t accumulate,
                     void* stream);
/* out[n] = bf16(sum_m x[m, n]) over a bf16 matrix (bias gradients of nn.Linear), fixed order, run-to-run bitwise.
 * N % 8 == 0, ldx % 8 == 0.  workspace: NULL = one launch (one block per 32 columns), or
 * svla_colsum_bf16_workspace_bytes(M, N) bytes (16-B aligned; 0 = the split does not pay) = row slices summed into
 * fp32 partial rows, then reduced in slice order (two launches, the chip filled for narrow N). */
size_t svla_colsum_bf16_workspace_bytes(int64_t M, int64_t N);
int svla_colsum_bf16(int64_t M, int64_t N, const void* x, int64_t ldx, void* out_bf16, int32_t accumulate,
                     float* workspace, void* stream);

/* ------------------------------------------------------------------------------------------
 * Elementwise / glue.
 * ---------------------------------------------------------------------------------------- */
/* Embedding merge (modeling_spatialvla.py:361-387 + modeling_gemma2.py:741-742):
 * out[b,t] = normalizer * (ids in [a0, a0+na) ? spatial[ids-a0] : (ids == image_id ? img[next] : embed[ids]))
 * img rows consumed in (b,t) order (masked_scatter); img_pos[b*L+t] = running image index (host computed). */
int svla_embed_merge(int64_t rows, int64_t H, const int64_t* ids, const int32_t* img_index, const void* embed,
                     const void* spatial, int64_t a0, int64_t na, const void* img, float normalizer, void* out,
                     void* stream);
/* Backward of the merge: spatial-table grad (deterministic per-row segmented sum) and image-feature grad. */
int svla_embed_merge_bwd(int64_t rows, int64_t H, const int64_t* ids, const int32_t* img_index,
                         const int32_t* spatial_sorted_rows, const int32_t* spatial_offsets, int64_t na,
                         const void* dout, float normalizer, void* dspatial, void* dimg, void* stream);
/* Ego3D (modeling_spatialvla.py:195-223, :74-91): area-pool fp32 depth [B,1,Hd,Wd] to (hp*reso)^2, back-project
 * with inv(K) @ uv_h (uv_h passed in, bf16-quantised as the model buffer), permute per patch,
 * normalise ((xyz-center)/2 -> bf16), frequency-encode -> feat [B, hp*wp, ldf] bf16 (cols >= 12*(2F+1) zeroed). */
int svla_ego3d_encode(int32_t B, int32_t Hd, int32_t Wd, const void* depth, const float* kinv, const float* uv_h,
                      int32_t patch, int32_t reso, int32_t n_freqs, void* feat, int64_t ldf, float* xyz_out,
                      void* stream);
/* inv(K) of B row-major 3x3 fp32 matrices by the closed-form adjugate / determinant (camera intrinsics;
 * replaces torch.linalg.inv(K.float()) of backproject_patch, model/modeling_spatialvla.py:221).  No host sync. */
int svla_inv3x3_f32(int32_t B, const float* K, float* kinv, void* stream);
/* SigLIP patchify (Conv2d k=s=patch): x [B,3,S,S] bf16 already normalised -> cols [B*(S/p)^2, ldc]
 * with column order (c, ky, kx) as the conv weight flattening; columns >= 3p^2 zeroed. */
int svla_im2col_patch(int32_t B, int32_t S, int32_t patch, const void* x, void* cols, int64_t ldc,
                      void* stream);
/* out = bf16(bf16(x + offset) * scale) elementwise: TF.normalize((x), mean, std) with offset=-mean,
 * scale=1/std (modeling_spatialvla.py:309; bf16 rounding after the subtraction as torchvision does). */
int svla_affine_bf16(int64_t n, const void* x, float scale, float offset, void* out, void* stream);
/* y = relu(x) (Ego3D head.2) fwd/bwd */
int svla_relu_fwd(int64_t n, const void* x, void* y, void* stream);
int svla_relu_bwd(int64_t n, const void* x, const void* dy, void* dx, void* stream);
/* out = bf16(a + b) */
/* GeGLU backward of Gemma2MLP (modeling_gemma2.py:91-92): dg = bf16(dh*u)*gelu_tanh'(g), du = dh*bf16(gelu_tanh(g))
 * over [M, I] bf16 rows with leading dimensions (I % 8 == 0, 16-B aligned rows); dg may alias dh. */
int svla_geglu_bwd(int64_t M, int64_t I, const void* dh, int64_t ldh, const void* g, int64_t ldg, const void* u,
                   int64_t ldu, void* dg, int64_t lddg, void* du, int64_t lddu, void* stream);
/* svla_geglu_bwd that also writes the MX e4m3 copy of the [dg | du] row pair -- q [M][ldq >= 2I] bytes (dg in
 * columns 0..I-1, du in I..2I-1) with its E8M0 scales in svla_quant_mx_rows' layout (sld >= 4 M) -- bitwise
 * svla_quant_mx_rows of the bf16 [dg | du] it stores, without reading them back (the fp8 gate|up dgrad operand).
 * I % 128 == 0. */
int svla_geglu_bwd_mx(int64_t M, int64_t I, const void* dh, int64_t ldh, const void* g, int64_t ldg, const void* u,
                      int64_t ldu, void* dg, int64_t lddg, void* du, int64_t lddu, void* q, int64_t ldq, void* scales,
                      int64_t sld, void* stream);
int svla_add_bf16(int64_t n, const void* a, const void* b, void* out, void* stream);
/* GELU pass over a [M][N] bf16 matrix (N % 8 == 0), the rounding points of the fused GEMM epilogues: mode 0
 * y = bf16(gelu_tanh(x)) (SigLIP MLP fc1 activation, transformers SiglipMLP gelu_pytorch_tanh), 1 y = bf16(gelu_erf(x))
 * (BEiT MLP, exact GELU; in place allowed), 2 y = bf16(x * gelu_tanh'(pre)) (the fc1 input gradient, x = dL/dact). */
int svla_gelu_rows(int64_t M, int64_t N, int32_t mode, const void* x, int64_t ldx, const void* pre, int64_t ldp,
                   void* y, int64_t ldy, void* stream);

/* Decode step (M <= 8 token rows, K <= 2560): the two Gemma2 norms between sublayers fused into the next projection,
 * modeling_gemma2.py:487-496 -- h = bf16(res + bf16(rms(y; w1))) (stored to h_out, the new residual stream) and
 * x = bf16(rms(h; w2)), bitwise svla_add_rmsnorm2_fwd -- then C = epi(x @ B^T) as svla_gemm_bf16's small-M path:
 * epi STORE (q|k|v, B KC, segments allowed) or GEGLU (gate|up, two SVLA_SEG_GEGLU segments, out1 = g, out2 = u).
 * res / y / h_out share the row stride ldx. */
int svla_gemv_rmsnorm2(int64_t M, int64_t N, int64_t K, const void* res, const void* y, int64_t ldx, const void* w1,
                       const void* w2, float eps1, float eps2, void* h_out, const svla_operand* B, void* c,
                       int64_t ldc, const svla_epilogue* epi, void* stream);
/* Decode step (M <= 8 token rows), the whole Gemma2 MLP with the norm pair before it in ONE persistent launch
 * (modeling_gemma2.py:91-92, :487-490): h_out = bf16(res + bf16(rms(y; w1))), x = rms(h_out; w2),
 * act = bf16(gelu_tanh(x Wg^T) * (x Wu^T)) [M][I] (caller scratch, row stride ldact), out = act Wd^T [M][H] --
 * bitwise svla_gemv_rmsnorm2 (GEGLU) followed by svla_gemm_bf16's small-M down GEMV.  With attn != NULL the o
 * projection runs first in the same launch: y = attn w_o^T (w_o [H][KO], KO <= 2048; y is then an output), bitwise
 * the small-M GEMV.  H <= 2560, I <= 10240, all multiples of 8; w_gate / w_up [I][H] share ldw, w_down [H][I].
 * `sync` points at svla_decode_mlp_sync_bytes() zeroed bytes, reused by every later call on that stream (the grid
 * barriers' counters return to zero).  The grid is svla_decode_mlp_grid(M, H, I) blocks (occupancy-capped, so an
 * otherwise idle device holds them all at once), launched plainly, or cooperatively with SVLA_DECODE_MLP_COOP=1
 * (dispatched only when every block can be resident; ~21 us more per launch).  A block whose barrier wait hits its
 * bound (1 s: its grid was not co-resident) adds 1 to the 32-bit word 32 of `sync` and writes NaN where it would
 * have written numbers -- callers read that word after a decode and raise. */
size_t svla_decode_mlp_sync_bytes(void);
/* Blocks svla_decode_mlp launches for these sizes (DM_BPC per CU, capped by the occupancy of the instance and its
 * LDS and by I / 4), or 0 when no block fits on a CU: take the two-launch path then. */
int svla_decode_mlp_grid(int64_t M, int64_t H, int64_t I);
/* Test hook: grid_override > 0 launches that many blocks instead of svla_decode_mlp_grid's; cooperative 1 / 0 forces
 * the launch mode (-1: the default); timeout_ms bounds each barrier wait (default 1000).  Not for production use. */
void svla_decode_mlp_debug(int grid_override, int cooperative, int timeout_ms);
int svla_decode_mlp(int64_t M, int64_t H, int64_t I, const void* res, void* y, int64_t ldx, const void* w1,
                    const void* w2, float eps1, float eps2, void* h_out, const void* w_gate, const void* w_up,
                    int64_t ldw, const void* w_down, int64_t ldd, void* act, int64_t ldact, void* out, int64_t ldo,
                    const void* attn, int64_t ld_attn, int64_t KO, const void* w_o, int64_t ldwo, unsigned* sync,
                    void* stream);

/* ------------------------------------------------------------------------------------------
 * Softcapped lm_head cross-entropy (modeling_gemma2.py:993-997 + modeling_spatialvla.py:415-430,
 * action argmax train/monkey_patch.py:267-309).  Logits come from svla_gemm_bf16 with
 * SVLA_EPI_SOFTCAP_CE, which leaves per (row, 128-col tile) {max, sumexp, argmax} in row_stats.
 * ---------------------------------------------------------------------------------------- */
/* The same softcap and row_stats as SVLA_EPI_SOFTCAP_CE, as a streaming pass over raw bf16 logits [M][ld] (N valid
 * columns) written by a plain-store GEMM, in place: logits = bf16(cap*tanh(bf16(bf16(y)/cap))) (the reference's bf16
 * op order, modeling_gemma2.py:993-997), row_stats [M][ceil(N/128)][3] bitwise the epilogue's.  One read and one
 * write of the logits at HBM rate instead of the VALU-heavy epilogue inside the MFMA loop's tiles. */
int svla_softcap_ce_rows(int64_t M, int64_t N, void* logits, int64_t ld, float cap, float* row_stats, void* stream);
/* Reduce row_stats -> lse[m], argmax[m]; loss_rows[m] = lse - logit[m, target[m]] for target >= 0
 * (else 0); loss_out[0] = sum(loss_rows)/max(n_valid,1) where n_valid = #(target >= 0). */
int svla_ce_finalize(int64_t M, int64_t N, int64_t ntiles, const float* row_stats, const void* logits, int64_t ldl,
                     const int64_t* target, float* lse, int64_t* argmax, float* loss_rows, float* loss_out,
                     void* stream);
/* dlogits[m, n] = scale*(softmax(y)[n] - [n==target]) * (1 - (y/cap)^2), y = bf16 logits; rows with
 * target < 0 get 0; columns in [N, ldd) zeroed.  scale = grad_loss / n_valid (device scalar). */
int svla_ce_bwd(int64_t M, int64_t N, const void* logits, int64_t ldl, const float* lse, const int64_t* target,
                float cap, const float* grad_scale, void* dlogits, int64_t ldd, void* stream);
/* Action-token accuracy of one training step (train/monkey_patch.py:267-309): pred [B, >=L-1] int64 argmax ids
 * (row stride ldp; pred[b,t] = argmax of logits[b,t]), labels [B, L] int64 (row stride ldl); gt[b,t] =
 * labels[b,t+1].  ranges: HOST array of 6 inclusive token-id bounds {translation lo, hi, rotation lo, hi,
 * gripper lo, hi}.  counts[8] (device, int64) = {n, correct} for {all action rows, translation, rotation,
 * gripper}; acc[4] (device, fp32) = correct / n per class, computed as torch's float32 division (0/0 -> nan). */
int svla_action_accuracy(int64_t B, int64_t L, const int64_t* pred, int64_t ldp, const int64_t* labels, int64_t ldl,
                         const int64_t* ranges, int64_t* counts, float* acc, void* stream);

/* ------------------------------------------------------------------------------------------
 * Optimizer (DeepSpeed FusedAdam / torch AdamW semantics, scripts/zero1.json:23-34).
 * ---------------------------------------------------------------------------------------- */
/* partial sums of squares of a bf16 vector -> out[0] += sum (single fp32; deterministic tree). */
int svla_sumsq_bf16(int64_t n, const void* x, float* partial, int64_t n_partial, float* out, void* stream);
/* AdamW over a flat shard: g = bf16 grad * clip_scale(device scalar);
 * m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr*(m/bc1 / (sqrt(v/bc2)+eps) + wd*p);
 * master fp32 updated, param_bf16 = bf16(master). */
int svla_adamw(int64_t n, float* master, void* param_bf16, const void* grad_bf16, float* m, float* v, float lr,
               float beta1, float beta2, float eps, float weight_decay, float bc1, float bc2,
               const float* clip_scale, void* stream);
/* clip_scale[0] = min(1, max_norm / (sqrt(sumsq[0]) + 1e-6)); norm_out[0] = sqrt(sumsq[0]). */
int svla_clip_scale(const float* sumsq, float max_norm, float* clip_scale, float* norm_out, void* stream);

/* ZoeDepthAttractorLayerUnnormed bin update (transformers zoedepth [3p], the frozen estimator of
 * model/modeling_spatialvla.py:314-323): out = bf16(c + bf16(sum_i bf16(inv(bf16(A_i - c))) [/ n_att])) with the
 * eager bf16 rounding of each op, inv(dx) = dx / (1 + alpha dx^gamma) in fp32.  Maps [B, C, H, W] by element strides
 * (b, c, y, x); n_bins % 8 == 0. */
int svla_zoe_attractor(int B, int H, int W, int n_att, int n_bins, const void* attractors, const int64_t* a_strides,
                       const void* centres, const int64_t* c_strides, float alpha, int gamma, int mean, void* out,
                       const int64_t* out_strides, void* stream);
/* DPT readout "project" input of the frozen Zoe estimator (transformers ZoeDepthReassembleStage.forward [3p], called
 * from model/modeling_spatialvla.py:314-323): hidden [B, T + 1, C] bf16 (CLS first) -> out [B * T, 2C] with row
 * (b, t) = [hidden(b, 1 + t), hidden(b, 0)] -- the values torch.cat(hidden_states) + permute + torch.cat((tokens,
 * readout), -1) produce, in one pass; C % 8 == 0, 16-B aligned. */
int svla_zoe_readout_cat(int64_t B, int64_t T, int64_t C, const void* hidden, void* out, void* stream);
/* process_zoe (model/modeling_spatialvla.py:99-110) in one pass: out[b,c] = bf16(bf16(bicubic(reflect_pad(x, pad))
 * - mean[c]) / std[c]) at OH x OW, bicubic as torch's upsample_bicubic2d with align_corners=True (A = -0.75, border
 * taps clamped, fp32, one bf16 rounding), TF.normalize's sub and div each rounded to bf16.  x, out bf16 NCHW
 * contiguous; C <= 4; mean/std host arrays of C floats (their bf16 values). */
int svla_zoe_preprocess(int B, int C, int H, int W, int pad, int OH, int OW, const void* x, const float* mean,
                        const float* stdv, void* out, void* stream);
/* The depth resize of model/modeling_spatialvla.py:318-323: out[b] = bicubic(depth[b], size (OH+2pad) x (OW+2pad),
 * align_corners=True)[pad:-pad, pad:-pad], bf16 [B][IH][IW] -> bf16 [B][OH][OW]; only the kept pixels computed. */
int svla_zoe_depth_resize(int B, int IH, int IW, int pad, int OH, int OW, const void* depth, void* out, void* stream);
/* Bilinear resize of a channels-last bf16 map [B, H1, W1, C] -> [B, H2, W2, C] with torch's
 * upsample_bilinear2d semantics (transformers ZoeDepthFeatureFusionLayer.forward interpolate(scale_factor=2,
 * align_corners=True) and the relative head's nn.Upsample, called from modeling_spatialvla.py:317-323's Zoe
 * forward).  rh/rw = torch's area_pixel_compute_scale: (in-1)/(out-1) with align_corners, else 1/scale_factor or
 * in/out.  C multiple of 8, 16-B aligned buffers. */
int svla_upsample_bilinear_nhwc(int B, int C, int H1, int W1, int H2, int W2, int align_corners, float rh, float rw,
                                const void* in, void* out, void* stream);
/* ------------------------------------------------------------------------------------------
 * ZoeDepth metric head tail, fused (frozen depth estimator; reference model/modeling_spatialvla.py:314-323
 * calls transformers ZoeDepthMetricDepthEstimationHead.forward [3p], whose tail after the last attractor is
 * replaced): cat(outconv activation, relative depth) + bilinear(align_corners) bin embedding -> 1x1 conv
 * (+bias) -> GELU(erf) -> 1x1 conv (+bias) -> softplus -> probability / temperature -> log-binomial
 * softmax over NBins -> expectation over bilinear(align_corners) bin centres.  Inputs bf16 with arbitrary
 * element strides (b, c, y, x) / (b, y, x) (channel stride 1 = channels-last, 16-B aligned).  params fp32:
 * W1^T [CF+1+CE][Hid], W2 [4][Hid], b1 [Hid], b2 [4], log_binom(NBins-1, k) [NBins] (as the reference computes
 * it).  out [B, H, W] fp32.  Built for NBins = 64, Hid = 80, CF and CE multiples of 8. */
int svla_zoe_metric_tail(int B, int H, int W, int h, int w, int CF, int CE, int NBins, int Hid,
                         const void* feat, const int64_t* feat_strides, const void* rel, const int64_t* rel_strides,
                         const void* emb, const int64_t* emb_strides, const void* ctr, const int64_t* ctr_strides,
                         const float* params, float p_eps, float max_t, float min_t, float clamp_eps, float* out,
                         void* stream);

/* Convolution on NHWC bf16 maps as an implicit GEMM (csrc/conv.hip): the frozen ZoeDepth DPT neck and depth heads
 * (transformers zoedepth [3p]: ZoeDepthReassembleLayer projection / resize, the neck's 3x3 convs, the
 * PreActResidualLayer pairs, FeatureFusionLayer projections, the relative-depth head), called by the reference at
 * model/modeling_spatialvla.py:314-323.
 *   out[b,oy,ox,co] = post( bf16(sum_{ky,kx,ci} pre(x[b, oy*stride+ky-pad, ox*stride+kx-pad, ci]) w[co,ky,kx,ci]
 *                                + bias[co]) ), then out = bf16(out + res1), then out = bf16(out + res2)
 * pre = ReLU with SVLA_CONV_PRE_RELU (DPT's pre-activation), post = ReLU with SVLA_CONV_POST_RELU; zero padding.
 * w: [Cout][KH][KW][Cin] bf16 (the torch [Cout][Cin][KH][KW] weight permuted once).  x [B,H,W,Cin],
 * out / res1 / res2 [B,OH,OW,Cout], all NHWC and 16-B aligned; Cin and Cout multiples of 8; x under 2 GiB.
 * SVLA_CONV_TRANSPOSED: nn.ConvTranspose2d with kernel == stride == factor, padding 0: w [factor][factor][Cout][Cin],
 * OH = H*factor, each input pixel's output block written once (no residuals, no pre-activation). */
enum { SVLA_CONV_PRE_RELU = 1, SVLA_CONV_POST_RELU = 2, SVLA_CONV_TRANSPOSED = 4 };
typedef struct {
  int32_t B, H, W, Cin;
  int32_t OH, OW, Cout;
  int32_t KH, KW, stride, pad;
  int32_t flags;
  int32_t factor;
  int32_t _pad;
  const void* x;
  const void* w;
  const void* bias;   /* [Cout] bf16 or NULL */
  const void* res1;   /* NULL or [B,OH,OW,Cout] */
  const void* res2;   /* NULL or [B,OH,OW,Cout] */
  void* out;
  /* optional: the caller's svla_gemm_bf16 workspace for this stream (NULL = no split-K).  Grids of 64x64 tiles under
   * one wave (the B = 1 DPT neck) split K over workgroups into its fp32 slabs + arrival counters */
  void* workspace;
  size_t ws_bytes;
} svla_conv_args;
int svla_conv2d_nhwc(const svla_conv_args* a, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SVLA_H_ */

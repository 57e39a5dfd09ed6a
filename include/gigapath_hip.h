/*
 * gigapath_hip.h — C ABI of the MI355X (gfx950) slide-encoder hot path.
 *
 * One shared library, libgigapath_hip.so, built with hipcc --offload-arch=gfx950.
 * Conventions (all entry points):
 *   - extern "C", plain pointers and sizes, no framework types.
 *   - Every tensor pointer is a DEVICE pointer to caller-allocated, contiguous memory;
 *     the library never allocates.  16-bit buffers ("act": bf16 or fp16 per the entry's fmt
 *     argument) are uint16_t bit patterns.
 *   - Work is enqueued on `stream` (a hipStream_t passed as void*; NULL = default stream)
 *     and is stream-ordered; nothing synchronises the host.
 *   - Return value: 0 = ok, GP_EARG (-1) = bad argument, otherwise a hipError_t.
 *     gp_last_error_string() describes the last failure of the calling thread.
 *   - No global mutable state; calls on distinct streams may run concurrently.
 *
 * Each entry cites the reference interface it replaces (paths relative to the reference
 * repository root, qimingfan10/Prov-gigapath-replication).
 */
#ifndef GIGAPATH_HIP_H
#define GIGAPATH_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GP_ABI_VERSION 10
#define GP_EARG (-1)
#define GP_MAX_BRANCHES 8
#define GP_MAX_DESTS 8

/* 16-bit activation format (the `fmt` argument of every entry point with 16-bit activations):
 * bf16 (BASELINE's compute dtype) or fp16 (the reference pipeline's
 * torch.cuda.amp.autocast(dtype=torch.float16), pipeline.py:186-187).  Residual stream, LN
 * parameters, LSEs and readouts stay fp32 in both. */
#define GP_FMT_BF16 0
#define GP_FMT_F16 1
/* fp16, except the V third of a fused [M, 3E] q | k | v buffer, which is bf16 (ABI 8).  Written by
 * gp_linear / gp_linear_ln (output columns [2N/3, N) in bf16) and read by gp_dilated_attn_fwd(_ex) /
 * gp_dilated_attn_fwd_varlen (fp16 S = Q.K^T, bf16 P and P.V, fp16 o): the reference pipeline's fp16
 * autocast caller at the bf16 kernel's speed.  Other entry points take GP_FMT_F16. */
#define GP_FMT_F16_VBF16 2

/* ABI version of the loaded library (== GP_ABI_VERSION). */
int gp_abi_version(void);

/* Human-readable description of the calling thread's last error ("" if none). */
const char* gp_last_error_string(void);

/* Coordinates -> flat pos-embed index, bit-exact with
 * LongNetViT.coords_to_pos (gigapath/slide_encoder.py:166-179):
 *   pos = (int64)(floor(x / tile) * grid + floor(y / tile)) + 1, computed in the coords dtype.
 * coords: [n_tiles, 2] float32 (coords_is_f64 = 0) or float64 (= 1).  pos: [n_tiles] int64.
 * err_count (device int32, may be NULL) is incremented once per index outside the
 * [-(grid*grid+1), grid*grid] range torch indexing of pos_embed accepts (slide_encoder.py:200). */
int gp_coords_to_pos(const void* coords, int coords_is_f64, int64_t n_tiles, int grid,
                     double tile_size, int64_t* pos, int32_t* err_count, void* stream);

/* Patch-embed epilogue + 2-D sin-cos position add + CLS concat (slide_encoder.py:195-205,
 * pos_embed.py:30-77) fused with the first pre-LN (encoder.py:126).
 *   x_out[b, 0, :]   = cls                                  (pos_embed row 0 is zero)
 *   x_out[b, 1+t, :] = xp[b, t, :] + [tab[(p-1) % G] | tab[(p-1) / G]],  p = pos[b, t]
 *   ln_out           = LayerNorm(x_out; ln_w, ln_b, eps)    (skipped if ln_w == NULL)
 *   row_mean[row]    = mean of x_out's row                  (skipped if row_mean == NULL: the shift of
 *                                                             the first gp_linear_resid)
 * xp: [B, N, E] act (patch projection incl. bias); tab: [G, E/2] fp32 one-axis sin-cos
 * table (fp64-built); cls: [E] fp32; x_out: [B, N+1, E] fp32; ln_out: [B, N+1, E] act.
 * cls == NULL: no CLS row (a sequence-parallel shard that does not hold token 0):
 *   x_out[b, t, :] = xp[b, t, :] + pos row, t < N  (x_out, ln_out: [B, N, E]).
 * E must be 64 * {12, 16, 24}. */
int gp_posembed_cls_ln(const uint16_t* xp, const int64_t* pos, const float* tab, const float* cls,
                       int64_t B, int64_t N, int E, int G, const float* ln_w, const float* ln_b,
                       float eps, float* x_out, uint16_t* ln_out, float* row_mean, int fmt, void* stream);

/* Dilated sparsify of one branch (DilatedAttention.gathering / dense_to_sparse,
 * torchscale/component/dilated_attention.py:16-31, 76-98), bit-exact:
 *   dst[((b*nseg + n)*H + h)*m + i, :] = src[b*L + n*s + i*r + h/(Hp/r), col_off + h*D + :]
 *   or zeros where the reference pads (i*r + j >= s, or the token >= L).
 * s = min(sl, L), nseg = ceil(L/s), m = ceil(s/r), Hp = H rounded up to a multiple of r.
 * src: [B*L, row_stride] 16-bit; dst: [B*nseg*H*m, D] same (a copy: any 16-bit format).  D % 8 == 0. */
int gp_dilated_gather(const uint16_t* src, int64_t row_stride, int64_t col_off, int64_t B, int64_t L,
                      int H, int D, int sl, int r, uint16_t* dst, void* stream);

/* All dilation branches of one DilatedAttention layer in ONE launch: the dilated gather is
 * folded into the attention addressing, and zero-padded keys are added analytically
 * (replaces gathering x3 + flash_attn_func per branch: dilated_attention.py:199-208,
 * multihead_attention.py:97-107, flash_attention.py:13-16).
 * q/k/v: [B*L, row_stride] act (head h at columns h*D .. h*D+D-1 of each pointer; a fused
 *   QKV buffer passes q = base, k = base + E, v = base + 2E, row_stride = 3E).
 * Branch b (sl = seg_len[b], r = ratios[b]) writes
 *   o_out[b]:   [B*nseg_b, m_b, H, D] act    (flash_attn's "out" layout per segment)
 *   lse_out[b]: [B*nseg_b, H, m_b]    fp32   (natural-log LSE, flash_attn's softmax_lse)
 * Rows whose values the merge can never read (beyond the last segment's tokens) are left
 * unwritten.  softmax_scale <= 0 selects D^-0.5.  D in {48, 64, 96}.
 * q_log2_prescaled != 0: the caller already multiplied q by softmax_scale*log2(e) (e.g. folded
 * into the Q projection), softmax_scale is ignored and scores are used as log2-domain logits
 * (D in {48, 64}); outputs keep the same meaning (lse stays natural-log). */
int gp_dilated_attn_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, int64_t row_stride,
                        int64_t B, int64_t L, int H, int D, const int32_t* seg_len,
                        const int32_t* ratios, int nbranch, uint16_t* const* o_out,
                        float* const* lse_out, float softmax_scale, int q_log2_prescaled,
                        int fmt, void* stream);

/* One branch of gp_dilated_attn_fwd_ex: where its keys/values live and where its outputs go. */
typedef struct GpAttnBranch {
  int32_t seg_len;           /* sl (segment length before min(sl, L)) */
  int32_t ratio;             /* r  (dilation ratio) */
  const uint16_t* k;         /* key rows: token t of batch b is row (b*L + t - kv_tok_base) */
  const uint16_t* v;         /* value rows, same indexing */
  int64_t kv_row_stride;     /* elements between consecutive rows */
  int64_t kv_tok_base;       /* token index held by row 0 */
  int32_t kv_sparse_cols;    /* 0: head h at columns h*D (dense projection rows);
                                1: head h at columns (h % (H/r))*D (token-major sparsified rows
                                   written by gp_dilated_sparsify, where K is at column 0 and V at
                                   column (H/r)*D of each row; pass v = k + (H/r)*D) */
  uint16_t* o;               /* [B*nseg, m, H, D] act */
  float* lse;                /* [B*nseg, H, m] fp32 */
  int32_t key_part;          /* ABI 10: key_parts > 1 -- this entry attends to key part key_part of key_parts
                                (the segment's key tiles split evenly; the reference's zero-pad keys go to
                                the last part): o / lse are the softmax over those keys only, and the merge
                                combines the parts as branches (gp_branch_merge_ln* with the entry repeated
                                per part).  An empty part writes o = 0, lse = -inf.  0 / <= 1: all keys.
                                Needs the LDS-DMA pair (D = 48, q_log2_prescaled, k / v in one row layout,
                                fmt BF16 or F16_VBF16) and 0 <= key_part < key_parts <= 64. */
  int32_t key_parts;
} GpAttnBranch;

/* Generalised gp_dilated_attn_fwd: per-branch K/V sources and a query window.  Computes, for
 * every branch, the sparse rows whose sparse_to_dense slot n*g + i*r + j (g = m*r,
 * dilated_attention.py:33-53) lies in [win_lo, win_hi) of each batch's sequence -- exactly the
 * rows gp_branch_merge_ln_window reads for tokens [win_lo, win_hi).  The sequence-parallel
 * shard of one rank passes its own token range; win = [0, L) is the single-device forward.
 * q: token t of batch b at row (b*L + t - q_tok_base), row stride q_row_stride, head h at
 * columns h*D.  Keys of a segment are rows n*s + i*r + j for every valid i (all of the segment),
 * so each branch's k/v rows must cover the gather range of every segment the window meets. */
int gp_dilated_attn_fwd_ex(const uint16_t* q, int64_t q_row_stride, int64_t q_tok_base, int64_t B,
                           int64_t L, int H, int D, int64_t win_lo, int64_t win_hi,
                           const GpAttnBranch* branches, int nbranch, float softmax_scale,
                           int q_log2_prescaled, int fmt, void* stream);

/* The attention launch plan's build constants, for host-side planners that size work against it
 * (gigapath/seqpar.py's key-part rule; no reference counterpart -- the reference has no launch plan):
 * params[0] = query rows per 8-wave LDS-DMA work item (256), params[1] = such workgroups resident per
 * CU (3), params[2] = 8-wave items per CU below which a launch counts as under-filled and runs 4-wave
 * workgroups (3; 0 when that switch is built off), params[3] = largest key_parts (64).  n: entries of
 * params (at most 4 are written).  Host only, no device work. */
int gp_attn_launch_params(int32_t* params, int n);

/* Token-major sparsified K/V rows for sequence parallelism (one rank's share of
 * DilatedAttention.gathering, dilated_attention.py:16-31,76-98).  For tokens
 * p in [tok_lo, tok_lo + n_tok) (rows of src, first row = tok_lo) and branch b with
 * s = min(sl, L), j = (p % s) % r, C = (H/r)*D:
 *   dst[b][p - base_b, 0:C]  = src[p - tok_lo, k_col + j*C : k_col + (j+1)*C]
 *   dst[b][p - base_b, C:2C] = src[p - tok_lo, v_col + j*C : v_col + (j+1)*C]
 * dst[b]: [rows, 2C] 16-bit (a copy of src's format) whose row 0 holds token base_b = dst_tok_base[b] (NULL: all 0,
 * i.e. full-length [L, 2C] buffers); base_b <= tok_lo.  B = 1.  H % r == 0 for every branch. */
int gp_dilated_sparsify(const uint16_t* src, int64_t src_row_stride, int64_t k_col, int64_t v_col,
                        int64_t tok_lo, int64_t n_tok, int64_t L, int H, int D, const int32_t* seg_len,
                        const int32_t* ratios, int nbranch, uint16_t* const* dst,
                        const int64_t* dst_tok_base, void* stream);

/* One destination of gp_dilated_sparsify_dests: tokens [tok_lo, tok_hi) of a branch, token p
 * written at dst + (p - tok_lo) * 2C (a peer's chunk of an all-to-all send buffer). */
typedef struct GpRowDest {
  int64_t tok_lo;
  int64_t tok_hi;
  uint16_t* dst;
} GpRowDest;

/* gp_dilated_sparsify writing each token's branch row to every destination whose range holds it
 * (up to GP_MAX_DESTS per branch): the sequence-parallel send buffers, packed per peer, in one
 * pass.  dests: [nbranch * GP_MAX_DESTS] (branch b's entries at b*GP_MAX_DESTS ..), ndest:
 * [nbranch] entries used per branch. */
int gp_dilated_sparsify_dests(const uint16_t* src, int64_t src_row_stride, int64_t k_col, int64_t v_col,
                              int64_t tok_lo, int64_t n_tok, int64_t L, int H, int D, const int32_t* seg_len,
                              const int32_t* ratios, int nbranch, const GpRowDest* dests,
                              const int32_t* ndest, void* stream);

/* Drop-in for the operator seam flash_attn_func(q, k, v, 0.0, None, scale, False)
 * (torchscale/component/flash_attention.py:13-16): non-causal, no mask, dropout 0.
 * q/k/v/o: [nbatch, seqlen, H, D] bf16 contiguous; lse: [nbatch, H, seqlen] fp32. */
int gp_seg_attn_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, int64_t nbatch,
                    int64_t seqlen, int H, int D, float softmax_scale, uint16_t* o, float* lse,
                    void* stream);

/* The same seam for fp16 q / k / v / o (the reference pipeline runs the encoder under
 * torch.cuda.amp.autocast(dtype=torch.float16), pipeline.py:186-187, so flash-attn receives fp16
 * tensors and computes in fp16: P rounded to fp16, fp32 accumulation).  Exact running-max kernel
 * with f16 MFMAs (v_mfma_f32_32x32x16_f16 / 16x16x32_f16); D in {48, 64, 96}. */
int gp_seg_attn_fwd_f16(const uint16_t* q, const uint16_t* k, const uint16_t* v, int64_t nbatch,
                        int64_t seqlen, int H, int D, float softmax_scale, uint16_t* o, float* lse,
                        void* stream);

/* Branch merge (DilatedAttention.scattering / sparse_to_dense, dilated_attention.py:33-53,
 * 100-131) fused with inner_attn_ln (:212-213):
 *   per (token p, head h): lse_b = covered ? lse_b[..] : -1e8, lse_b == 0 -> -1e8,
 *   w_b = softmax_b(lse_b) in fp32, out = sum_b w_b * o_b, then LayerNorm over H*D
 *   (skipped if ln_w == NULL).  Inputs are gp_dilated_attn_fwd's outputs.
 * out: [B*L, H*D] act (the o_in format). */
int gp_branch_merge_ln(const uint16_t* const* o_in, const float* const* lse_in,
                       const int32_t* seg_len, const int32_t* ratios, int nbranch, int64_t B,
                       int64_t L, int H, int D, const float* ln_w, const float* ln_b, float eps,
                       uint16_t* out, int fmt, void* stream);

/* gp_branch_merge_ln restricted to tokens [tok_lo, tok_lo + n_tok) of each batch (a
 * sequence-parallel shard): out row b*n_tok + (p - tok_lo).  Reads only the branch rows
 * gp_dilated_attn_fwd_ex computed for the same window. */
int gp_branch_merge_ln_window(const uint16_t* const* o_in, const float* const* lse_in,
                              const int32_t* seg_len, const int32_t* ratios, int nbranch, int64_t B,
                              int64_t L, int64_t tok_lo, int64_t n_tok, int H, int D, const float* ln_w,
                              const float* ln_b, float eps, uint16_t* out, int fmt, void* stream);

/* ---- Varlen packing (config C5, SURVEY §8e: "concatenate slides with per-slide segment
 * tables, no cross-slide attention").  nslide slides packed token-major in one qkv buffer
 * [T, qkv_row_stride] (slide i at rows [tok_off[i], tok_off[i] + L[i]), q | k | v at columns
 * 0, H*D, 2*H*D), each with its OWN segment schedule s = min(sl, L[i]) -- the reference's
 * per-slide B = 1 forward (slide_encoder.py:181-223), batched into one launch per layer.
 * Replaces: one gp_dilated_attn_fwd / gp_branch_merge_ln pair per slide.
 *
 * gp_varlen_plan_bytes: size of the host plan buffer.
 * gp_varlen_plan: with plan_host == NULL, only writes o_elems[b] / lse_elems[b] (elements of the
 *   packed per-branch output buffers the caller allocates: slide-major [nseg_ib, m_ib, H, D] and
 *   [nseg_ib, H, m_ib] regions).  Otherwise also fills plan_host with the work table (device
 *   pointers into qkv / o / lse, not dereferenced here); the caller copies the plan_bytes to a
 *   16-byte aligned device buffer (plan_dev) that stays alive while launches use it.
 * gp_dilated_attn_fwd_varlen: every slide's five-branch attention in one launch (D = 48,
 *   q pre-scaled by D^-1/2 * log2 e).
 * gp_branch_merge_ln_varlen: every packed token's LSE merge + inner LN (E = 768, D = 48);
 *   out: [T, E] act (the plan's qkv format), row = packed token. */
int64_t gp_varlen_plan_bytes(int nslide, int nbranch);
int gp_varlen_plan(const int64_t* L, int nslide, int H, int D, const int32_t* seg_len,
                   const int32_t* ratios, int nbranch, const uint16_t* qkv, int64_t qkv_row_stride,
                   uint16_t* const* o_out, float* const* lse_out, void* plan_host, int64_t plan_bytes,
                   int64_t* o_elems, int64_t* lse_elems);
int gp_dilated_attn_fwd_varlen(const void* plan_host, const void* plan_dev, int q_log2_prescaled,
                               int fmt, void* stream);
int gp_branch_merge_ln_varlen(const void* plan_host, const void* plan_dev, const float* ln_w,
                              const float* ln_b, float eps, uint16_t* out, int fmt, void* stream);

/* Residual add fused with the next pre-LN (encoder.py:141,147 / :159,126):
 *   x += y + bias (fp32 residual stream, in place);  ln_out = LayerNorm(x) (skipped if ln_w == NULL).
 * x: [rows, cols] fp32; y: [rows, cols] act (GEMM output without bias); bias: [cols] fp32 or NULL;
 * ln_out: [rows, cols] act.  cols = 64 * {12, 16, 24}. */
int gp_residual_layernorm(float* x, const uint16_t* y, const float* bias, const float* ln_w,
                          const float* ln_b, float eps, uint16_t* ln_out, int64_t rows, int cols,
                          int fmt, void* stream);

/* One encoder layer's two residual adds (encoder.py:141, 159) without the mid-layer store of the fp32
 * residual stream (round 6).  y2 == NULL: x1 = x + (y1 + b1), ln_out = LayerNorm(x1) (ln_w required),
 * x left unchanged.  y2 != NULL: x = (x + (y1 + b1)) + (y2 + b2), ln_out = LayerNorm(new x) when ln_w
 * != NULL.  x1 is rounded exactly as gp_residual_layernorm rounds it, so the pair equals two
 * gp_residual_layernorm calls bit for bit while moving 22 instead of 24 bytes per element.  y1 / y2:
 * [rows, cols] act GEMM outputs without bias; b1 / b2: [cols] fp32 or NULL. */
int gp_residual2_layernorm(float* x, const uint16_t* y1, const float* b1, const uint16_t* y2, const float* b2,
                           const float* ln_w, const float* ln_b, float eps, uint16_t* ln_out, int64_t rows,
                           int cols, int fmt, void* stream);

/* FFN middle (feedforward_network.py:131-137): out = LayerNorm(gelu_erf(h)) in fp32.
 * h, out: [rows, cols] act (in place allowed); cols = 64 * {48, 64, 96}.  GELU is rounded to act
 * before the LN (gelu(x.float()).type_as(x), feedforward_network.py:135). */
int gp_gelu_layernorm(const uint16_t* h, const float* ln_w, const float* ln_b, float eps,
                      uint16_t* out, int64_t rows, int cols, int fmt, void* stream);

/* ---- Projection GEMMs on MFMAs (nn.Linear of torchscale/component/multihead_attention.py:43-48,
 * feedforward_network.py:131-142, gigapath/slide_encoder.py:47-51).  A [M, K] and W [N, K] are
 * K-contiguous act (row strides lda / ldw), C [M, N] act (ldc); fp32 accumulation.  N % 256 == 0;
 * strides multiples of 8, operands 16-byte aligned.
 * ws: device workspace of gp_gemm_workspace_bytes(M, N, K) bytes (fp32 partials of the last, split
 * round of tiles; the value depends on the current device's CU count); NULL disables the split.
 * (ABI 7: N any multiple of 256, K in {768, 1024, 1536, 3072, 4096, 6144} -- the three registered
 * archs, slide_encoder.py:261-270.) */
int64_t gp_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K);

/* C = A . W^T (+ bias).  bias: [N] fp32 or NULL. */
int gp_linear(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const float* bias,
              uint16_t* C, int64_t ldc, int64_t M, int64_t N, int64_t K, void* ws, int64_t ws_bytes,
              int fmt, void* stream);

/* FFN first half (feedforward_network.py:131-135): fc1 with the GELU in its epilogue,
 *   h = act(gelu(act(A . W1^T + b1)))     (gelu(x.float()).type_as(x), exact erf; for bf16 h is
 *                                          torch's CPU F.gelu bit for bit, a table of the 16-bit inputs)
 * and the LayerNorm statistics of h per 256-column group g:
 *   stats[g][m] = (mean, sum of squared deviations) of h[m, 256 g : 256 g + 256]   (fp32 pairs)
 * A: [M, K] act; W1: [F, K] act; b1: [F] fp32 or NULL; h: [M, F] act (ldh); stats: [F/256 + 1, M, 2]
 * fp32 (the last plane is gp_ffn_fc2_ln's).  F % 256 == 0. */
int gp_ffn_fc1_gelu(const uint16_t* A, int64_t lda, const uint16_t* W1, int64_t ldw, const float* b1,
                    uint16_t* h, int64_t ldh, float* stats, int64_t M, int64_t F, int64_t K, int fmt,
                    void* stream);

/* FFN second half (feedforward_network.py:136-142): fc2(ffn_layernorm(h)) with the LayerNorm folded
 * into the GEMM epilogue:
 *   y = act( rstd_m * (h . W2g^T - mean_m * c) + d )
 * mean_m / rstd_m = LayerNorm statistics of row m merged from gp_ffn_fc1_gelu's stats (biased
 * variance, + eps; written into the stats' last plane first); W2g [N, F] act = W2 * gamma (each column
 * k scaled by the LN weight); c [N] fp32 = row sums of W2g (as rounded); d [N] fp32 = W2 . beta + b2.
 */
int gp_ffn_fc2_ln(const uint16_t* h, int64_t ldh, const uint16_t* W2g, int64_t ldw, float* stats,
                  const float* c, const float* d, float eps, uint16_t* y, int64_t ldy, int64_t M, int64_t N,
                  int64_t F, void* ws, int64_t ws_bytes, int fmt, void* stream);

/* ---- The residual stream inside the GEMMs (ABI 7).  EncoderLayer.forward's residual adds and the pre-LNs
 * that follow them (encoder.py:141,147 -> final_layer_norm; :159 -> the next layer's self_attn_layer_norm
 * at :126) without a separate pass: the producing GEMM (out-proj, fc2) adds its output into the fp32
 * residual stream x and writes the next LayerNorm's input as
 *   xb = act(gamma * (x - s))   (s [M] = a per-row shift: the row's mean of x BEFORE the add, so the 16-bit
 *                                rounding sees a nearly centred row; gamma = that LayerNorm's weight)
 * with (mean, M2) of x - s per 256-column group; the consuming GEMM (QKV, fc1) folds the LayerNorm:
 *   LN(x) . W^T + b = rstd * (xb . W^T - mean' c) + d,  c = W . gamma (fp32), d = W . beta + b,
 * mean' / rstd of x - s merged from the groups (the merge also writes s_out = s_in + mean' = the row's
 * mean of x, the next producer's shift).  The reference rounds LN(x) to act before the GEMM; here
 * gamma * (x - s) is rounded instead. */

/* out-proj + residual (multihead_attention.py:48 + encoder.py:141,147):
 *   x += A . W^T + bias  (fp32, in place; x [M, ldx]);  xb [M, ldxb] act, xstats [N/256, M, 2] fp32 as above.
 * gamma == NULL: no xb / xstats (x only).  shift: [M] fp32.
 * s_out != NULL (ABI 9): also merge the N/256 planes into plane N/256 of xstats ([N/256 + 1, M, 2]: mean, rstd
 * with eps_next) and write s_out = shift + the row mean -- the merge the consuming gp_linear_ln /
 * gp_ffn_fc1_gelu_ln would do; call those with nst < 0 then.  With a split-K tail the reduce launch does it
 * (no extra launch); otherwise one merge launch follows the GEMM.  Needs gamma, eps_next > 0, N <= 2048. */
int gp_linear_resid(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, const float* bias,
                    float* x, int64_t ldx, const float* shift, const float* gamma, uint16_t* xb,
                    int64_t ldxb, float* xstats, float eps_next, float* s_out, int64_t M, int64_t N, int64_t K,
                    void* ws, int64_t ws_bytes, int fmt, void* stream);

/* QKV with the pre-LN folded (encoder.py:126 + multihead_attention.py:43-45): merges stats planes
 * 0 .. nst-1 ([nst + 1, M, 2] fp32, gp_linear_resid / gp_ffn_fc2_ln_resid's xstats) into plane nst
 * (mean', rstd; s_out = s_in + mean' when s_out != NULL), then C = act(rstd (A . W^T - mean' c) + d).
 * nst < 0 (ABI 9): plane -nst is already merged (the producer's s_out); no merge here. */
int gp_linear_ln(const uint16_t* A, int64_t lda, const uint16_t* W, int64_t ldw, float* stats, int nst,
                 const float* c, const float* d, float eps, const float* s_in, float* s_out, uint16_t* C,
                 int64_t ldc, int64_t M, int64_t N, int64_t K, void* ws, int64_t ws_bytes, int fmt,
                 void* stream);

/* fc1 + GELU with final_layer_norm folded (encoder.py:147-150 + feedforward_network.py:131-135): the fold
 * of gp_linear_ln (nst < 0: merged by the producer, as there), then gp_ffn_fc1_gelu's GELU and hstats
 * ([F/256 + 1, M, 2]).  No F limit. */
int gp_ffn_fc1_gelu_ln(const uint16_t* A, int64_t lda, const uint16_t* W1, int64_t ldw, float* xstats,
                       int nst, const float* c1, const float* d1, float eps, const float* s_in, float* s_out,
                       uint16_t* h, int64_t ldh, float* hstats, int64_t M, int64_t F, int64_t K, int fmt,
                       void* stream);

/* fc2 with ffn_layernorm folded (gp_ffn_fc2_ln) + residual (encoder.py:157-159): x += fc2(LN(h)),
 * xb / xstats for the next layer's pre-LN as gp_linear_resid (gamma == NULL: the last layer, x only;
 * eps_next / s_out: the next LN's statistics merge, as gp_linear_resid). */
int gp_ffn_fc2_ln_resid(const uint16_t* h, int64_t ldh, const uint16_t* W2g, int64_t ldw, float* hstats,
                        const float* c, const float* d, float eps, float* x, int64_t ldx, const float* shift,
                        const float* gamma, uint16_t* xb, int64_t ldxb, float* xstats, float eps_next,
                        float* s_out, int64_t M, int64_t N, int64_t F, void* ws, int64_t ws_bytes, int fmt,
                        void* stream);

/* Plain fp32 LayerNorm over rows with a row stride (readout: encoder.py:387-388,
 * slide_encoder.py:213-221).  out: [rows, cols] fp32 contiguous.  cols = 64 * {12, 16, 24}. */
int gp_layernorm_f32(const float* x, int64_t row_stride, const float* ln_w, const float* ln_b,
                     float eps, float* out, int64_t rows, int cols, void* stream);

/* Global average pool (slide_encoder.py:215): out[b, :] = mean_{t >= start} x[b, t, :].
 * x: [B, L, E] fp32; out: [B, E] fp32. */
int gp_mean_tokens(const float* x, int64_t B, int64_t L, int E, int64_t start, float* out,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GIGAPATH_HIP_H */

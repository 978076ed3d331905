/*
 * codonlm_hip.h -- C-ABI of the MI355X-native codon-LM hot path (libcodonlm_hip.so).
 *
 * The reference (AvishaiBarnoy/genomics-lm) is pure PyTorch: its "boundary" is the
 * nn.Module API of src/codonlm/model_tiny_gpt.py and the op calls inside it.  Every
 * entry point below replaces one such call site (cited per function), with plain
 * pointers + sizes, no torch types.  All functions are stream-ordered on the
 * caller's hipStream_t (passed as void*), never allocate, never synchronise, and
 * return CG_OK (0) or a negative cg_status.  Buffers are caller-owned device memory.
 *
 * dtype codes: CG_F32 = fp32 storage/compute (parity mode), CG_BF16 = bf16 storage
 * with fp32 accumulation (throughput mode), CG_BF16X2 = split bf16 (a value v stored as
 * hi = bf16(v) and lo = bf16(v - hi) in the two halves of a row: [hi(ldd/2) | lo(ldd/2)]),
 * accepted where noted (gradient operands whose later sums cancel).
 */
#ifndef CODONLM_HIP_H
#define CODONLM_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { CG_F32 = 0, CG_BF16 = 1, CG_BF16X2 = 2 };
enum { CG_OK = 0, CG_EINVAL = -1, CG_EUNSUPPORTED = -2, CG_ELAUNCH = -3 };

/* GEMM epilogue flags (bit set) */
enum {
  CG_EPI_BIAS = 1,       /* + bias[n] (fp32)                                           */
  CG_EPI_GELU = 2,       /* out = gelu(v); aux_out (dtype of C) receives v (pre-act)   */
  CG_EPI_DGELU = 4,      /* out = v * gelu'(aux[m,n]) (aux in dtype of C)              */
  CG_EPI_RESID = 8,      /* out = resid[m,n] + v   (resid fp32, may alias C)           */
  CG_EPI_DROPOUT = 16,   /* v = v * keep(seed, m, n) / (1-p) before RESID              */
  CG_EPI_ACCUM = 32,     /* out (fp32) += v                                            */
  CG_EPI_COLSUM = 64,    /* also column sums of the final values into `workspace` as    */
                         /* [ceil(M/64)][N] fp32 partials (reduce: cg_colsum_reduce) --  */
                         /* a fused bias gradient; needs split_k == 1                     */
  /* SwiGLU (model_tiny_gpt.py:47-57), bf16 persistent tile only (else CG_EUNSUPPORTED): */
  CG_EPI_SWIGLU = 128,   /* B = [w_gate; w_up] (2N rows): aux_out [M][2N] receives the  */
                         /* pre-activations g|u, C [M][N] = silu(g) * u (0 for n >= n_valid) */
  CG_EPI_DSWIGLU = 256,  /* v = dL/ds; aux = g|u [M][2N]: C [M][2N] = d(g|u)             */
                         /* (0 for n >= n_valid)                                         */
  CG_EPI_GELU_DERIV = 512, /* modifies GELU / DGELU: the forward's aux_out receives gelu'(v) */
                         /* instead of v, and the backward's aux holds gelu' (out = v*aux): */
                         /* the derivative is formed once, from the unrounded pre-activation */
  CG_EPI_ROPE = 1024     /* (with or without BIAS) rotate-half RoPE of the q / k heads after */
                         /* the bias (model_tiny_gpt.py:91-93): columns [0, rope_heads*rope_hd) */
                         /* of row m rotated at position m % rope_T by the rope_cos / rope_sin */
                         /* [>= rope_T][rope_hd/2] tables (16-B aligned); bf16 in / out, the */
                         /* loader-wave persistent tile only (else CG_EUNSUPPORTED); rope_hd */
                         /* % 16 == 0 and N % 16 == 0                                   */
};

/*
 * C[m,n] = epilogue( alpha * sum_k A(m,k) * B(n,k) )
 *   A(m,k) = a_kcontig ? A[m*lda + k] : A[k*lda + m]
 *   B(n,k) = b_kcontig ? B[n*ldb + k] : B[k*ldb + n]
 * Replaces nn.Linear / matmul call sites of model_tiny_gpt.py:85-93,132,143-148,50-57,327
 * and their autograd (dX = dY W, dW = dY^T X).  Inputs are `in_dtype`; C is c_dtype.
 * Contiguous extents must be multiples of 8 and leading dims multiples of 8 elements.
 * split_k > 1 needs `workspace` of split_k*M*N floats (dW GEMMs); CG_EPI_COLSUM needs
 * ceil(M/64)*N floats.  ws_bytes is the workspace's size: a short one is CG_EINVAL.
 */
typedef struct {
  int in_dtype, c_dtype;
  int M, N, K;
  const void* A; long long lda; int a_kcontig;
  const void* B; long long ldb; int b_kcontig;
  void* C; long long ldc;
  int epilogue;
  float alpha;
  const float* bias;
  const float* resid; long long ldr;
  const void* aux; void* aux_out; long long ld_aux;
  uint32_t drop_seed; float drop_p;
  int split_k; float* workspace;
  int n_valid; /* SWIGLU / DSWIGLU: columns < n_valid are live (0 = all N) */
  size_t ws_bytes; /* bytes at `workspace` */
  /* CG_EPI_ROPE (ABI 0.3): tables and geometry */
  const float* rope_cos; const float* rope_sin;
  int rope_T, rope_hd, rope_heads;
  /* ABI 0.4: kernel choice per call (the library holds no mutable process-wide settings).
   * tile: CG_TILE_AUTO (0, what the engine uses) or a forced bf16 kernel for tests / A/B runs
   * (CG_EUNSUPPORTED where it cannot run the product); max_wg: cap on the persistent grid
   * (0 = one workgroup per CU; N > 0 = at most N workgroups, each walking more tiles). */
  int tile, max_wg;
} cg_gemm_desc;
enum {
  CG_TILE_AUTO = 0,    /* persistent 256x128 (loader-wave variant where measured faster), else    */
                       /* 256x128 LDS-DMA tile for large K-contiguous products, else 128x128      */
  CG_TILE_VEC = 1,     /* 128x128 register-staged tile                                           */
  CG_TILE_WIDE = 2,    /* 256x128 LDS-DMA tile, one tile per workgroup                           */
  CG_TILE_PERS = 3,    /* persistent 256x128, 8 waves issuing their own LDS-DMA (gemm_pers.h)    */
  CG_TILE_PERS_LW = 4  /* persistent 256x128 with 4 dedicated loader waves (gemm_lw.h)           */
};
int cg_gemm(const cg_gemm_desc* d, void* stream);
/* the CU count the persistent launches (and the dW planner) spread over */
int cg_pers_cus(void);

/* Grouped weight-gradient GEMM: for every product p of the group
 *   C_p[n][k] (+)= alpha_p * sum_{m < K} A_p[m*lda_p + n] * B_p[m*ldb_p + k]
 * (dW = dY^T X of the nn.Linear call sites, A = dY and B = X both token-major bf16, C fp32).
 * Each output tile is reduced over all K rows inside one workgroup (no split-K partials);
 * the tiles of all products form one persistent launch (tile_m codes: 128 = 128x128 (0 = this),
 * 129 = the same with a 5-stage ring, 256 = 256x128, 512 = 256x256).  Any K >= 1 (a ragged last 64-row k-step is zero-filled);
 * N_out, K_out, lda, ldb % 8 == 0; ldc % 4. */
#define CG_DW_MAX 32
typedef struct {
  const void* A; long long lda;
  const void* B; long long ldb;
  float* C; long long ldc;
  int N_out, K_out;
  float alpha; int accumulate;
  float* col_sum;  /* ABI 0.5, optional: [N_out] fp32 (+)= alpha * sum_m A_p[m][n] (the bias gradient */
                   /* of the nn.Linear whose output gradient A_p is), from the A fragments the tiles  */
                   /* already stream; NULL = none; needs ksplit <= 1 (else CG_EUNSUPPORTED)           */
} cg_dw_product;
typedef struct {
  int n, K, tile_m;
  cg_dw_product p[CG_DW_MAX];
  /* ABI 0.3: ksplit > 1 (<= 8) splits every tile's token range over ksplit workgroups (more work
   * items where a group's tiles do not fill the CUs); slices 1.. write fp32 slabs into workspace
   * (ws_bytes >= cg_gemm_dw_grouped_workspace(grp), 16-B aligned, else CG_EINVAL) and one
   * reduction launch adds them into C in slice order -- deterministic.  0 / 1 = no split. */
  int ksplit;
  float* workspace; size_t ws_bytes;
  int max_wg; /* ABI 0.4: grid cap (0 = one workgroup per CU) */
} cg_dw_group;
int cg_gemm_dw_grouped(const cg_dw_group* grp, void* stream);
size_t cg_gemm_dw_grouped_workspace(const cg_dw_group* grp);
/* tiles one product contributes at tile_m */
int cg_gemm_dw_tiles(int tile_m, int N_out, int K_out);

/* LayerNorm (nn.LayerNorm, biased var, eps) -- model_tiny_gpt.py:137,139,216 */
int cg_layernorm_fwd(int out_dtype, const float* x, long long ldx, const float* gamma,
                     const float* beta, void* y, long long ldy, float* mean, float* rstd,
                     int rows, int cols, float eps, void* stream);
/* ABI 0.5: cg_layernorm_fwd and cg_attn_drop_mask(B, T, H, drop_seed, drop_p, mask) in one launch
 * (the LayerNorm of a block's input is HBM-bound, the keep words of the same block's attention
 * dropout VALU-bound: their workgroups alternate in one grid and run side by side).  Results are
 * those of the two calls, bit for bit; drop_p in (0, 1) and mask non-NULL (else CG_EINVAL). */
int cg_layernorm_fwd_mask(int out_dtype, const float* x, long long ldx, const float* gamma,
                          const float* beta, void* y, long long ldy, float* mean, float* rstd,
                          int rows, int cols, float eps, int B, int T, int H, uint32_t drop_seed,
                          float drop_p, void* mask, void* stream);
/* dx = LN backward(dy) [+ g_in]; writes g_out (fp32) and optionally g_out_t (out_dtype,
 * optionally multiplied by a dropout keep mask (seed,p) for the consumer branch);
 * per-block column partials for dgamma/dbeta go to `partials` [nblk][2*cols]
 * (nblk = cg_layernorm_bwd_blocks(rows)), reduced into dgamma/dbeta (accumulate flag).
 * dcolsum (optional, needs g_out_t): column sums of g_out_t before rounding = the bias
 * gradient of the Linear that produced the branch g_out_t feeds (partials then [nblk][3*cols]).
 * partials_bytes: the partials buffer's size, at least cg_layernorm_bwd_workspace(rows, cols,
 * want_col = dcolsum != NULL), else CG_EINVAL.  g_in may equal g_out (in-place accumulation). */
int cg_layernorm_bwd_blocks(int rows);
size_t cg_layernorm_bwd_workspace(int rows, int cols, int want_col);
int cg_layernorm_bwd(int dy_dtype, const void* dy, long long lddy, const float* x, long long ldx,
                     const float* mean, const float* rstd, const float* gamma,
                     const float* g_in, float* g_out, int out_dtype, void* g_out_t,
                     uint32_t drop_seed, float drop_p, float* partials, size_t partials_bytes,
                     float* dgamma, float* dbeta, float* dcolsum, int accumulate, int rows, int cols,
                     float eps, void* stream);
/* the same backward without the reduction: only the partial rows are written,
 * [nblk][(2 + want_col) * cols] = dgamma | dbeta | (consumer column sums); they are reduced
 * later, batched with other layers' partials, by cg_reduce_columns (the engine defers the
 * per-layer parameter-gradient reductions of a dW group to one launch) */
int cg_layernorm_bwd_partials(int dy_dtype, const void* dy, long long lddy, const float* x,
                              long long ldx, const float* mean, const float* rstd,
                              const float* gamma, const float* g_in, float* g_out, int out_dtype,
                              void* g_out_t, uint32_t drop_seed, float drop_p, float* partials,
                              size_t partials_bytes, int want_col, int rows, int cols, void* stream);

/* batched column reductions of partial rows (parameter / bias gradients, the backward of the
 * sums autograd performs per nn.Parameter): per job, dst[c] (+)= sum_r part[r * ld + c],
 * c < cols, r < nrows, in a fixed summation order; all jobs in one launch */
typedef struct {
  const float* part;
  long long ld;
  int nrows, cols;
  float* dst;
  int accumulate;
  int first_block; /* filled by cg_reduce_columns */
} cg_reduce_job;
#define CG_REDUCE_MAX 48
typedef struct {
  int n;
  cg_reduce_job j[CG_REDUCE_MAX];
} cg_reduce_batch;
int cg_reduce_columns(const cg_reduce_batch* batch, void* stream);

/* token + position embedding (+dropout) -- model_tiny_gpt.py:305-312 */
int cg_embed_fwd(const int64_t* idx, const float* tok_emb, const float* pos_emb, float* x,
                 int B, int T, int d, uint32_t drop_seed, float drop_p, void* stream);
/* scatter-add backward into tok_emb grad (V rows) and pos grad; with dtok, ws of ws_bytes >=
 * cg_embed_bwd_workspace(B,T,V,d) bytes (else CG_EINVAL) */
size_t cg_embed_bwd_workspace(int B, int T, int V, int d);
int cg_embed_bwd(const int64_t* idx, const float* g, float* dtok, float* dpos, int B, int T,
                 int V, int d, uint32_t drop_seed, float drop_p, int accumulate, void* ws,
                 size_t ws_bytes, void* stream);

/* segment starts from SEP ids: segstart[b,t] = last p<=t with idx[b,p]==sep (else 0);
 * build_attention_mask's cumsum(idx==sep) equality, model_tiny_gpt.py:289-294 */
int cg_segment_starts(const int64_t* idx, int32_t* segstart, int B, int T, int sep_id,
                      void* stream);

/* RoPE (half-split rotate_half) applied in place to the q and k column blocks of the
 * packed qkv rows -- model_tiny_gpt.py:9-45,98-100.  cos_tab/sin_tab: fp32 [T][hd/2]
 * built on the host exactly like RotaryEmbedding._set_cos_sin_cache.  inverse=1
 * applies R^T (backward of the rotation). */
int cg_rope_tab(int dtype, void* qkv, long long ldqkv, int B, int T, int H, int KV, int hd,
                const float* cos_tab, const float* sin_tab, int inverse, void* stream);

/* Fused causal + SEP-segment (+window) attention with GQA and attention-prob
 * dropout, flash-style (no T x T materialisation) -- model_tiny_gpt.py:102-131.
 * qkv rows: [q(H*hd) | k(KV*hd) | v(KV*hd)] with leading dim ldqkv; y: [B*T, H*hd];
 * lse: [B*H*T] fp32 (natural-log logsumexp of the scaled scores). window<=0: none. */
int cg_attn_fwd(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart,
                void* y, long long ldy, float* lse, int B, int T, int H, int KV, int hd,
                int window, uint32_t drop_seed, float drop_p, const void* drop_mask, void* stream);
/* Attention-dropout keep bits (the same keep(seed, (b*H+h)*T + q, key) as the in-kernel hash),
 * precomputed once per (layer, step) so the bf16 MFMA kernels test one bit per (query, key):
 * a tile-major bit array ([b*H][key tile][query][2 words]) over the causal lower triangle, in a buffer of
 * cg_attn_drop_mask_bytes(B, T, H) bytes.  drop_mask (fwd / bwd): such a buffer made with the
 * same seed and p, or NULL to hash in the kernels (identical keep decisions). */
size_t cg_attn_drop_mask_bytes(int B, int T, int H);
int cg_attn_drop_mask(int B, int T, int H, uint32_t drop_seed, float drop_p, void* mask, void* stream);
/* cg_attn_fwd with dropout (0 < drop_p < 1) whose forward also writes the keep bits into mask_out
 * (a cg_attn_drop_mask_bytes buffer) for the backward: the bf16 MFMA forward hashes the keep
 * decisions itself and stores, for every (query, key) pair a query can see, the bits
 * cg_attn_drop_mask would store (bits of pairs no query sees are left as they are); other paths
 * run cg_attn_drop_mask and then cg_attn_fwd.  Replaces the drop_mask + fwd pair of
 * model_tiny_gpt.py:104-114 (SDPA dropout_p) in the training forward. */
int cg_attn_fwd_keep(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart, void* y,
                     long long ldy, float* lse, int B, int T, int H, int KV, int hd, int window,
                     uint32_t drop_seed, float drop_p, void* mask_out, void* stream);
/* Attention probabilities materialised (the manual path's `last_attn`, model_tiny_gpt.py:117-128):
 * out fp32 [B][H][T][T] = exp(S/sqrt(hd) - lse) on visible (query, key), 0 elsewhere, from the
 * forward's qkv rows (post-RoPE) and lse.  Inspection path. */
int cg_attn_probs(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart, const float* lse,
                  float* out, int B, int T, int H, int KV, int hd, int window, void* stream);
/* backward: writes dqkv (dtype) for q,k,v column blocks.  ws: ws_bytes >= cg_attn_bwd_workspace()
 * bytes (else CG_EINVAL; 2 B H T + 4096 B H ceil(T/64) floats: the per-query rows and the fused pass's
 * dQ accumulator).
 * bias_part (optional, bf16 MFMA path only -- CG_EUNSUPPORTED otherwise): fp32 column sums of
 * dqkv (before bf16 rounding) per (batch, 128-row tile), rows b*ceil(T/128) + tile, leading dim
 * ld_part >= (H + 2 KV) hd; reduced by cg_colsum_reduce into the q/k/v bias gradients. */
size_t cg_attn_bwd_workspace(int B, int T, int H);
int cg_attn_bwd(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart,
                const void* y, long long ldy, const void* dy, long long lddy, const float* lse,
                void* dqkv, long long lddqkv, int B, int T, int H, int KV, int hd, int window,
                uint32_t drop_seed, float drop_p, const void* drop_mask, float* bias_part,
                long long ld_part, void* ws, size_t ws_bytes, void* stream);
/* cg_attn_bwd for RoPE models (ABI 0.3): qkv holds the ROTATED q / k (model_tiny_gpt.py:91-93
 * applies RotaryEmbedding after the projection), and the dQ / dK outputs -- and bias_part -- are
 * rotated back to the gradients w.r.t. the un-rotated projections in the kernels' registers
 * (the inverse rotation at each row's position), replacing a separate inverse-rotation pass.
 * rope_cos / rope_sin: 16-B aligned fp32 [>= T][hd/2] tables as cg_rope_tab takes; both NULL =
 * cg_attn_bwd.  Tables with a non-MFMA configuration (fp32, hd not 32/48/64): CG_EUNSUPPORTED. */
int cg_attn_bwd_rope(int dtype, const void* qkv, long long ldqkv, const int32_t* segstart,
                     const void* y, long long ldy, const void* dy, long long lddy, const float* lse,
                     void* dqkv, long long lddqkv, int B, int T, int H, int KV, int hd, int window,
                     uint32_t drop_seed, float drop_p, const void* drop_mask, float* bias_part,
                     long long ld_part, const float* rope_cos, const float* rope_sin, void* ws,
                     size_t ws_bytes, void* stream);
/* ABI 0.5: cg_attn_bwd_rope with the bf16 MFMA backward's algorithm chosen per call.
 *   CG_ATTN_BWD_AUTO  (0): the split pass (measured faster in the step at every benchmarked geometry,
 *                          profiles/round6/attn_bwd_fused_ab.txt)
 *   CG_ATTN_BWD_SPLIT (1): two kernels -- dQ (S, dP, dQ per query tile), then dK / dV (S, dP, dV,
 *                          dK per key tile): seven MFMA products per tile
 *   CG_ATTN_BWD_FUSED (2): one pass per (batch, kv head) -- S, dP, dV, dK and dQ, five products per
 *                          tile, dQ summed over the key blocks in an fp32 part of ws that only that
 *                          workgroup writes (no atomics: bitwise reproducible) -- between a row-
 *                          statistics pre-pass and a pass that writes the bf16 dQ columns
 * Both replace the autograd of model_tiny_gpt.py:102-131 with the same results up to fp32
 * summation order.  FUSED needs the bf16 MFMA configuration and, with dropout, drop_mask
 * (CG_EUNSUPPORTED otherwise); AUTO and SPLIT run every configuration. */
enum { CG_ATTN_BWD_AUTO = 0, CG_ATTN_BWD_SPLIT = 1, CG_ATTN_BWD_FUSED = 2 };
int cg_attn_bwd_algo(int algo, int dtype, const void* qkv, long long ldqkv, const int32_t* segstart,
                     const void* y, long long ldy, const void* dy, long long lddy, const float* lse,
                     void* dqkv, long long lddqkv, int B, int T, int H, int KV, int hd, int window,
                     uint32_t drop_seed, float drop_p, const void* drop_mask, float* bias_part,
                     long long ld_part, const float* rope_cos, const float* rope_sin, void* ws,
                     size_t ws_bytes, void* stream);

/* Label-smoothed, class-weighted, ignore_index cross-entropy fwd+bwd over logits rows
 * (F.cross_entropy at model_tiny_gpt.py:343-349).  logits fp32 [rows][ldl], V used
 * columns; writes loss (1 float, mean per the reference weighting), dlogits (d_dtype
 * CG_F32 / CG_BF16 / CG_BF16X2, pad columns [V, ldd) -- per half for CG_BF16X2 -- zeroed)
 * scaled by `grad_scale`.  ws: ws_bytes >= cg_ce_workspace(rows) bytes (else CG_EINVAL) */
size_t cg_ce_workspace(int rows);
int cg_cross_entropy(const float* logits, long long ldl, const int64_t* targets, int rows,
                     int V, float eps, const float* class_w, int ignore_index,
                     float grad_scale, int d_dtype, void* dlogits, long long ldd,
                     float* loss, void* ws, size_t ws_bytes, void* stream);

/* SwiGLU: s = silu(gu[:, :H]) * gu[:, Hp:Hp+H] (model_tiny_gpt.py:57) and backward */
int cg_swiglu_fwd(int dtype, const void* gu, long long ldgu, int Hp, void* s, long long lds,
                  int rows, int H, void* stream);
int cg_swiglu_bwd(int dtype, const void* gu, long long ldgu, int Hp, const void* ds,
                  long long ldds, void* dgu, long long lddgu, int rows, int H, void* stream);

/* column sums (bias gradients): out[n] (+)= sum_m X[m*ldx+n]; ws of ws_bytes >=
 * cg_colsum_workspace(rows, cols) bytes (else CG_EINVAL) */
size_t cg_colsum_workspace(int rows, int cols);
int cg_colsum(int dtype, const void* X, long long ldx, int rows, int cols, float* out,
              int accumulate, void* ws, size_t ws_bytes, void* stream);
/* the first stage alone: *nparts partial rows [*nparts][cols] fp32 into part (part_bytes >=
 * cg_colsum_workspace), for a reduction batched with others (cg_reduce_columns) */
int cg_colsum_partials(int dtype, const void* X, long long ldx, int rows, int cols, float* part,
                       size_t part_bytes, int* nparts, void* stream);

/* out[c] (+)= sum_i part[i*cols + c] over nparts partial rows (the second stage of the fused
 * bias-gradient column sums, e.g. CG_EPI_COLSUM GEMM partials) */
int cg_colsum_reduce(const float* part, int nparts, int cols, float* out, int accumulate, void* stream);

/* batched transpose of 2-byte matrices: dst[c][r] = src[r][c]; rows, cols, lds, ldd multiples
 * of 8, 16-B aligned pointers.  Used to give the backward dX products K-contiguous weight
 * operands (bf16 shadow weights transposed once per step). */
#define CG_TRANSPOSE_MAX 64
typedef struct {
  const void* src; void* dst;
  long long lds, ldd;
  int rows, cols;
} cg_transpose_item;
typedef struct {
  int n;
  cg_transpose_item items[CG_TRANSPOSE_MAX];
} cg_transpose_batch;
int cg_transpose16_batch(const cg_transpose_batch* tb, void* stream);

/* elementwise casts / utilities */
int cg_cast_f32_to_bf16(const float* src, uint16_t* dst, long long n, void* stream);
int cg_cast_bf16_to_f32(const uint16_t* src, float* dst, long long n, void* stream);
/* x[r][c] *= *scale (device float; exactly 1 is a no-op) for dtype CG_F32 / CG_BF16 / CG_BF16X2 */
int cg_scale_dev(int dtype, void* x, long long ld, int rows, int cols, const float* scale, void* stream);
/* dst[r][c] = src[r][c] (c < cols), 0 for cols <= c < dcols; dst in `dtype` (CG_BF16X2: hi in
 * columns [0, dcols), lo in [dcols, 2 dcols); ldd >= 2 dcols) */
int cg_cast_pad_2d(const float* src, long long lds, int rows, int cols, int dtype, void* dst,
                   long long ldd, int dcols, void* stream);

/* Device-resident batches (src/codonlm/data_loading.py): the token arrays live in HBM and a
 * batch is one gather launch (no per-step host->device copy of tokens).  elem_bytes: 1
 * (uint8), 2 (int16), 4 (int32) or 8 (int64) storage, widened to int64.
 * fixed windows (PackedDataset X/Y :43-129): out[b][t] = X[rows[b]][t]
 * dynamic sequences (flat X + lengths, dynamic_lm_collate_fn :380-393): x[b][t] = seq[t],
 * y[b][t] = seq[t+1] for t < len-1, PAD (0) beyond; seq = flat[starts[r] .. +lens[r]).
 * rows: device int64 sample indices; out-of-range rows give PAD rows. */
int cg_gather_windows(int elem_bytes, const void* X, long long ldx, long long nrows,
                      const int64_t* rows, int B, int T, int64_t* out, void* stream);
int cg_gather_sequences(int elem_bytes, const void* flat, const int64_t* starts,
                        const int64_t* lens, long long nseq, const int64_t* rows, int B, int Tout,
                        int64_t* x, int64_t* y, void* stream);

/* Sequence embeddings from hidden states (scripts/extract_embeddings.py _pool_state :94-114):
 * h: [B*T rows][ldh] (dtype) as cg_model_hidden returns; out fp32 [B][d].
 * mode 0 = mean over idx != pad_id, 1 = mean over ids set in content_mask (host, 8 x 32-bit
 * words = ids 0..255), 2 = the state at position (#non-PAD - 1, clamped at 0). */
enum { CG_POOL_MEAN_NONPAD = 0, CG_POOL_MEAN_CONTENT = 1, CG_POOL_EOS = 2 };
int cg_pool_hidden(int dtype, const void* h, long long ldh, const int64_t* idx, int B, int T,
                   int d, int pad_id, int mode, const uint32_t* content_mask, float* out,
                   void* stream);

/* Auxiliary objectives' label construction (src/codonlm/training/objectives.py).
 * offset targets (offset_target_mask :6-23): out[b][t] = y[b][t+k-1] where that target is
 * valid (t+k-1 < T, not PAD, no boundary id among y[b][t..t+k-2]), else 0 (= ignored by the
 * PAD-ignoring cross-entropy); *n_valid (device int, optional) += number of valid targets. */
int cg_offset_targets(const int64_t* y, int B, int T, int offset, const int* boundary_ids,
                      int n_boundary, int64_t* out, int* n_valid, void* stream);
/* termination_distance_bucket_labels (:63-91): distance to the next stop id bucketed by
 * the sorted edges (count of edges < distance); no later stop -> n_edges; PAD -> ignore. */
int cg_termination_labels(const int64_t* y, int B, int T, const int* stop_ids, int n_stop,
                          const int* edges, int n_edges, int ignore_index, int64_t* labels,
                          void* stream);

/* Fused AdamW over the flat parameter buffer (torch.optim.AdamW semantics,
 * loop.py:681-731): up to 4 contiguous segments with their own (lr, wd); grads are
 * multiplied by grad_scale (1/(n_micro*world)) first; optionally refreshes the bf16
 * shadow copy used by the bf16 GEMMs.  step is the 1-based AdamW step count. */
typedef struct { long long begin, end; float lr, wd; } cg_adamw_segment;
int cg_adamw(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
             uint16_t* shadow_bf16, const cg_adamw_segment* segs, int nseg, float beta1,
             float beta2, float eps, int step, float grad_scale, void* stream);
/* nonfinite flag: flag |= any(!isfinite(x[0..n))) (device int) */
int cg_nonfinite_flag(const float* x, long long n, int* flag, void* stream);

/* ------------------------------------------------------------------------------
 * Whole-model engine: the TinyGPT forward/backward sequence as one native call per
 * phase (replaces TinyGPT.forward + loss.backward(), model_tiny_gpt.py:297-352,
 * loop.py:1067-1233).  Parameters live in ONE flat fp32 buffer whose layout is owned
 * by the library (cg_model_param_layout); grads use the same layout.
 * ----------------------------------------------------------------------------*/
/* engine options (ABI 0.4): all zero = the defaults the engine was measured fastest with; each
 * field selects a measured alternative for tests and same-box A/B runs.  They are part of the
 * model's configuration (fixed for its lifetime), so the workspace size and the dW plan that
 * cg_model_workspace_bytes / cg_model_dw_plan report are the ones forward / backward use. */
typedef struct {
  int dw_group;           /* blocks per grouped dW launch (0 = the planner's choice)            */
  int dw_ksplit;          /* token-range split of the grouped dW tiles, 1..3 (0 = planner);     */
                          /* out of range -> CG_EINVAL                                          */
  int dw_remainder_first; /* 1: the short remainder dW group runs first from the top (0: last) */
  int head_dw_separate;   /* 1: the tied head's dW as its own split-K product in backward phase */
                          /* 0 (0: inside the first grouped dW launch)                          */
  int rope_tables;        /* 1: RoPE as separate cg_rope_tab passes (0: fused into the qkv      */
                          /* projection's epilogue and the attention backward)                  */
  int attn_mask_kernel;   /* 1: the attention dropout keep bits by cg_attn_drop_mask before     */
                          /* each block's forward (0: written by the attention forward itself); */
                          /* 2 (ABI 0.5): made in the block's LN1 launch, cg_layernorm_fwd_mask */
  int dw_plan_tokens;     /* > 0: plan the grouped dW as for steps of this many tokens (a small  */
                          /* parity step then runs a large step's plan); 0: the step's own B*T  */
  int attn_bwd_algo;      /* ABI 0.5: CG_ATTN_BWD_* for every block's attention backward (0 auto) */
  int pers_max_wg;        /* ABI 0.5: grid cap of every persistent launch (grouped dW, persistent */
                          /* fwd / dX GEMMs); 0 = one workgroup per CU.  A data-parallel run sets */
                          /* cg_pers_cus() - R to leave R CUs to the bucket all-reduce's kernels  */
} cg_model_opts;
typedef struct {
  int vocab_size, block_size, n_layer, n_head, n_kv_head, n_embd;
  int use_swiglu, use_rope, sep_id /* <0: none */, tie_embeddings;
  int termination_aux, termination_n_classes;
  int n_offsets; int offsets[8];
  float dropout, label_smoothing, ln_eps;
  int dtype; /* CG_F32 or CG_BF16 */
  cg_model_opts opts;
} cg_model_cfg;

/* parameter tensor kinds (layer = -1 for global tensors) */
enum {
  CG_P_TOK_EMB = 0, CG_P_POS_EMB, CG_P_LN1_W, CG_P_LN1_B, CG_P_Q_W, CG_P_K_W, CG_P_V_W,
  CG_P_Q_B, CG_P_K_B, CG_P_V_B, CG_P_PROJ_W, CG_P_PROJ_B, CG_P_LN2_W, CG_P_LN2_B,
  CG_P_FC1_W, CG_P_FC1_B, CG_P_FC2_W, CG_P_FC2_B, CG_P_GATE_W, CG_P_UP_W, CG_P_DOWN_W,
  CG_P_LNF_W, CG_P_LNF_B, CG_P_HEAD_W, CG_P_TERM_W, CG_P_TERM_B, CG_P_OFF1_W, CG_P_OFF1_B,
  CG_P_OFF2_W, CG_P_OFF2_B, CG_P_NKINDS
};
typedef struct {
  int kind, layer;        /* layer: block index, offset index (OFF*), or -1 */
  long long offset;       /* element offset into the flat buffer */
  int rows, cols;         /* logical (state_dict) shape; cols=0 for 1-D */
  long long ld;           /* row stride in elements (>= cols) */
} cg_param_entry;
/* returns number of entries (<= max) and the flat buffer size in *total_elems */
int cg_model_param_layout(const cg_model_cfg* cfg, cg_param_entry* out, int max,
                          long long* total_elems);
size_t cg_model_workspace_bytes(const cg_model_cfg* cfg, int B, int T);
/* the grouped weight-gradient plan of the bf16 engine for a (B, T) step on the current device:
 * blocks per grouped dW launch, the tile code of a full group and its token-range split (the plan
 * forward / backward use at that B * T; it depends on the token count) */
int cg_model_dw_plan(const cg_model_cfg* cfg, int B, int T, int* group_layers, int* tile_m, int* ksplit);

typedef struct {
  cg_model_cfg cfg;
  float* params;            /* flat fp32 master */
  const uint16_t* shadow;   /* flat bf16 copy (dtype==CG_BF16) */
  float* grads;             /* flat fp32 grads, same layout */
  const float* loss_weights;/* [V] or NULL (uniform) */
  const float* rope_cos;    /* [block_size][hd/2] (use_rope) */
  const float* rope_sin;
  void* workspace; size_t workspace_bytes;
  /* filled by cg_model_forward, consumed by cg_model_backward / cg_model_hidden */
  int B, T, training, window;
  uint32_t seed;
  const int64_t* idx;
  const int64_t* targets;
  float* logits;
  /* auxiliary heads (model_tiny_gpt.py:329-337).  cg_model_forward resets these to
   * (0, 1, NULL...); the caller sets the gradients of the aux outputs between
   * cg_model_aux_forward and cg_model_backward phase 0. */
  int aux_ready;                    /* set by cg_model_aux_forward                      */
  float head_grad_scale;            /* d(objective)/d(next-codon loss)                  */
  const float* head_grad_scale_dev; /* optional device float multiplying it (no host sync) */
  const float* d_term_logits;       /* fp32 [B*T][ld_d_term] or NULL                    */
  long long ld_d_term;
  const float* d_offset_logits[8];  /* fp32 [B*T][V] per offset head, or NULL           */
  /* set by cg_model_backward: the weight gradients of blocks are produced in groups (one
   * grouped dW launch per group of blocks, bf16 engine); after each call every parameter
   * gradient of blocks >= dw_done_layer (and of the head / ln_f after phase 0) is final --
   * the point a data-parallel caller may start that bucket's all-reduce. */
  int dw_done_layer;
  /* engine-private backward state (zero-initialise; the caller never writes it): the tied
   * head's weight gradient deferred from phase 0 into the first grouped dW launch (bf16, tied,
   * no aux heads).  Phase 0 sets it, the first dW group or phase 2 consumes it. */
  long long head_dw_off;
  float head_dw_alpha;
  int head_dw_accumulate;
  int head_dw_pending;
  /* engine-private: the parameter / bias gradient column reductions deferred to the end of the
   * current dW group (one cg_reduce_columns launch per group) */
  cg_reduce_batch reduce_pending;
} cg_model;

/* forward: logits (fp32 [B*T][V] contiguous; NULL => internal buffer), loss (device
 * float; targets NULL => no loss).  With targets, d(loss)/d(logits) is produced here
 * (fused CE fwd+bwd).  training enables dropout with `seed`; window<=0: no window. */
int cg_model_forward(cg_model* m, const int64_t* idx, const int64_t* targets, int B, int T,
                     int training, uint32_t seed, int window, float* logits, float* loss,
                     void* stream);
/* auxiliary heads on the ln_f output of the last forward (model_tiny_gpt.py:329-337):
 * termination logits fp32 [B*T][ld_term] = xf W_t^T + b_t (termination_aux), and per
 * offset head i: logits_i fp32 [B*T][ld_off] = head(W2 gelu(W1 xf + b1) + b2) (tied head);
 * ld_off >= V; with ld_off >= round_up(V, 16) the zero pad columns are computed too (the
 * product then takes the vector / persistent GEMM tiles).
 * The offset activations stay in the workspace for the backward. */
int cg_model_aux_forward(cg_model* m, float* term_logits, long long ld_term,
                         float* const* offset_logits, long long ld_off, void* stream);
/* backward in phases so the caller can overlap per-bucket gradient all-reduce:
 *   phase 0: head (+ aux heads) + ln_f; phase 1: one block `layer` (call L-1 .. 0; block
 *   weight gradients complete per dW group, see cg_model.dw_done_layer);
 *   phase 2: embeddings.  Phase 0 scales the next-codon head gradient by head_grad_scale
 *   and adds the aux-head gradients given in d_term_logits / d_offset_logits; aux
 *   parameters without a gradient are zeroed when accumulate=0.
 * accumulate=0 overwrites grads (first microbatch of a group), 1 adds. */
int cg_model_backward(cg_model* m, int phase, int layer, int accumulate, void* stream);
/* pointer to hidden state `which` (0 = embedding output, 1..L = block outputs,
 * L+1 = ln_f output) inside the workspace after a forward; dtype in *dtype_out */
const void* cg_model_hidden(const cg_model* m, int which, int* dtype_out, long long* ld);
/* attention probabilities of block `layer` of the last forward: fp32 [B][H][T][T] (cg_attn_probs) */
int cg_model_attn_probs(const cg_model* m, int layer, float* out, void* stream);

/* Incremental decoding with a KV cache (query_model.py generate / next_token :160-214 without
 * re-running the whole prefix).  The cache holds, per layer and sequence, the post-RoPE K and
 * V rows of every position: layout [L][B][Tmax][2*kv_dim] in the model dtype.  Valid while
 * the context fits block_size (the reference then slides its window and recomputes).
 *   cg_model_prefill: full eval forward of idx [B][T] (logits [B*T][V]), fills cache rows
 *     0..T-1 and segstate[b] (start of the last SEP segment; 0 without sep masking).
 *   cg_model_decode: one new token per sequence at position pos (= current length): writes
 *     its cache rows and logits [B][V].  dec_ws: cg_decode_workspace_bytes(cfg, B). */
size_t cg_kv_cache_bytes(const cg_model_cfg* cfg, int B, int Tmax);
size_t cg_decode_workspace_bytes(const cg_model_cfg* cfg, int B);
int cg_model_prefill(cg_model* m, const int64_t* idx, int B, int T, int window, void* cache, int Tmax,
                     int32_t* segstate, float* logits, void* stream);
int cg_model_decode(cg_model* m, const int64_t* tok, int B, int pos, void* cache, int Tmax,
                    int32_t* segstate, void* dec_ws, size_t dec_ws_bytes, float* logits, void* stream);
/* the decode step's attention: query rows q [B][ldq] (head h at column h*hd), cache rows of
 * one layer [B][Tmax][ldc] (K at kv_head*hd, V at KV*hd + kv_head*hd), keys
 * max(segstate[b], pos-window+1) .. pos; y [B][ldy] */
int cg_attn_decode(int dtype, const void* q, long long ldq, const void* cache, long long ldc, int Tmax,
                   int pos, const int32_t* segstate, int window, int B, int H, int KV, int hd, void* y,
                   long long ldy, void* stream);
/* segstate[b] = pos where tok[b] == sep_id (the SEP token opens its segment) */
int cg_segstate_step(const int64_t* tok, int B, int sep_id, int pos, int32_t* segstate, void* stream);

/* Live probe of one kernel class during a real run: HIP events are recorded on the
 * launching stream around each launch of the selected kernel together with its
 * algorithmic work (FLOPs for MFMA kernels).  kind 0 disables.  cg_probe_read
 * synchronises on the recorded events and returns (work, total device ms, launches). */
enum {
  CG_PROBE_NONE = 0,
  CG_PROBE_GEMM_DW = 1,      /* bf16 dW GEMM main kernel (A,B MN-contiguous)       */
  CG_PROBE_GEMM_FWD = 2,     /* bf16 forward GEMM main kernel (A,B K-contiguous)   */
  CG_PROBE_GEMM_DX = 3,      /* bf16 dX GEMM main kernel                           */
  CG_PROBE_ATTN_FWD = 4,     /* attn_fwd_mfma                                      */
  CG_PROBE_ATTN_DQ = 5,      /* attn_bwd_dq_mfma                                   */
  CG_PROBE_ATTN_DKDV = 6,    /* attn_bwd_dkdv_mfma                                 */
  CG_PROBE_GEMM_DW_GROUPED = 7, /* grouped weight-gradient GEMM (gemm_dw_kernel)     */
  CG_PROBE_GEMM_PERS = 8,      /* persistent fwd / dX GEMM (gemm_bf16_pers_kernel, all */
                               /* epilogue specialisations: one kernel class)           */
  CG_PROBE_ATTN_BWD = 9,       /* attn_bwd_fused_mfma (the fused dQ / dK / dV pass)     */
  CG_PROBE_DW_SLAB = 10        /* dw_slab_reduce_kernel: the k-split slab sum after the */
                               /* grouped dW (HBM-bound; work = its adds, bytes = slabs */
                               /* read + dW read and written)                           */
};
int cg_probe_enable(int kind);
/* record 1 of every `every` launches of the probed kernel (default 1 = all); the launch
 * count and work returned by cg_probe_read cover the recorded launches only */
int cg_probe_sample(int every);
int cg_probe_read(double* work, double* ms, long long* launches);
/* algorithmic HBM bytes (operands once + outputs once) of the same recorded launches */
int cg_probe_bytes(double* bytes);

/* diagnostic: occupy n_cus CUs (one 1024-thread workgroup holding all 160 KiB of LDS each) for
 * `usec` microseconds on `stream` -- stands in for kernels that run beside the step (an RCCL
 * all-reduce) when measuring the persistent launches' sensitivity to busy CUs */
int cg_diag_occupy(int n_cus, int usec, void* stream);

/* sizeof the named ABI struct ("cg_gemm_desc", "cg_dw_product", "cg_dw_group", "cg_reduce_job",
 * "cg_reduce_batch", "cg_transpose_item", "cg_transpose_batch", "cg_adamw_segment",
 * "cg_model_cfg", "cg_param_entry", "cg_model", "cg_model_opts"), 0 for another name: lets a binding that mirrors
 * the layouts check them against the library it loaded. */
size_t cg_struct_bytes(const char* name);

/* "codonlm_hip <abi> gfx950".  ABI 0.2 (round 3): cg_gemm_desc.ws_bytes and the size_t
 * workspace-size argument after every workspace pointer.  ABI 0.3 (round 4): cg_model gained
 * the engine-private head_dw_* fields at its end.  ABI 0.4 (round 5): no process-wide setters --
 * cg_gemm_desc.tile / max_wg, cg_dw_group.max_wg and cg_model_cfg.opts replace the cg_set_* /
 * cg_gemm_set_* calls and the environment switches; cg_model_dw_plan takes (B, T) and reports the
 * token split; cg_model.embed_done is gone.  ABI 0.5 (round 6): the fused attention backward --
 * cg_attn_bwd_algo, cg_model_opts.attn_bwd_algo, CG_PROBE_ATTN_BWD; cg_attn_bwd_workspace also
 * covers the fused pass's dQ accumulator. */
const char* cg_version(void);

#ifdef __cplusplus
}
#endif
#endif

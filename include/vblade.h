/*
 * vblade.h — C ABI of libvblade_hip.so, the MI355X (gfx950) block-sparse attention path of
 * Video-BLADE. Plain pointers, sizes and strides; no framework types. Every device pointer is
 * a HIP device address; `stream` is a hipStream_t (NULL = the null stream).
 *
 * Contract:
 *   - the caller owns every buffer (inputs read-only, outputs fully overwritten); the library
 *     never allocates, frees or synchronises, so every entry point is hipGraph-capturable;
 *   - return 0 on success, a negative VB_ERR_* code otherwise; vb_last_error() holds the message
 *     of the last failure on the calling thread; no C++ exception crosses the ABI;
 *   - stateless and reentrant; all work is enqueued on `stream`.
 *
 * Tensor convention: "[B,H,L,D] strided" = element (b,h,l,d) at base + b*s[0] + h*s[1] + l*s[2] + d,
 * strides in ELEMENTS, innermost (d) stride 1. Row-index arrays ("rows") map a position of the
 * reordered (Gilbert) sequence to the row of the caller's tensor that holds it; NULL = identity.
 */
#ifndef VBLADE_H_
#define VBLADE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VB_ABI_VERSION 4   /* 2: mask_head_mode argument of vb_block_sparse_attn_fwd/bwd; 3: vb_attn_args.q_order;
                              4: work_queue (persistent forward), kernel_select/kernels_ran (backward) */

/* Work queue of the persistent forward launches (vb_attn_args / vb_ml_attn_args.work_queue): device
 * int32[VB_WORK_QUEUE_INTS], ALL ZERO before its first use; every launch leaves it zero again. One
 * queue serves one launch at a time (launches that may overlap, e.g. on two streams, need one each). */
#define VB_WORK_QUEUE_INTS 288

enum vb_status {
  VB_OK = 0,
  VB_ERR_INVALID = -1,     /* bad argument / shape */
  VB_ERR_UNSUPPORTED = -2, /* valid for the reference op but not implemented (dropout, causal, streaming, head dim) */
  VB_ERR_LAUNCH = -3       /* the HIP launch failed */
};

enum vb_dtype { VB_DTYPE_BF16 = 0, VB_DTYPE_F16 = 1 };
/* reading of head_mask_type = ones(H) (see vb_block_sparse_attn_fwd) */
enum vb_mask_head_mode { VB_MASK_HEAD_PER_HEAD = 0, VB_MASK_HEAD_SHARED0 = 1 };

/* Message of the last failing call on this thread ("" if none). */
const char* vb_last_error(void);
int vb_abi_version(void);

/* ------------------------------------------------------------------------------------------
 * Gilbert 3-D curve permutation (host). Replaces GilbertRearranger.__init__ /
 * _gilbert3d_with_index + utils/gilbert3d.py:6-167
 * (cogvideox/train/special_attentions_local/TrainRelated/cogvideo_blocksparseattn.py:112-140).
 * perm_out[g] = x + width*(y + height*z) of the g-th curve point (length width*height*depth).
 * ------------------------------------------------------------------------------------------ */
int vb_gilbert3d_perm(int width, int height, int depth, int32_t* perm_out);

/* ------------------------------------------------------------------------------------------
 * Drop-in for block_sparse_attn_func forward (mit-han-lab/Block-Sparse-Attention) exactly as the
 * reference calls it: cogvideo_blocksparseattn.py:316-320 (also :106-109 for the dense pooled
 * call; wanx_blocksparseattn.py:301-305).
 *   q/k/v_unpad   [total, H, D] contiguous, dtype `dtype`
 *   cu_seqlens_*  int32 [batch+1] (device)
 *   head_mask_type int32 [H] (device): 0 dense; m>0 block-sparse with base_blockmask head m-1;
 *                 m<0 (streaming) -> that head's output is NaN. How the reference's
 *                 head_mask_type = ones(H) (cog :313) reads is open offline:
 *                 mask_head_mode VB_MASK_HEAD_PER_HEAD (0, default) first renumbers every 1 to
 *                 1,2,3,... in head order (Block-Sparse-Attention's replace_ones_with_count: one
 *                 predicted mask per head); VB_MASK_HEAD_SHARED0 (1) reads m literally, so ones(H)
 *                 gives every head base_blockmask head 0.
 *   streaming_info ignored (only used by streaming heads)
 *   base_blockmask uint8/bool [batch, n_sparse, ceil(max_q/128), ceil(max_k/128)] contiguous
 *   out_unpad     [total_q, H, D]; softmax_lse fp32 [batch, H, max_seqlen_q] (natural log).
 *                 A query row with no kept key block gets a zero output row and lse = +inf,
 *                 FlashAttention-2's convention for an empty softmax (its normalize_softmax_lse);
 *                 the native entry vb_attn_fwd reports -inf for such rows instead.
 *   p_dropout must be 0, is_causal/exact_streaming must be 0 (the reference's call) else
 *   VB_ERR_UNSUPPORTED. softmax_scale <= 0 means head_dim^-1/2. `deterministic` is accepted
 *   and ignored (the forward is deterministic).
 * ------------------------------------------------------------------------------------------ */
int vb_block_sparse_attn_fwd(const void* q_unpad, const void* k_unpad, const void* v_unpad,
                             const int32_t* cu_seqlens_q, const int32_t* cu_seqlens_k,
                             const int32_t* head_mask_type, const int32_t* streaming_info,
                             const uint8_t* base_blockmask, int batch, int num_heads, int head_dim,
                             int max_seqlen_q, int max_seqlen_k, float p_dropout, int deterministic,
                             float softmax_scale, int is_causal, int exact_streaming, int dtype,
                             void* out_unpad, float* softmax_lse, int mask_head_mode, void* stream);

/* ------------------------------------------------------------------------------------------
 * Native strided block-sparse attention forward (the adaptive module's hot kernel). One softmax
 * over the union of
 *   (a) full-resolution keys of the 128x128 blocks kept by `block_mask` (NULL = all kept), and
 *   (b) optionally, `Lkp` pooled keys kp/vp carrying an additive score bias `kp_log_bias`
 *       (= ln sample_gap: the LSE combine of cogvideo_blocksparseattn.py:374-393 fused as one
 *       softmax).
 * Setting use_main=0 attends only to (b) (the reference's standard_attn, :106-109).
 * q rows are read at q_rows[g] and out/lse written at q_rows[g] (g = reordered position), so
 * the Gilbert reorder and its inverse (:141-161) cost no separate pass; k/v rows read at kv_rows[g].
 * ------------------------------------------------------------------------------------------ */
typedef struct vb_attn_args {
  const void* q; const void* k; const void* v;
  int64_t q_stride[3]; int64_t k_stride[3]; int64_t v_stride[3];
  const int32_t* q_rows;  /* [Lq] or NULL */
  const int32_t* kv_rows; /* [Lk] or NULL */
  int use_main;           /* attend to the block-masked full-resolution keys */
  const uint8_t* block_mask; int64_t mask_stride[3]; /* [B,H,ceil(Lq/128),ceil(Lk/128)] or NULL */
  const void* kp; const void* vp;                     /* pooled keys [B,H,Lkp,D] strided or NULL */
  int64_t kp_stride[3]; int64_t vp_stride[3];
  int Lkp; float kp_log_bias;
  void* out; int64_t out_stride[3];
  float* lse;             /* [B,H,Lq] fp32 natural-log LSE (written at q_rows) or NULL */
  int B, H, Lq, Lk, D;
  float scale;            /* <= 0 -> D^-1/2 */
  int dtype;
  int heavy_rows;         /* scheduling hint: the last N q-block rows keep (almost) every key
                             block (CogVideoX's forced text rows: 2); 0 = none. Never affects results. */
  int32_t* q_order;       /* scheduling workspace [B*H*ceil(Lq/128)] int32, or NULL (ABI 3): with a
                             block mask, each XCD's q-blocks are dispatched head by head, longest
                             (most kept key blocks) first, so its last workgroups are the short ones.
                             Written by a small launch before the attention kernel. Never affects results. */
  const int32_t* q_lengths; /* [B,H,ceil(Lq/128)] kept key blocks per mask row (vb_predict_args.
                             mask_rows_kept), or NULL: the ordering launch counts them from the mask */
  int order_window;       /* > 0: only the last order_window q-blocks of each XCD range are re-ordered
                             (the tail; the rest keeps the kernel's head-major, Gilbert-neighbour
                             order and its L2 reuse); 0: the whole range */
  int32_t* work_queue;    /* ABI 4, nullable: persistent dispatch — a resident-sized grid whose workgroups
                             pull q-blocks from per-XCD queues (in the order above) and, once their own
                             XCD's queue is empty, from the others'. NULL: one workgroup per q-block.
                             Never affects results. See VB_WORK_QUEUE_INTS. */
} vb_attn_args;
int vb_attn_fwd(const vb_attn_args* args, void* stream);

/* ------------------------------------------------------------------------------------------
 * Fused mask predictor (a3+a4+a5): efficient_attn_with_pooling + attn_with_pooling (Triton,
 * attn_pooling_kernel.py:17-255) + transfer_attn_to_mask(mode="energy")
 * (cogvideo_blocksparseattn.py:57-82, 177-249; wanx_blocksparseattn.py:162-233).
 * For each (b,h): the reordered sequence (rows, replicate-padded to a multiple of `block`) is
 * sampled at the `num_keep` offsets q_off[b,h,:] / k_off[b,h,:] of every block; pooled scores
 * Po [nb,nb] (storage dtype, row-normalised) are written to `po` and the energy rule
 * (threshold, min/max kept blocks, last `force_tail` rows/cols forced) writes `mask` [B,H,nb,nb].
 * Ties between equal Po values are kept lowest-block-first. `mask_count` (nullable) receives
 * an atomic add of the number of kept blocks (device-side sparsity statistic, no host sync).
 * ------------------------------------------------------------------------------------------ */
typedef struct vb_predict_args {
  const void* q; const void* k;
  int64_t q_stride[3]; int64_t k_stride[3];
  const int32_t* rows;     /* [L] reordered -> caller row, or NULL */
  int32_t* q_off;          /* [B,H,num_keep] int32 in [0,block): input, or output with rand_q/rand_k */
  int32_t* k_off;
  int B, H, L, D, block, num_keep;
  float scale;             /* <= 0 -> D^-1/2 */
  float energy_threshold;
  int min_keep, max_keep, force_tail;
  void* po;                /* [B,H,nb,nb] storage dtype, contiguous */
  uint8_t* mask;           /* [B,H,nb,nb] contiguous, or NULL: scores only (no energy rule) */
  unsigned long long* mask_count; /* nullable */
  int dtype;
  void* workspace;         /* device, 16-byte aligned, >= vb_mask_predict_workspace_size(args) bytes:
                              the sampled k rows staged contiguously and the per-row block maxima */
  uint64_t workspace_bytes;
  void* staged_event;      /* nullable hipEvent_t, recorded on `stream` once the sampled rows are
                              staged (before the score kernel): independent work on another stream
                              can start then and overlap the score kernel */
  /* Optional fusions (NULL = off):
   * rand_q/rand_k: [B,H,block] fp32 uniforms, the q then k torch.rand draws of
   *   random_sample_tokens (:45-46); the topk(num_keep) offsets are drawn in the sampling launch
   *   (as vb_sample_offsets) and WRITTEN to q_off/k_off.
   * pool_*: the pooled K/V pass of vb_pool_kv (on this call's k and pool_v, same rows) run by
   *   extra workgroups of the score kernel's own launch, beside it on `stream`: no second stream
   *   and no events. pool_kp/pool_vp [B,H,ceil(L/pool_gap),D]; pool_k_r/pool_v_r [B,H,L,D] or NULL. */
  const float* rand_q;
  const float* rand_k;
  const void* pool_v;
  int64_t pool_v_stride[3];
  int pool_gap;
  void* pool_kp; void* pool_vp;
  void* pool_k_r; void* pool_v_r;
  /* pyr_k/pyr_v: the multi-level path's KV pyramid pass of vb_kv_pyramid (this call's k and
   * pool_v, same rows; [B,H,vb_kv_pyramid_rows(L),D] each) run by extra workgroups of the score
   * kernel's launch, like pool_* (which it excludes): no second stream and no events. */
  void* pyr_k; void* pyr_v;
  /* philox != 0: the two torch.rand(B,H,1,block) draws of random_sample_tokens are generated inside
   * the sampling launch instead of read from rand_q/rand_k — PyTorch's uniform_ on a device
   * generator at state (philox_seed, philox_offset): element i of a draw = the x value of the first
   * hiprand_uniform4 of Philox4x32-10 subsequence i (1.0 mapped to 0.0), the q draw at
   * philox_offset and the k draw at philox_offset + 4 (each torch.rand call advances the offset by
   * 4 per call). Element i takes the x of thread i only while every element has a thread of its own
   * in torch.rand's grid-stride launch: B*H*block <= CUs x max threads per CU of the device (524288
   * on an unpartitioned MI355X); past that the call fails with VB_ERR_UNSUPPORTED. The offsets are WRITTEN
   * to q_off/k_off; the caller advances its generator by 8. */
  int philox;
  uint64_t philox_seed;
  uint64_t philox_offset;
  /* mask_level != 0: `mask` receives the multi-level rank-band mask instead of the energy mask —
   * vb_level_mask's rule (bands level_band_value / [level_band_start, level_band_end) as fractions
   * of nb, 0..8 of them; the last two rows and columns forced to level 1) applied by the score
   * kernel's epilogue to the normalised scores it has just written to po: no second launch and no
   * re-read of po. Replaces the vb_level_mask launch of the multi-level path
   * (Triton/cogvideo_newattn.py:154-207). */
  int mask_level;
  int level_bands;
  const int32_t* level_band_value;
  const double* level_band_start;
  const double* level_band_end;
  /* mask_rows_kept (ABI 3, nullable): [B,H,nb] int32, the number of key blocks the energy rule kept
   * in each mask row (the attention kernel's per-q-block work, for vb_attn_args.q_lengths). */
  int32_t* mask_rows_kept;
} vb_predict_args;
uint64_t vb_mask_predict_workspace_size(const vb_predict_args* args);
int vb_mask_predict(const vb_predict_args* args, void* stream);

/* random_sample_tokens' index draw (cogvideo_blocksparseattn.py:45-46): the caller draws the
 * uniforms (torch.rand(B,H,1,block), q first then k, so the RNG stream is the reference's); this
 * replaces the two topk(num_keep) calls: rand_q/rand_k fp32 [rows, n] -> q_off/k_off int32
 * [rows, keep], indices of the `keep` largest values in descending order (ties: lower index first). */
int vb_sample_offsets(const float* rand_q, const float* rand_k, int rows, int n, int keep,
                      int32_t* q_off, int32_t* k_off, void* stream);

/* Energy rule alone on given scores (transfer_attn_to_mask, mode="energy"):
 * po [B,H,nr,nc] contiguous storage dtype -> mask [B,H,nr,nc]. */
int vb_energy_mask(const void* po, int B, int H, int nr, int nc, float energy_threshold,
                   int min_keep, int max_keep, int force_tail, int dtype, uint8_t* mask,
                   unsigned long long* mask_count, void* stream);

/* ------------------------------------------------------------------------------------------
 * Mean pooling of K and V over `gap` consecutive reordered tokens with replicate padding
 * (simple_pooling, cogvideo_blocksparseattn.py:83-88): kp/vp [B,H,ceil(L/gap),D] contiguous.
 * Optionally (k_r, v_r non-NULL) also writes the reordered copies k_r/v_r [B,H,L,D] contiguous
 * (the reference's index_select, :148-150) in the same pass: every row is read once.
 * ------------------------------------------------------------------------------------------ */
int vb_pool_kv(const void* k, const void* v, const int64_t* k_stride, const int64_t* v_stride,
               const int32_t* rows, int B, int H, int L, int D, int gap, int dtype, void* kp,
               void* vp, void* k_r, void* v_r, void* stream);

/* ------------------------------------------------------------------------------------------
 * Reference-faithful LSE combine (cogvideo_blocksparseattn.py:374-393, each eager op rounded to
 * the storage dtype): out = out1*a + out2*(1-a), a = e1/(e1+e2) from lse1 and lse2 + ln(gap).
 * All tensors [B,H,L,(D)] contiguous; alpha (nullable) receives a as fp32 [B,H,L].
 * ------------------------------------------------------------------------------------------ */
int vb_lse_combine(const void* out1, const float* lse1, const void* out2, const float* lse2,
                   int B, int H, int L, int D, float gap, int dtype, void* out, float* alpha,
                   void* stream);

/* ------------------------------------------------------------------------------------------
 * Backward (FlashAttention-2 semantics, deterministic: no atomics) of the block-sparse attention
 * and of the adaptive module's two-branch form, as the reference's autograd computes it
 * (cogvideo_blocksparseattn.py:316-320 + :366-393):
 *   main branch   keys k/v [B,H,Lk,D] in REORDERED order (row g = reordered key g), block_mask
 *                 [B,H,ceil(Lq/128),ceil(Lk/128)] (NULL = dense), its output `out` and LSE `lse`
 *   pooled branch (kp != NULL) kp/vp [B,H,Lkp,D], its output out2 and LSE lse2 (no bias), the
 *                 combine weight alpha (fp32 [B,H,Lq], as vb_lse_combine writes it) — LSEs and alpha
 *                 are constants: dO1 = alpha*dO, dO2 = storage(1-alpha)*dO; the pooled K/V grads
 *                 are folded back through the mean pool over `pool_gap` reordered keys (replicate
 *                 padding onto the last key)
 * q/out/out2/dout/lse/lse2/alpha/dq rows are addressed through q_rows[g] like vb_attn_fwd; dk/dv of
 * reordered key g are written at row kv_rows[g] (NULL = g). dq/dk/dv are fully overwritten.
 * `workspace` (device, 16-byte aligned) of at least vb_attn_bwd_workspace_size(args) bytes.
 * The workspace grows linearly with B: besides the per-row statistics and the reordered q/dO
 * copies it holds the pooled-key dK/dV partials, psplit * B * H * Lkp * D fp32 values twice, with
 * psplit chosen from H and L only (never B) so that a sample's gradients are the same bits alone
 * or inside a micro-batch. At B=5 that is ~0.86 GB for CogVideoX (psplit 6) and ~1.9 GB for Wan
 * (psplit 14) — small against 288 GB of HBM, so no cap is applied.
 * ------------------------------------------------------------------------------------------ */
typedef struct vb_attn_bwd_args {
  const void* q; int64_t q_stride[3];
  const void* k; const void* v; int64_t k_stride[3]; int64_t v_stride[3];
  const int32_t* q_rows;    /* [Lq] or NULL */
  const int32_t* kv_rows;   /* [Lk] or NULL */
  const uint8_t* block_mask; int64_t mask_stride[3];
  const void* out; int64_t out_stride[3];
  const float* lse;         /* [B,H,Lq] natural log */
  const void* kp; const void* vp; int64_t kp_stride[3]; int64_t vp_stride[3];
  int Lkp;
  const void* out2; int64_t out2_stride[3];
  const float* lse2;        /* [B,H,Lq] */
  const float* alpha;       /* [B,H,Lq] or NULL (= 1: no pooled branch) */
  int pool_gap;
  const void* dout; int64_t dout_stride[3];
  void* dq; int64_t dq_stride[3];
  void* dk; void* dv; int64_t dk_stride[3]; int64_t dv_stride[3];
  void* workspace; uint64_t workspace_bytes;
  int B, H, Lq, Lk, D;
  float scale;              /* <= 0 -> D^-1/2 */
  int dtype;
  int heavy_rows;           /* scheduling hint as in vb_attn_args */
  int kernel_select;        /* ABI 4: VB_BWD_SEL_* bits, 0 = the default kernels (same results up to the
                               fp32 summation order; for A/B tests) */
  int32_t* kernels_ran;     /* ABI 4, HOST memory, nullable: receives the VB_BWD_RAN_* bits of the
                               kernels this call launched */
} vb_attn_bwd_args;
/* kernel_select bits: the earlier kernels each default replaced */
#define VB_BWD_SEL_DKDV_ROUND3 1   /* dK/dV (main and pooled keys; multi-level: level 1) on bwd_dkdv_kernel
                                      instead of the hand-placed stream bwd_dkdv_pipe_kernel */
#define VB_BWD_SEL_DQ_ROUND3 2     /* dQ on bwd_dq_kernel instead of the pipeline bwd_dq_pipe_kernel */
#define VB_BWD_SEL_DQ_RING4 4      /* D=128 pipeline dQ on the 4-slot ring (one workgroup per CU) */
/* kernels_ran bits */
#define VB_BWD_RAN_DKDV_PIPE 1
#define VB_BWD_RAN_DKDV_ROUND3 2
#define VB_BWD_RAN_DQ_PIPE_RING2 4
#define VB_BWD_RAN_DQ_PIPE_RING4 8
#define VB_BWD_RAN_DQ_ROUND3 16
#define VB_BWD_RAN_ML_PYRAMID 32   /* the multi-level pooled-level dK/dV pass */
uint64_t vb_attn_bwd_workspace_size(const vb_attn_bwd_args* args);
int vb_attn_bwd(const vb_attn_bwd_args* args, void* stream);

/* Drop-in for the block_sparse_attn_func backward (same tensor conventions as
 * vb_block_sparse_attn_fwd): dq/dk/dv [total, H, D]; softmax_lse as the forward wrote it.
 * workspace >= vb_block_sparse_attn_bwd_workspace_size(batch, num_heads, max_seqlen_q) bytes. */
uint64_t vb_block_sparse_attn_bwd_workspace_size(int batch, int num_heads, int max_seqlen_q);
int vb_block_sparse_attn_bwd(const void* dout, const void* q_unpad, const void* k_unpad,
                             const void* v_unpad, const void* out_unpad, const float* softmax_lse,
                             const int32_t* cu_seqlens_q, const int32_t* cu_seqlens_k,
                             const int32_t* head_mask_type, const int32_t* streaming_info,
                             const uint8_t* base_blockmask, int batch, int num_heads, int head_dim,
                             int max_seqlen_q, int max_seqlen_k, float p_dropout, float softmax_scale,
                             int is_causal, int exact_streaming, int deterministic, int dtype,
                             void* dq, void* dk, void* dv, void* workspace, uint64_t workspace_bytes,
                             int mask_head_mode, void* stream);

/* ==========================================================================================
 * Multi-level block-sparse attention: the VBench sampler's op (cogvideox/sample_evaluate/
 * modify_cogvideo.py:9 -> Triton/cogvideo_newattn.py:210-234, kernel Triton/kernels/
 * block_sparse_attn_kernel_with_backward_9_10.py). Every (query block i, key block j) pair has a
 * level p in {0, 1, 2, 4, 8}: 0 skips the block, p > 0 attends to the block's 128/p keys of K/V
 * mean-pooled by p, each with logit q.k*scale + ln p.
 * ========================================================================================== */

/* Rows of the KV pyramid of an L-row sequence: 15*Lpad/8 with Lpad = ceil(L/128)*128. */
int vb_kv_pyramid_rows(int L);

/* The KV pyramid (the _forward wrapper's pad_to_multiple + pooling x3, :1239-1270, :1311-1320):
 * k/v [B,H,L,D] with strides k_stride/v_stride (elements; batch, head, row), rows gathered through
 * `rows` (reordered row g = caller row rows[g]; NULL = g) -> kpyr/vpyr [B,H,R,D] contiguous:
 *   rows [0, Lpad)              level 1: the reordered rows, rows >= L ZERO (the kernel's masked
 *                               loads of the tail block, :111, :126)
 *   [Lpad, 3Lpad/2)             level 2: mean of reordered row pairs, rows >= L replicate row L-1
 *   [3Lpad/2, 7Lpad/4)          level 4: mean of level-2 pairs, rounded per level like torch.mean
 *   [7Lpad/4, 15Lpad/8)         level 8
 * One pass reads every row once. */
int vb_kv_pyramid(const void* k, const void* v, const int64_t* k_stride, const int64_t* v_stride,
                  const int32_t* rows, int B, int H, int L, int D, int dtype, void* kpyr, void* vpyr,
                  void* stream);

/* transfer_attn_to_mask (Triton/cogvideo_newattn.py:154-207): po [B,H,nr,nc] contiguous storage
 * dtype -> mask [B,H,nr,nc] uint8. Per row, the entry ranked r in descending order (ties: lower
 * column first; the reference's torch.sort is unstable) gets band_value[b] of the LAST band b with
 * floor(nc*band_start[b]) <= r < floor(nc*band_end[b]) (bounds computed in double, as Python does),
 * else 0; then the last two columns and the last two rows are set to 1. n_bands <= 8, values in
 * {0,1,2,4,8}; band arrays are HOST memory. nc <= 4096. */
int vb_level_mask(const void* po, int B, int H, int nr, int nc, int n_bands, const int32_t* band_value,
                  const double* band_start, const double* band_end, int dtype, uint8_t* mask,
                  void* stream);

/* Multi-level attention forward (_fwd_kernel, :338-692): queries q [B,H,L,D] (rows through q_rows as
 * in vb_attn_fwd), keys/values the pyramids of vb_kv_pyramid, level_mask [B,H,nb,nb] (nb =
 * ceil(L/128); entries other than 1,2,4,8 skip). out [B,H,L,D] written at q_rows[g]; lse (nullable,
 * fp32 [B,H,L] at the caller's row q_rows[g], as vb_attn_fwd) = m + ln(l) of the reference's (l, m).
 * ref_tail = 1 reproduces the reference on L % 128 != 0: a level-1 tail block's keys >= L are
 * zero vectors that still take part (logit 0, value 0); ref_tail = 0 masks them. */
typedef struct vb_ml_attn_args {
  const void* q; int64_t q_stride[3];
  const int32_t* q_rows;       /* [L] or NULL */
  const void* kpyr; const void* vpyr;   /* [B,H,vb_kv_pyramid_rows(L),D] contiguous */
  const uint8_t* level_mask; int64_t mask_stride[3];
  void* out; int64_t out_stride[3];
  float* lse;
  int B, H, L, D;
  float scale;                 /* <= 0 -> D^-1/2 */
  int ref_tail;
  int dtype;
  int heavy_rows;              /* last q-block rows known to be dense (the forced rows): dispatched first */
  int32_t* work_queue;         /* ABI 4, nullable: persistent dispatch as vb_attn_args.work_queue */
} vb_ml_attn_args;
int vb_ml_attn_fwd(const vb_ml_attn_args* args, void* stream);

/* Multi-level attention backward (_backward + the per-level kernels, :696-1237, :1375-1576),
 * FlashAttention-2 semantics from the forward's out and lse, deterministic (no atomics):
 *   dQ over every kept block's keys at its level (+ln p bias);
 *   dK/dV of each pyramid row, the pooled levels' folded back through the means:
 *   dk[r] = dK1[r] + dK2[r/2]/2 + dK4[r/4]/4 + dK8[r/8]/8 for r < L (gradient reaching the
 *   replicate-padded rows is dropped, as the reference does).
 * `rows` (nullable) is the reorder of the forward (pyramid rows and q_rows): q/out/dout/dq rows are
 * addressed through it, and dk/dv of reordered key g are written at caller row rows[g].
 * dq/dk/dv are fully overwritten. workspace >= vb_ml_attn_bwd_workspace_size(args) bytes. */
typedef struct vb_ml_attn_bwd_args {
  const void* q; int64_t q_stride[3];
  const int32_t* rows;         /* [L] or NULL */
  const void* kpyr; const void* vpyr;
  const uint8_t* level_mask; int64_t mask_stride[3];
  const void* out; int64_t out_stride[3];
  const float* lse;            /* as vb_ml_attn_fwd wrote it */
  const void* dout; int64_t dout_stride[3];
  void* dq; int64_t dq_stride[3];
  void* dk; void* dv; int64_t dk_stride[3]; int64_t dv_stride[3];
  void* workspace; uint64_t workspace_bytes;
  int B, H, L, D;
  float scale;                 /* <= 0 -> D^-1/2 */
  int ref_tail;
  int dtype;
  int heavy_rows;
  int kernel_select;           /* ABI 4: as vb_attn_bwd_args (DKDV_ROUND3: the level-1 pass) */
  int32_t* kernels_ran;        /* ABI 4, HOST memory, nullable: as vb_attn_bwd_args */
} vb_ml_attn_bwd_args;
uint64_t vb_ml_attn_bwd_workspace_size(const vb_ml_attn_bwd_args* args);
int vb_ml_attn_bwd(const vb_ml_attn_bwd_args* args, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VBLADE_H_ */

// Shared definitions of the block-sparse attention forward kernel (vb_attn_fwd.hip).
#pragma once
#include "vb_tiles.hpp"

namespace vb {

struct FwdParams {
  const void* q; const void* k; const void* v;
  int64_t qs[3], ks[3], vs[3];
  const int32_t* q_rows; const int32_t* kv_rows;
  const int32_t* cu_q; const int32_t* cu_k;   // varlen row offsets (reference API), nullable
  const int32_t* head_mask_type;              // reference API, nullable
  int hm_mode;                                // VB_MASK_HEAD_PER_HEAD / VB_MASK_HEAD_SHARED0
  int use_main;
  const uint8_t* mask; int64_t ms[3];
  const void* kp; const void* vp; int64_t kps[3], vps[3];
  int Lkp; float pool_bias_l2;                 // bias in the exp2 domain (log2 gap)
  void* out; int64_t os[3];
  float* lse; int64_t lse_s[2];               // row stride 1
  int B, H, Lq, Lk, nbq, nbk;
  float c;                                    // softmax scale * log2(e)
  int heavy_rows;                             // last q-block rows known to be dense (scheduling hint)
  const int32_t* q_order;                     // phase-2 dispatch order (attn_order_kernel), or NULL
  const int32_t* q_len;                       // kept key blocks per mask row (ordering input), or NULL
  int order_window;                           // re-order only the last N items of each XCD range (0: all)
  // multi-level mode (vb_ml_attn_fwd): k/v are the KV pyramids [B,H,15*Lpad/8,D]
  int Lpad;                                   // level-1 rows (ceil(L/128)*128)
  int ref_tail;                               // 1: level-1 tail keys >= L take part (zero rows)
  int dbg;                                    // diagnostic builds only (VB_DEBUG_ATTN)
  int* work_queue;                            // persistent dispatch: per-XCD queue heads, or NULL
  int n_items;                                // work items (nbq * B * H) behind the queue
};

#ifndef VB_DIAG
#define VB_DIAG 0
#endif
#ifndef VB_VPRE64
#define VB_VPRE64 4   // V^T k-steps prefetched before the softmax (D=64); 4 under the iterative-ilp scheduler
                      // (attention kernel 1.016-1.030x on three boxes, bit-identical; 3 was best before it)
#endif
#ifndef VB_VPRE64_ROWS
#define VB_VPRE64_ROWS 3   // the same for the launches that gather K/V rows through the Gilbert index:
                           // 4 spills a DMA offset into their tile-issue blocks (tests/test_codegen.py)
#endif
#ifndef VB_MFMA_ROWSUM
#define VB_MFMA_ROWSUM 0
#endif
#ifndef VB_FWD_SPLIT_PV
#define VB_FWD_SPLIT_PV 1   // D=64: P.V of the first 32 keys issued before the exp of the second 32
#endif
#ifndef VB_FWD_DMA_UNSCOPED
#define VB_FWD_DMA_UNSCOPED 1   // persistent launches: K/V DMAs invisible to hipcc's LDS-DMA waits
#endif
#ifndef VB_FWD_CBIAS
#define VB_FWD_CBIAS 1      // S accumulator seeded with (bias - m), Q pre-scaled: no per-score fma
#endif
#ifndef VB_FWD_LAZY
#define VB_FWD_LAZY 1       // inference launches: no per-tile row max (checked row sums instead)
#endif
// Lazy (inference) loop: s_setprio 1 around parts of the tile (bit 0: the S MFMA chain, bit 1: each
// P.V k-step's MFMAs, bit 2: the exp/pack of a half-tile); 0 = never. `tools/ab.py --what attn`,
// r02: the LSE-returning D=128 loop with 1 / 3 / 7 measured 1.00x / 0.97x / 0.98x (kept off there)
#ifndef VB_FWD_PRIO64
#define VB_FWD_PRIO64 0    // measured (CogVideoX, 3 waves per SIMD): 1 -2.6 %, 2 -0.6 %, 4 -4.1 %, 5 -6.2 %
#endif
#ifndef VB_FWD_PRIO128
#define VB_FWD_PRIO128 3   // measured (Wan, 2 waves per SIMD): 3 +4.1/+4.5 %, 1 +2.5/+5.6 %, 7 +4.2 %, 2 -2.6 %, 4 +0.0 %
#endif
// the Q fragment loaded after the ring's first DMAs (their round trips overlap), per launch form.
// Measured (tools/ab.py, r06, profiles/r06_qlate_ab.log, against the first item-loop build): D=64
// attention 1.044-1.048x, its LSE launch 1.058x; D=128 LSE launch 1.047-1.049x, the inference launch
// on gathered K/V (Wan's module path) 1.001-1.003x per call, on Gilbert copies 0.98x (kept off
// there). On the final tree the CogVideoX call runs 1.002x with it (profiles/r06_fwd_retune_ab.log)
#ifndef VB_FWD_QLATE64
#define VB_FWD_QLATE64 1
#endif
#ifndef VB_FWD_QLATE128
#define VB_FWD_QLATE128 1
#endif
#ifndef VB_FWD_QLATE128_LAZY
#define VB_FWD_QLATE128_LAZY 0   // D=128 inference launch on contiguous (copied) K/V
#endif
#ifndef VB_FWD_WAVES_D64
#define VB_FWD_WAVES_D64 3  // waves per SIMD the D=64 kernel is register-budgeted for
#endif

constexpr int kThreads = 256;
constexpr int kQBlk = 128;   // rows per workgroup (4 waves x 32)
constexpr int kKT = 64;      // keys per LDS tile
constexpr int kMaxBlocks = 1024;  // keys <= 131072
#ifndef VB_RESCALE_SLACK
#define VB_RESCALE_SLACK 4.0f
#endif
constexpr float kRescaleSlack = VB_RESCALE_SLACK;  // log2 units: P <= 16 between rescales
// lazy-max mode: a half-tile row sum (>= each of its P) above this raises m. bf16 P: with
// P <= 2^32, O and l stay below 2^32 * Lk * max|V| (Lk <= 2^17): no overflow for any |V| < 2^78.
// f16 P (max 65504): P <= 2^8, so P keeps the same normal range below it as P <= 1 does.
constexpr float kLazyBoundBF16 = 4294967296.0f;
constexpr float kLazyBoundF16 = 256.0f;

// ---- LDS images --------------------------------------------------------------------------------
// K: [64 rows][D] with 16-byte chunks XOR-swizzled so a ds_read_b128 column slice (32 rows, one
//    chunk) hits 16 distinct bank slots per lane group (guide T2).
template <int D>
__device__ __forceinline__ int k_off(int row, int ch) {
  constexpr int kRowBytes = D * 2;
  const int sw = (D == 64) ? ((row >> 1) & 7) : (row & 15);
  return row * kRowBytes + 16 * (ch ^ sw);
}
// V: [64 rows][D] row-major, 64-byte granules XOR-swizzled so the 4-row x 64-byte footprint of
//    a half-wave's ds_read_b64_tr_b16 covers a full 256-byte bank row.
template <int D>
__device__ __forceinline__ int v_off_bytes(int row, int col) {
  constexpr int kRowBytes = D * 2;
  const int g = col >> 5;
  const int sw = (D == 64) ? ((row >> 1) & 1) : (row & 3);
  return row * kRowBytes + 64 * (g ^ sw) + (col & 31) * 2;
}

// Describes where tile t's keys come from.
struct TileSrc {
  int pooled;   // 0 = main (block-masked) keys, 1 = pooled keys
  int kstart;   // first key (reordered index for main, pooled index otherwise)
  int klen;     // valid keys in this tile (1..64)
};

// Multi-level tile: 64 pyramid rows of one level. The rows this wave's LDS-DMA fills (its half of
// the tile, 32 rows) come as two 16-row quarters starting at pyramid rows srcA and srcB: a level-8
// block is 16 rows, a level-4 block 32, levels 1/2 are contiguous.
struct MlTileSrc {
  int srcA, srcB;   // pyramid rows of this wave's first and second 16-row quarter
  int klen;         // valid keys in this tile (1..64); the rest are masked
  int lvl;          // log2 of the level: the logit bias in the exp2 domain
};

}  // namespace vb

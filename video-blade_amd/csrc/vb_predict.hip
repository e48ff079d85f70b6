// Mask predictor for gfx950 (sampled pooled scores + energy top-k).
//
// vb_mask_predict fuses, per (b, h) and group of four 32-row sampled q-blocks:
//   * efficient_attn_with_pooling: replicate pad + per-block token sampling
//     (cogvideox/train/special_attentions_local/TrainRelated/cogvideo_blocksparseattn.py:20-82),
//     done as row-index arithmetic on the caller's (un-reordered) q/k through the Gilbert rows;
//   * the Triton pooled-score kernel (TrainRelated/attn_pooling_kernel.py:17-255): per sampled row
//     the max logit of every 32-key sampled block (MFMA 32x32x16, query on the lane), rounded to the
//     storage dtype (R), the running fp32 row max m, then Po[i,j] = max_rows exp2(R - m) and the
//     storage-dtype row normalisation;
//   * transfer_attn_to_mask(mode="energy") (:177-249; wanx_blocksparseattn.py:162-233): stable
//     descending rank, fp32-accumulated cumsum rounded to the storage dtype per prefix, the first
//     crossing of storage(total * thr), clamp to [min_keep, max_keep], forced tail rows/cols.
// Nothing but Po and the mask reaches HBM (R stays in LDS).
#include <cstdlib>

#include <type_traits>

#include <rocrand/rocrand_kernel.h>

#include "vb_tiles.hpp"
#include "vb_pool.hpp"
#include "vb_pyr.hpp"
#include "vb_trace.hpp"

namespace vb {

#ifndef VB_PRED_WAVES
#define VB_PRED_WAVES 4   // sampled q-blocks (one per wave) sharing one K stream through LDS
#endif
constexpr int kPWaves = VB_PRED_WAVES;
constexpr int kPThreads = 64 * kPWaves;
constexpr int kMaxNb = 320;        // sampled blocks per side (L <= 40960 at block 128)
constexpr int kEnergyRow = kMaxNb + 16;   // LDS floats per energy-rule row buffer (keys padded to 16)
// keys per LDS tile: D=64 streams four 32-key sampled blocks per barrier (16 MFMAs per wave),
// D=128 two (also 16 MFMAs); 16 KiB tiles in a 2-deep ring at D=64 (36.5 KiB with the row-offset
// ring: four workgroups per CU) and a 3-deep ring at D=128 (52.5 KiB: three per CU)
#ifndef VB_PRED_QPW64
#define VB_PRED_QPW64 1   // D=64: sampled q-blocks per wave (2: each K fragment read feeds two MFMAs)
#endif
template <int D> constexpr int kQPW = D == 64 ? VB_PRED_QPW64 : 1;
// (with two q-blocks per wave the tile halves: the same 16 MFMAs per wave and barrier)
#ifndef VB_PRED_KPT64
#define VB_PRED_KPT64 (128 / VB_PRED_QPW64)   // D=64 keys per LDS tile
#endif
template <int D> constexpr int kKeysPerTile = (D == 64) ? VB_PRED_KPT64 : 64;
#ifndef VB_PRED_BUFS
#define VB_PRED_BUFS 3
#endif
#ifndef VB_PRED_SPLIT_ENERGY
#define VB_PRED_SPLIT_ENERGY 0   // 1: the energy rule runs as its own kernel after the scores
#endif
#ifndef VB_PRED_SCHED
#define VB_PRED_SCHED 4   // K-fragment reads issued this many MFMAs ahead (0: the compiler's order)
#endif
#ifndef VB_PRED_RCOLS
#define VB_PRED_RCOLS 3   // R-readback columns per lane per pass in the epilogue
#endif
#ifndef VB_PRED_OCC
#define VB_PRED_OCC   // e.g. __attribute__((amdgpu_waves_per_eu(4, 4))): a register budget for 4 waves/SIMD
#endif
#ifndef VB_PRED_MIN_WG
#define VB_PRED_MIN_WG 2
#endif
#ifndef VB_PRED_BUFS64
#define VB_PRED_BUFS64 2   // D=64: a 2-slot ring (36.5 KiB of LDS, four workgroups per CU), see kFusedPoolWgs64
#endif
template <int D> constexpr int kPBufs = D == 64 ? VB_PRED_BUFS64 : VB_PRED_BUFS;
#ifndef VB_PRED_GATHER
#define VB_PRED_GATHER 1   // K rows gathered by the score kernel's DMA (no sampled-row copy)
#endif
typedef int i32x4 __attribute__((ext_vector_type(4)));
#ifndef VB_FUSED_POOL_LAST
// pooling workgroups after the score workgroups: D=128 (Wan) only. Round 5, with the pipelined pass:
// Wan call 1.004-1.006x (launch span 246 -> 232 us), CogVideoX 0.945x (its pass outlasts the score
// kernel's last round); before the pipelining it measured 1-4 % slower on both
// (profiles/archive/r05_pool_pipeline_ab.log)
#define VB_FUSED_POOL_LAST 2   // 0: never, 1: both head dims, 2: D=128 only
#endif
template <int D> constexpr bool kPoolLast = VB_FUSED_POOL_LAST == 1 || (VB_FUSED_POOL_LAST == 2 && D == 128);
#ifndef VB_FUSED_POOL_WGS
// workgroups of the predictor's launch that run the pooled K/V pass (D=128, Wan). Round 5: with the
// pass pipelined (vb_pool.hpp) 512 measured 0.995x per Wan call against the serial pass, 320 0.999x,
// 192 0.995x, 128 0.981x (profiles/archive/r05_pool_pipeline_ab.log)
#define VB_FUSED_POOL_WGS 320
#endif
constexpr int kFusedPoolWgs = VB_FUSED_POOL_WGS;
#ifndef VB_FUSED_POOL_WGS64
// D=64 (CogVideoX): with four score workgroups per CU, 384 pooling workgroups leave more slots to the
// score workgroups while the pass runs (per call 1.006x against the 3-slot ring with 512; 512 with
// the 2-slot ring 0.97x, 256 0.99x; Wan keeps the 3-slot ring and 512: 0.98x with 2 slots + 384)
#define VB_FUSED_POOL_WGS64 384
#endif
constexpr int kFusedPoolWgs64 = VB_FUSED_POOL_WGS64;

// multi-level rank bands (value, [start, end) in ranks) for the fused level-mask epilogue
struct PredBands {
  int n;
  int value[8], start[8], end[8];
};

struct PredParams {
  const void* q; const void* k;
  int64_t qs[3], ks[3];
  uint8_t* q_s; uint8_t* k_s;   // sampled k rows [B,H,nb*32,D] contiguous (workspace); q_s unused
  uint16_t* rbuf;               // R [B,H,nb(q-block),nb(key block),32 rows] storage bits (workspace)
  const int32_t* rows;
  int32_t* q_off; int32_t* k_off;   // inputs, or outputs when rand_q/rand_k are given
  const float* rand_q; const float* rand_k;   // [B,H,block] uniforms (nullable): offsets drawn here
  int philox; unsigned long long philox_seed, philox_offset;   // or the uniforms generated here
  PoolTask pool;                    // pooled K/V pass run by the first n_pool workgroups (fused launch)
  PyrTask pyr;                      // or the multi-level KV pyramid pass (pool_kind 2)
  int n_pool, pool_kind;
  int level;        // 1: the epilogue writes the multi-level rank-band mask (bands lv), not the energy mask
  PredBands lv;
  int B, H, L, D, block, nb;
  float c;             // fp32(scale) * fp32(1.44269504), as the Triton kernel forms qk_scale
  float thr;
  int min_keep, max_keep, force_tail;
  void* po;
  uint8_t* mask;
  unsigned long long* count;
  int32_t* rows_kept;   // [B,H,nb] kept blocks per mask row (nullable)
  int dbg;   // diagnostic builds only (VB_DEBUG_PRED): 1 = skip epilogue, 2 = skip main loop, 4 = no MFMA, 8 = no energy rule
};

#ifndef VB_DIAG
#define VB_DIAG 0
#endif
#ifndef VB_PRED_TRACE
#define VB_PRED_TRACE 0   // diagnostic builds only (tools/diag/pred_trace.py): per-workgroup start/end times
#endif
#if VB_PRED_TRACE
__device__ TraceBuf g_pred_trace;
#define VB_TRACE_START(k) trace_start(g_pred_trace, k)
#define VB_TRACE_END() trace_end(g_pred_trace)
#else
#define VB_TRACE_START(k)
#define VB_TRACE_END()
#endif
#ifndef VB_PRED_STAMPS
#define VB_PRED_STAMPS 0   // diagnostic builds only (tools/pred_stamps.py): per-phase s_memtime sums
#endif
#if VB_PRED_STAMPS
__device__ unsigned long long g_pred_stamp[8];
__device__ __forceinline__ unsigned long long pred_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define VB_PST(var) const unsigned long long var = pred_stamp()
#else
#define VB_PST(var)
#endif

// caller row holding reordered-padded position `pos` of a (b,h) stream
__device__ __forceinline__ int sampled_row(int blk, int off, int block, int L, const int32_t* rows) {
  int pos = blk * block + off;
  pos = min(pos, L - 1);  // replicate padding (F.pad mode='replicate')
  return rows ? rows[pos] : pos;
}

// storage bits of a value already rounded to T (non-negative): orders like the value
template <class T>
__device__ __forceinline__ uint32_t storage_bits(float v) {
  const typename T::raw r = T::from_f32(v);
  uint16_t u;
  __builtin_memcpy(&u, &r, 2);
  return u;
}

// Energy rule on one row of nc normalised scores held (storage-rounded, as f32) in LDS `val`
// (room for kEnergyRow floats); `keys` is LDS scratch for kEnergyRow uint32. One full wave.
// Sort key = (storage bits << 16) | (0xFFFF - index): larger value first, ties -> lower index
// first (a stable descending sort), one unsigned compare per pair. The fp32-accumulated
// cumulative sum over the sorted values runs sequentially (bit-identical to torch's CPU cumsum)
// as one uniform chain; lane t keeps the prefix at its own position where the clamp can see it.
// The stable descending rank of each of the lane's U values (columns lane + 64u), by one wave.
template <class T, int U>
__device__ __forceinline__ void row_ranks(const float* val, uint32_t* keys, int nc, int (&rank)[U]) {
  const int lane = threadIdx.x & 63;
  uint32_t mykey[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = lane + 64 * u;
    mykey[u] = (j < nc) ? ((storage_bits<T>(val[j]) << 16) | (0xFFFFu - j)) : 0u;
    if (j < nc) keys[j] = mykey[u];
    rank[u] = 0;
  }
  const int nc16 = (nc + 15) & ~15;
  if (nc + lane < nc16) keys[nc + lane] = 0u;  // pad to 16: never greater than a real key
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  // 16 keys (four 16-byte broadcasts) per step: four LDS reads in flight
#pragma unroll 1
  for (int t16 = 0; t16 < nc16; t16 += 16) {
    u32x4 kk[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) kk[c] = *reinterpret_cast<const u32x4*>(keys + t16 + 4 * c);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int u = 0; u < U; ++u) rank[u] += (kk[c][e] > mykey[u]) ? 1 : 0;
  }
}

template <class T, int U>
__device__ __forceinline__ int energy_row_u(const float* val, uint32_t* keys, uint8_t* mrow, int nc, float thr,
                            int min_keep, int max_keep, int force_cols, bool force_all) {
  const int lane = threadIdx.x & 63;
  int rank[U];
  row_ranks<T, U>(val, keys, nc, rank);
  const int nc16 = (nc + 15) & ~15;
  // scatter values into sorted order (reuse `keys` as float storage after a wave barrier)
  __builtin_amdgcn_wave_barrier();
  float* sorted = reinterpret_cast<float*>(keys);
  float vals[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = lane + 64 * u;
    vals[u] = (j < nc) ? val[j] : 0.f;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (lane + 64 * u < nc) sorted[rank[u]] = vals[u];
  if (nc + lane < nc16) sorted[nc + lane] = 0.f;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  // fp32 sequential cumulative sum (torch's CPU cumsum) as ONE chain, identical in every lane,
  // over the sorted values read by 16-byte LDS broadcasts. The clamped count k only depends on the
  // first min(nc, max_keep) prefixes (cum is non-decreasing, k = #prefixes below the threshold,
  // then clamped to max_keep), so lane t records the prefix at position t + 64u only there; the
  // total is the chain's end.
  const int need = min(nc, max_keep);
  float acc = 0.f;
  float pre[U];
  const float4* s4 = reinterpret_cast<const float4*>(sorted);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    pre[u] = 0.f;
    if (64 * u >= nc16) break;
    if (64 * u < need) {
#pragma unroll 4
      for (int i4 = 0; i4 < 16; ++i4) {
        if (64 * u + 4 * i4 >= nc16) break;
        const float4 w = s4[16 * u + i4];
        const int i = 4 * i4;
        acc += w.x; pre[u] = (lane == i) ? acc : pre[u];
        acc += w.y; pre[u] = (lane == i + 1) ? acc : pre[u];
        acc += w.z; pre[u] = (lane == i + 2) ? acc : pre[u];
        acc += w.w; pre[u] = (lane == i + 3) ? acc : pre[u];
      }
    } else {
#pragma unroll 4
      for (int i4 = 0; i4 < 16; ++i4) {
        if (64 * u + 4 * i4 >= nc16) break;
        const float4 w = s4[16 * u + i4];
        acc += w.x; acc += w.y; acc += w.z; acc += w.w;   // padding past nc adds zeros
      }
    }
  }
  const float total = round_to<T>(acc);   // cum_energy[..., -1]
  const float th = round_to<T>(total * thr);
  int k = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int t = lane + 64 * u;
    k += __popcll(__ballot(t < need && round_to<T>(pre[u]) < th));
  }
  // all `need` prefixes below the threshold: the crossing is at or past need (k = need, which the
  // clamp maps like the reference's first crossing / nc)
  k = min(max(k, min_keep), max_keep);
  int kept = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = lane + 64 * u;
    if (j < nc) {
      const bool keep = force_all || rank[u] < k || j >= nc - force_cols;
      mrow[j] = keep ? 1 : 0;
      kept += keep;
    }
  }
  for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o);
  return kept;
}
// U = values per lane, the smallest that covers the row (ranks cost nc * U compares per lane)
template <class T>
__device__ __forceinline__ int energy_row(const float* val, uint32_t* keys, uint8_t* mrow, int nc, float thr,
                          int min_keep, int max_keep, int force_cols, bool force_all) {
  switch ((nc + 63) >> 6) {
    case 1: return energy_row_u<T, 1>(val, keys, mrow, nc, thr, min_keep, max_keep, force_cols, force_all);
    case 2: return energy_row_u<T, 2>(val, keys, mrow, nc, thr, min_keep, max_keep, force_cols, force_all);
    case 3: return energy_row_u<T, 3>(val, keys, mrow, nc, thr, min_keep, max_keep, force_cols, force_all);
    case 4: return energy_row_u<T, 4>(val, keys, mrow, nc, thr, min_keep, max_keep, force_cols, force_all);
    default: return energy_row_u<T, (kMaxNb + 63) / 64>(val, keys, mrow, nc, thr, min_keep, max_keep, force_cols,
                                                           force_all);
  }
}

// Multi-level rank bands (transfer_attn_to_mask, Triton/cogvideo_newattn.py:154-207; vb_level_mask's
// rule, vb_ml.hip) on one row of normalised scores in LDS `val`: the column of stable descending rank
// r gets the value of the last band whose [start, end) holds r (0 if none); the last two rows and
// columns are forced to level 1. Ranks as the energy rule's (same keys), so ties go to the lower column.
template <class T, int U>
__device__ __forceinline__ void level_row_u(const float* val, uint32_t* keys, uint8_t* mrow, int nc, int row,
                                            const PredBands& lv) {
  const int lane = threadIdx.x & 63;
  int rank[U];
  row_ranks<T, U>(val, keys, nc, rank);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = lane + 64 * u;
    int l = 0;
    for (int b = 0; b < lv.n; ++b)
      if (rank[u] >= lv.start[b] && rank[u] < lv.end[b]) l = lv.value[b];
    if (j >= nc - 2 || row >= nc - 2) l = 1;
    if (j < nc) mrow[j] = (uint8_t)l;
  }
}
template <class T>
__device__ __forceinline__ void level_row(const float* val, uint32_t* keys, uint8_t* mrow, int nc, int row,
                                          const PredBands& lv) {
  switch ((nc + 63) >> 6) {
    case 1: return level_row_u<T, 1>(val, keys, mrow, nc, row, lv);
    case 2: return level_row_u<T, 2>(val, keys, mrow, nc, row, lv);
    case 3: return level_row_u<T, 3>(val, keys, mrow, nc, row, lv);
    case 4: return level_row_u<T, 4>(val, keys, mrow, nc, row, lv);
    default: return level_row_u<T, (kMaxNb + 63) / 64>(val, keys, mrow, nc, row, lv);
  }
}

// random_sample_tokens' topk (cogvideo_blocksparseattn.py:45-46) by one wave: the indices of the
// `keep` largest of n <= 256 uniforms r (global), in descending order of value, ties -> lower index
// first, written to dst[rank] (LDS or global). `sv` is LDS scratch for n floats.
__device__ __forceinline__ void topk_wave_lds(int n, int keep, int32_t* dst, const float* sv);
__device__ __forceinline__ void topk_wave(const float* r, int n, int keep, int32_t* dst, float* sv) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < n; i += 64) sv[i] = r[i];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  topk_wave_lds(n, keep, dst, sv);
}

// torch.rand(B,H,1,block) on a device generator at Philox state (seed, offset), element base + t of
// the draw for t < n (PyTorch's uniform_: distribution_elementwise_grid_stride_kernel with one
// grid-stride pass, hiprand_init(seed, element, offset), the x of hiprand_uniform4, 1.0 -> 0.0),
// written to LDS sv[t] by one wave.
__device__ __forceinline__ void philox_draw_wave(unsigned long long seed, unsigned long long offset,
                                                 long long base, int n, float* sv) {
  const int lane = threadIdx.x & 63;
  for (int t = lane; t < n; t += 64) {
    rocrand_state_philox4x32_10 st;
    rocrand_init(seed, (unsigned long long)(base + t), offset, &st);
    const float u = rocrand_uniform4(&st).x;
    sv[t] = u == 1.0f ? 0.0f : u;
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
}

// the rank loop of topk_wave on draws already in LDS sv[0..n)
__device__ __forceinline__ void topk_wave_lds(int n, int keep, int32_t* dst, const float* sv) {
  const int lane = threadIdx.x & 63;
  // the rank loop reads 4 draws per 16-byte LDS broadcast, 8 reads in flight: a one-float loop was
  // LDS-latency bound (~6 us of sample_rows_kernel's 10 us at the CogVideoX shape)
  const float4* s4 = reinterpret_cast<const float4*>(sv);
  const int n4 = n >> 2;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const float v = i < n ? sv[i] : 0.f;
    int rank = 0;
#pragma unroll 8
    for (int j4 = 0; j4 < n4; ++j4) {
      const float4 w = s4[j4];
      const int j = 4 * j4;
      rank += (w.x > v || (w.x == v && j < i)) ? 1 : 0;
      rank += (w.y > v || (w.y == v && j + 1 < i)) ? 1 : 0;
      rank += (w.z > v || (w.z == v && j + 2 < i)) ? 1 : 0;
      rank += (w.w > v || (w.w == v && j + 3 < i)) ? 1 : 0;
    }
    for (int j = 4 * n4; j < n; ++j) {
      const float w = sv[j];
      rank += (w > v || (w == v && j < i)) ? 1 : 0;
    }
    if (i < n && rank < keep) dst[rank] = i;
  }
}

// Sampled rows of k, gathered once into contiguous [B,H,nb*32,D] (the q fragments are gathered by the
// predictor's prologue directly, one row per lane):
// row j*32 + t of (b,h) = reordered position min(j*block + off[b,h,t], L-1) (replicate padding),
// read at the caller's row rows[pos]. The predictor then streams K by plain LDS-DMA.
// grid (row chunks, B*H). With rand_q/rand_k the offsets are drawn here first (topk_wave: one launch
// instead of two) and the first chunk of every (b,h) writes them out for the score kernel.
template <class T>
__global__ void __launch_bounds__(256) sample_rows_kernel(const PredParams p) {
  __shared__ alignas(16) float sv[2][256];
  __shared__ int32_t koff_s[32];
  const int bh = blockIdx.y;
  const int wave = threadIdx.x >> 6;
  const int32_t* koff = p.k_off + (int64_t)bh * 32;
  if (p.philox) {   // the two torch.rand draws generated here: q at offset, k at offset + 4
    if (wave == 0) {
      philox_draw_wave(p.philox_seed, p.philox_offset + 4, (long long)bh * p.block, p.block, sv[0]);
      topk_wave_lds(p.block, 32, koff_s, sv[0]);
    }
    if (blockIdx.x == 0 && wave == 1) {
      philox_draw_wave(p.philox_seed, p.philox_offset, (long long)bh * p.block, p.block, sv[1]);
      topk_wave_lds(p.block, 32, p.q_off + (int64_t)bh * 32, sv[1]);
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < 32) p.k_off[(int64_t)bh * 32 + threadIdx.x] = koff_s[threadIdx.x];
    koff = koff_s;
  } else if (p.rand_k) {
    if (wave == 0) topk_wave(p.rand_k + (int64_t)bh * p.block, p.block, 32, koff_s, sv[0]);
    if (blockIdx.x == 0 && wave == 1)
      topk_wave(p.rand_q + (int64_t)bh * p.block, p.block, 32, p.q_off + (int64_t)bh * 32, sv[1]);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < 32) p.k_off[(int64_t)bh * 32 + threadIdx.x] = koff_s[threadIdx.x];
    koff = koff_s;
  }
  // one thread per sampled row: the two index loads once, then D/8 independent 16-byte copies
  const int jt = blockIdx.x * blockDim.x + threadIdx.x;
  if (jt >= p.nb * 32) return;
  const int b = bh / p.H, h = bh % p.H;
  int pos = min((jt >> 5) * p.block + koff[jt & 31], p.L - 1);
  if (p.rows) pos = p.rows[pos];
  if (VB_PRED_GATHER) {   // the score kernel gathers the rows: only their byte offsets in the (b,h) slice
    reinterpret_cast<int32_t*>(p.k_s)[(int64_t)bh * p.nb * 32 + jt] = (int32_t)((int64_t)pos * p.ks[2] * 2);
    return;
  }
  const u32x4* src = reinterpret_cast<const u32x4*>(reinterpret_cast<const uint8_t*>(p.k) +
                                                    2 * (b * p.ks[0] + h * p.ks[1] + (int64_t)pos * p.ks[2]));
  u32x4* dst = reinterpret_cast<u32x4*>(p.k_s + ((int64_t)bh * p.nb * 32 + jt) * p.D * 2);
  if (p.D == 64) {
    u32x4 x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = src[c];
#pragma unroll
    for (int c = 0; c < 8; ++c) dst[c] = x[c];
  } else {
    u32x4 x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = src[c];
#pragma unroll
    for (int c = 0; c < 16; ++c) dst[c] = x[c];
  }
}

template <int D, class T, bool kEnergy>
__global__ void __launch_bounds__(kPThreads, VB_PRED_MIN_WG) VB_PRED_OCC mask_predict_kernel(const PredParams p) {
  constexpr int KS = D / 16;
  constexpr int kRowB = D * 2;                        // bytes per key row
  constexpr int kKT = kKeysPerTile<D> / 32;          // sampled key blocks per tile
  constexpr int kTileBytes = kKeysPerTile<D> * kRowB;
  constexpr int kRowsPerInst = 1024 / kRowB;          // rows one 1-KiB LDS-DMA wave-instruction fills
  constexpr int kInstPerWave = kTileBytes / 1024 / kPWaves;
  constexpr int kBufs = kPBufs<D>;                    // tile t read, the younger ones in flight
  constexpr int KQ = kQPW<D>;                         // sampled q-blocks per wave
  constexpr int kSt = KQ * (kKT / 2);                 // R stores per wave and tile
  // LDS: m [4][32] f32 | K tiles x4 (after the main loop: per-wave row scratch). The per-row
  // block maxima R go to a global scratch in [key block][32 rows] order (as the Triton kernel keeps
  // R in HBM): a tile's two columns are one contiguous 128-byte store, and the LDS stays small
  // enough for 3 workgroups per CU at any nb.
  // The first n_pool workgroups of the launch run the pooled K/V pass (HBM-bound) beside the score
  // workgroups (MFMA-bound): one launch, no second stream or events. n_pool is a multiple of 8, so
  // the score workgroups keep their XCD (blockIdx % 8).
  // kPoolLast<D>: the pooling workgroups come after the score workgroups instead, where they fill the
  // score kernel's partial last round.
  const bool pool_wg = kPoolLast<D> ? (int)blockIdx.x >= (int)gridDim.x - p.n_pool : (int)blockIdx.x < p.n_pool;
  if (pool_wg) {
    VB_TRACE_START(1);
    const int pw = kPoolLast<D> ? (int)blockIdx.x - ((int)gridDim.x - p.n_pool) : (int)blockIdx.x;
    const int64_t i0 = (int64_t)pw * blockDim.x + threadIdx.x, st = (int64_t)p.n_pool * blockDim.x;
    if (p.pool_kind == 2) kv_pyramid_span<D, T>(p.pyr, i0, st);
    else pool_kv_span<T>(p.pool, i0, st);
    VB_TRACE_END();
    return;
  }
  VB_TRACE_START(0);
  const int wg = kPoolLast<D> ? (int)blockIdx.x : (int)blockIdx.x - p.n_pool;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int nb = p.nb;
  float* mrow_s = reinterpret_cast<float*>(smem);
  uint8_t* ktile = smem + kPWaves * KQ * 32 * 4;
  float* rowbuf = reinterpret_cast<float*>(ktile);  // [4][2][kEnergyRow], reused after the loop

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;
  // XCD-aware order: give each XCD a contiguous range of (head, q-group) work, so a head's sampled
  // keys are re-read from that XCD's own L2. Placement only affects speed.
  const int nqg = (nb + kPWaves * KQ - 1) / (kPWaves * KQ);
  const int lin = xcd_linear(wg, nqg * p.B * p.H);
  const int bh = lin / nqg;
  int qbs[KQ];   // this wave's sampled q-blocks
#pragma unroll
  for (int e = 0; e < KQ; ++e) qbs[e] = (lin % nqg) * kPWaves * KQ + wave * KQ + e;
#if !VB_PRED_GATHER
  const int64_t slice = (int64_t)nb * 32 * kRowB;   // bytes of one (b,h) sampled stream
#endif

  // Q fragment of this lane's sampled row (B operand of S^T = K_s . Q_s^T), gathered straight from
  // the caller's q: reordered-padded position qb*block + q_off[l32] (replicate padding) at row rows[pos]
  typename T::vec8 qf[KQ][KS];
#pragma unroll
  for (int e = 0; e < KQ; ++e) {
    const int b = bh / p.H, h = bh % p.H;
    const int qrow = sampled_row(qbs[e] < nb ? qbs[e] : 0, p.q_off[(int64_t)bh * 32 + l32], p.block, p.L, p.rows);
    const uint8_t* qp = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + (int64_t)qrow * p.qs[2]);
#pragma unroll
    for (int s = 0; s < KS; ++s)
      qf[e][s] = *reinterpret_cast<const typename T::vec8*>(qp + (16 * s + 8 * half) * 2);
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(qf[e][s]));  // see vb_attn_fwd.hip
  }
  // K tiles by LDS-DMA from the contiguous sampled stream: a buffer descriptor per (b,h), each
  // lane's fixed (row, swizzled chunk) as voffset, the tile's first row as soffset. Rows past the
  // stream (a partial last tile) read as zeros and are never used.
#if VB_PRED_GATHER
  // Gather mode: the sampling launch wrote only the byte offsets of the sampled rows within the
  // (b,h) slice of k (int32 table [bh][nb*32]); K tiles are gathered straight from k. Per tile each
  // wave DMAs the offsets of its own rows into a small LDS ring two tiles ahead (one 4-byte lane
  // each, ordered so that lane L's four rows are 16 contiguous bytes), reads them back and issues
  // the row DMAs with per-lane voffsets. 27 MB of row copies per CogVideoX call are not made.
  static_assert(kBufs == 2 || kBufs == 3, "the gather pipeline's vmcnt counts assume a 2- or 3-slot K ring");
  constexpr int kChunks = kRowB / 16;
  const uint8_t* kslice = reinterpret_cast<const uint8_t*>(p.k) + 2 * ((bh / p.H) * p.ks[0] + (bh % p.H) * p.ks[1]);
  const srd_t ksrd = make_srd(kslice, (int)((int64_t)(p.L - 1) * p.ks[2] * 2 + kRowB));
  const srd_t isrd = make_srd(reinterpret_cast<const int32_t*>(p.k_s) + (int64_t)bh * nb * 32, nb * 32 * 4);
  uint8_t* ibuf = ktile + kBufs * kTileBytes + wave * 256;   // [4 tiles][4 waves][64 dwords]
  int cv[kInstPerWave];   // the lane's swizzled chunk within its row, per DMA instruction
#pragma unroll
  for (int i = 0; i < kInstPerWave; ++i) {
    const int r = (wave * kInstPerWave + i) * kRowsPerInst + lane / kChunks;
    const int sw = (D == 64) ? ((r >> 1) & 7) : (r & 15);
    cv[i] = 16 * ((lane % kChunks) ^ sw);
  }
  // offset-DMA lane 4j + i fetches row (wave*kIPW + i)*kRowsPerInst + j of the tile (lanes past the
  // wave's rows repeat the last one)
  const int ivoff = 4 * ((wave * kInstPerWave + (lane & 3)) * kRowsPerInst + min(lane >> 2, kRowsPerInst - 1));
#else
  const srd_t ksrd = make_srd(p.k_s + bh * slice, (int)slice);
  int voff[kInstPerWave];
#pragma unroll
  for (int i = 0; i < kInstPerWave; ++i) {
    const int r = (wave * kInstPerWave + i) * kRowsPerInst + lane / (kRowB / 16);
    const int sl = lane % (kRowB / 16);
    const int sw = (D == 64) ? ((r >> 1) & 7) : (r & 15);
    voff[i] = r * kRowB + 16 * (sl ^ sw);
  }
#endif
  float m[KQ];
#pragma unroll
  for (int e = 0; e < KQ; ++e) m[e] = -INFINITY;
  __syncthreads();   // all plain global loads retired before the DMA pipeline

  const int ntiles = (VB_DIAG && (p.dbg & 2)) ? 0 : (nb + kKT - 1) / kKT;
  // K tile t by LDS-DMA (global_load_lds_dwordx4): the LDS image is written linearly (1 KiB per
  // wave-instruction), so the 16-byte-chunk XOR swizzle of the image is applied to each lane's
  // SOURCE address: LDS slot `sl` of row r holds chunk sl ^ sw(r).
#if VB_PRED_GATHER
  // offsets of tile t's rows -> LDS ring slot t & 3 (one instruction per wave; past the table: 0).
  // Four slots: the prologue has I0..I2 in flight at once, a body reads I(t+2) while I(t+3) lands.
  auto issue_idx = [&](int t) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(isrd.base), (short)0, isrd.bytes, 0x00020000),
        (__attribute__((address_space(3))) void*)(ibuf + (t & 3) * (kPWaves * 256)), 4, ivoff,
        __builtin_amdgcn_readfirstlane(t * kKeysPerTile<D> * 4), 0, 0);
  };
  // rows of tile t (offsets already in LDS) -> K ring slot t % kBufs
  auto issue = [&](int t) __attribute__((always_inline)) {
    uint8_t* dst = ktile + (t % kBufs) * kTileBytes;
    const i32x4 o = *reinterpret_cast<const i32x4*>(ibuf + (t & 3) * (kPWaves * 256) + 16 * (lane / kChunks));
#pragma unroll
    for (int i = 0; i < kInstPerWave; ++i) dma16(ksrd, dst + (wave * kInstPerWave + i) * 1024, o[i] + cv[i], 0);
  };
#else
  auto issue = [&](int t) __attribute__((always_inline)) {
    uint8_t* dst = ktile + (t % kBufs) * kTileBytes;
#pragma unroll
    for (int i = 0; i < kInstPerWave; ++i)
      dma16(ksrd, dst + (wave * kInstPerWave + i) * 1024, voff[i], t * kTileBytes);
  };
#endif
  // loop-invariant lane addresses of the K fragment reads (the swizzle depends on the lane's row
  // bits only), so every read of every slot is base + compile-time immediate
  int k_lane[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int sw = (D == 64) ? ((l32 >> 1) & 7) : (l32 & 15);
    k_lane[ks] = l32 * kRowB + 16 * ((2 * ks + half) ^ sw);
  }
  uint16_t* Rqs[KQ];   // this wave's q-blocks' R slices
  srd_t rsrd[KQ];
#pragma unroll
  for (int e = 0; e < KQ; ++e) {
    Rqs[e] = p.rbuf + ((int64_t)bh * nb + (qbs[e] < nb ? qbs[e] : 0)) * nb * 32;
    rsrd[e] = make_srd(Rqs[e], qbs[e] < nb ? nb * 64 : 0);
  }
#if VB_PRED_GATHER
  // Issue order: I0 I1 I2 K0 K1, then per body t: I(t+3) K(t+2) [compute] S(t) — every DMA is
  // issued, past the last tile too (offsets past the table read 0: row 0 into a slot no tile reads
  // any more), so the counts below are constant. Body t needs K(t) and I(t+2); younger than I(t+2)
  // are K(t+1) and S(t-1) (for t = 0: only K1), so K(t+1) stays in flight.
  // 2-slot ring (36 KiB of LDS: four workgroups per CU): I0 I1 K0, then per body t: I(t+2) K(t+1)
  // [compute] S(t); K(t+1) can only go after the barrier that frees its slot, so a body waits for
  // its own K(t) with only S(t-1) younger.
  if (ntiles > 0) {
    if constexpr (kBufs == 2) {
      issue_idx(0);
      issue_idx(1);
      VB_WAIT_VMCNT(1);
      asm volatile("" ::: "memory");
      issue(0);
    } else {
      issue_idx(0);
      issue_idx(1);
      issue_idx(2);
      VB_WAIT_VMCNT(2);
      asm volatile("" ::: "memory");   // the offsets' LDS reads stay behind the wait
      issue(0);
      VB_WAIT_VMCNT(1 + kInstPerWave);
      asm volatile("" ::: "memory");
      issue(1);
    }
  }
#else
  for (int t = 0; t < kBufs - 1 && t < ntiles; ++t) issue(t);
#endif
#if VB_PRED_STAMPS
  unsigned long long pst[4] = {0, 0, 0, 0};
#endif
  auto halfmax = [&](const f32x16& a) __attribute__((always_inline)) -> float {
    float y = fmaxf(fmaxf(a[0], a[1]), a[2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) y = fmaxf(fmaxf(y, a[r]), a[r + 1]);
    return fmaxf(y, a[15]);
  };
  auto body = [&](int t, auto U) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    VB_PST(b0);
#if VB_PRED_GATHER
    if constexpr (kBufs == 2) {
      if (t == 0) VB_WAIT_VMCNT(0);
      else VB_WAIT_VMCNT(kSt);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue_idx(t + 2);
      issue(t + 1);
    } else {
      if (t == 0) VB_WAIT_VMCNT(kInstPerWave);
      else VB_WAIT_VMCNT(kInstPerWave + kSt);
      VB_PST(b1);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      VB_PST(b2);
      issue_idx(t + 3);
      issue(t + 2);
      VB_PST(b3);
#if VB_PRED_STAMPS
      pst[0] += b1 - b0;
      pst[1] += b2 - b1;
      pst[2] += b3 - b2;
#endif
    }
#else
    // retire this wave's DMA of tile t, then the barrier makes every wave's part visible and
    // guarantees tile t-1's buffer is no longer being read. vmcnt counts the R stores too, in issue
    // order: younger than DMA(t) are the stores of the (up to kBufs-1) bodies since it was issued
    // and the DMAs of tiles t+1 .. t+kBufs-2. Every body issues exactly kSt stores (see below), so
    // the count is exact and the younger tiles' DMAs stay in flight.
    const int nst = min(t, kBufs - 1);
    const int ndma = max(0, min(kBufs - 2, ntiles - 1 - t));
    if (nst == kBufs - 1 && ndma == kBufs - 2) VB_WAIT_VMCNT((kBufs - 1) * kSt + (kBufs - 2) * kInstPerWave);
    else wait_vmcnt_upto<kBufs * kSt + kBufs * kInstPerWave>(nst * kSt + ndma * kInstPerWave);
    __builtin_amdgcn_s_barrier();
    if (t + kBufs - 1 < ntiles) issue(t + kBufs - 1);
#endif
    const uint8_t* kl = ktile + u * kTileBytes;
    if (VB_DIAG && (p.dbg & 4)) return;   // diagnostic: stream the K tiles only
    // one accumulator per 32-key block: the MFMAs of block kt+1 do not wait for the row-max
    // reads of block kt (a shared accumulator serialises MFMA -> s_nop -> VALU -> MFMA)
    f32x16 sc[KQ][kKT];
#pragma unroll
    for (int kt = 0; kt < kKT; ++kt) {
      typename T::vec8 kf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        kf[ks] = *reinterpret_cast<const typename T::vec8*>(kl + kt * 32 * kRowB + k_lane[ks]);
#pragma unroll
      for (int e = 0; e < KQ; ++e)
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[e][kt][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int e = 0; e < KQ; ++e) sc[e][kt] = T::mfma32(kf[ks], qf[e][ks], sc[e][kt]);
    }
#if VB_PRED_SCHED
    // Pin the issue order: each K-fragment read VB_PRED_SCHED MFMAs ahead of the MFMA that consumes
    // it (left alone, hipcc reuses one fragment register and serialises read -> wait -> MFMA).
#pragma unroll
    for (int i = 0; i < VB_PRED_SCHED; ++i) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
#pragma unroll
    for (int i = 0; i < kKT * KS; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x8, KQ, 0);
      if (i + VB_PRED_SCHED < kKT * KS) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
#endif
    // row maxima, two 32-key blocks per v_permlane32_swap: after the swap lanes 0-31 hold block
    // 2pr's full row max and lanes 32-63 block 2pr+1's (the halves of each block's C tile meet)
    const int j0 = kKT * t;
    constexpr int kPairs = kKT / 2;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
    float mxp[kKT / 2];
#pragma unroll
    for (int pr = 0; pr < kPairs; ++pr) {
      const float x0 = halfmax(sc[q][2 * pr]), x1 = halfmax(sc[q][2 * pr + 1]);
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x0), __float_as_uint(x1), false, false);
      mxp[pr] = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * p.c;   // tl.max(qk, 1) * qk_scale
    }
    if (j0 + kKT > nb) {   // partial last tile: blocks past nb take no part (their rows are zeros)
      asm volatile("");
#pragma unroll
      for (int pr = 0; pr < kPairs; ++pr)
        if (j0 + 2 * pr + half >= nb) mxp[pr] = -INFINITY;
    }
#pragma unroll
    for (int pr = 0; pr < kPairs; ++pr) m[q] = fmaxf(m[q], mxp[pr]);   // this half's blocks; halves meet below
    // R[j][row]: lane (half, row) stores block j0 + 2pr + half, so one store writes 128 contiguous
    // bytes. Issued unconditionally (kSt per body, the vmcnt arithmetic above relies on it): blocks
    // past nb fall outside the descriptor and an inactive q-block's descriptor is empty, so the
    // hardware drops those lanes.
#pragma unroll
    for (int pr = 0; pr < kPairs; ++pr) store16(rsrd[q], (uint16_t)storage_bits<T>(mxp[pr]), lane * 2, (j0 + 2 * pr) * 64);
    }

#if VB_PRED_STAMPS
    VB_PST(b4);
    pst[3] += b4 - b0;
#endif
  };
  for (int t0 = 0; t0 < ntiles; t0 += kBufs) {
    body(t0, std::integral_constant<int, 0>{});
    if (t0 + 1 < ntiles) body(t0 + 1, std::integral_constant<int, 1>{});
    if constexpr (kBufs > 2)
      if (t0 + 2 < ntiles) body(t0 + 2, std::integral_constant<int, 2 % kBufs>{});
    if constexpr (kBufs > 3)
      if (t0 + 3 < ntiles) body(t0 + 3, std::integral_constant<int, 3>{});
  }
  static_assert(kBufs >= 2 && kBufs <= 4, "the loop body is instantiated once per ring slot");

#if VB_PRED_GATHER
  VB_WAIT_VMCNT(0);   // the DMAs issued past the last tile land before the epilogue reuses the LDS
#endif
#if VB_PRED_STAMPS
  VB_PST(e0);
#endif
#pragma unroll
  for (int e = 0; e < KQ; ++e) {
    m[e] = max_xor32(m[e]);   // the two halves saw alternate key blocks
    if (half == 0) mrow_s[(wave * KQ + e) * 32 + l32] = m[e];
  }
  __syncthreads();
  if (VB_DIAG && (p.dbg & 1)) return;

  // Po[qb, j] = storage(max_r exp2(R[r][j] - m_r)) = storage(exp2(max_r (R[r][j] - m_r)))
  // (exp2 and the rounding are monotone), then the storage-dtype row normalisation; one q-block
  // after the other (the wave's row scratch is reused)
  float* val = rowbuf + wave * 2 * (kEnergyRow);
  uint32_t* keys = reinterpret_cast<uint32_t*>(val + kEnergyRow);
  auto epilogue = [&](const int qb, const uint16_t* Rq, const float* mw) __attribute__((always_inline)) {
    // this wave's R columns were stored by its own lanes: wait for them and drop any stale L1 line
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    float mreg[32];
#pragma unroll
    for (int r = 0; r < 32; r += 4) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(mw + r);
#pragma unroll
      for (int e = 0; e < 4; ++e) mreg[r + e] = x[e];
    }
    float part = 0.f;
    // VB_PRED_RCOLS columns per lane per pass (4 loads each in flight): the block's 32 row maxima
    // are 64 contiguous bytes
    constexpr int kRC = VB_PRED_RCOLS;
    for (int j0 = 0; j0 < nb; j0 += 64 * kRC) {
      u32x4 w[kRC][4];
#pragma unroll
      for (int h = 0; h < kRC; ++h) {
        const int jj = min(j0 + 64 * h + lane, nb - 1);
#pragma unroll
        for (int c = 0; c < 4; ++c) w[h][c] = reinterpret_cast<const u32x4*>(Rq + jj * 32)[c];
      }
#pragma unroll
      for (int h = 0; h < kRC; ++h) {
        const int j = j0 + 64 * h + lane;
        float cm = -INFINITY;
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 8 * c + 2 * e;
            cm = max3f(cm, T::bits_to_f32((uint16_t)(w[h][c][e] & 0xFFFF)) - mreg[r],
                       T::bits_to_f32((uint16_t)(w[h][c][e] >> 16)) - mreg[r + 1]);
          }
        cm = round_to<T>(exp2_fast(cm));
        if (j < nb) {
          val[j] = cm;
          part += cm;
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    const float tot = round_to<T>(part);
    typename T::raw* po = reinterpret_cast<typename T::raw*>(p.po) + ((int64_t)bh * nb + qb) * nb;
    for (int j = lane; j < nb; j += 64) {
      const float v = round_to<T>(val[j] / tot);
      val[j] = v;
      po[j] = T::from_f32(v);
    }
#if VB_PRED_STAMPS
    {
      VB_PST(e1);
      if (lane == 0) {
        for (int i = 0; i < 4; ++i) atomicAdd(&g_pred_stamp[i], pst[i]);
        atomicAdd(&g_pred_stamp[4], e1 - e0);
        atomicAdd(&g_pred_stamp[5], 1ull);
      }
    }
#endif
    if (!kEnergy || p.mask == nullptr) return;   // scores only (energy rule elsewhere / not wanted)
    if (VB_DIAG && (p.dbg & 8)) return;   // diagnostic: no energy rule (Po written)
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    uint8_t* mrow = p.mask + ((int64_t)bh * nb + qb) * nb;
    if (p.level) {   // the multi-level path's rank bands instead of the energy rule
      level_row<T>(val, keys, mrow, nb, qb, p.lv);
      return;
    }
    const bool force_all = p.force_tail > 0 && qb >= nb - p.force_tail;
    const int kept = energy_row<T>(val, keys, mrow, nb, p.thr, p.min_keep, p.max_keep, p.force_tail, force_all);
    if (p.count && lane == 0) atomicAdd(p.count, (unsigned long long)kept);
    if (p.rows_kept && lane == 0) p.rows_kept[(int64_t)bh * nb + qb] = kept;
  };
#pragma unroll
  for (int e = 0; e < KQ; ++e)
    if (qbs[e] < nb) epilogue(qbs[e], Rqs[e], mrow_s + (wave * KQ + e) * 32);
  VB_TRACE_END();
}

// random_sample_tokens' topk (cogvideo_blocksparseattn.py:45-46): for every row of `n` uniform draws,
// the indices of the `keep` largest values in descending order of value (ties -> lower index
// first). One wave per row; blockIdx.y selects the q or the k draws.
__global__ void __launch_bounds__(256) topk_offsets_kernel(const float* rq, const float* rk, int rows, int n,
                                                           int keep, int32_t* oq, int32_t* ok) {
  __shared__ alignas(16) float buf[4][256];
  const int wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows || n > 256) return;
  topk_wave((blockIdx.y ? rk : rq) + (int64_t)row * n, n, keep, (blockIdx.y ? ok : oq) + (int64_t)row * keep, buf[wave]);
}

template <class T>
__global__ void __launch_bounds__(256) energy_mask_kernel(const void* po, int rows_total, int nc, float thr,
                                                          int min_keep, int max_keep, int force_tail, int nr,
                                                          uint8_t* mask, unsigned long long* count) {
  __shared__ __attribute__((aligned(16))) float buf[4][2 * (kEnergyRow)];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows_total) return;
  const typename T::raw* src = reinterpret_cast<const typename T::raw*>(po) + (int64_t)row * nc;
  float* val = buf[wave];
  for (int j = lane; j < nc; j += 64) val[j] = T::to_f32(src[j]);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const int i = row % nr;
  const bool force_all = force_tail > 0 && i >= nr - force_tail;
  const int kept = energy_row<T>(val, reinterpret_cast<uint32_t*>(val + kEnergyRow), mask + (int64_t)row * nc, nc,
                                 thr, min_keep, max_keep, force_tail, force_all);
  if (count && lane == 0) atomicAdd(count, (unsigned long long)kept);
}

static size_t predict_smem_bytes(int nb, int D) {
  (void)nb;
  const size_t tiles = D == 64 ? (size_t)kPBufs<64> * kKeysPerTile<64> * 64 * 2
                               : (size_t)kPBufs<128> * kKeysPerTile<128> * 128 * 2;
  const size_t scratch = (size_t)kPWaves * 2 * (kEnergyRow) * 4;
  const size_t ring = VB_PRED_GATHER ? 4 * kPWaves * 256 : 0;   // gather mode: the row-offset ring
  const size_t mrow = (size_t)kPWaves * (D == 64 ? kQPW<64> : kQPW<128>) * 32 * 4;
  return mrow + (tiles + ring > scratch ? tiles + ring : scratch);
}

// workspace: sampled k rows (gather mode: their int32 byte offsets) | R
static uint64_t predict_rows_bytes(int B, int H, int L, int D) {
  const int nb = (L + 127) / 128;
  return (uint64_t)B * H * nb * 32 * (VB_PRED_GATHER ? 4 : D * 2);
}
static uint64_t predict_ws_bytes(int B, int H, int L, int D) {
  const uint64_t nb = (L + 127) / 128;
  return predict_rows_bytes(B, H, L, D) + (uint64_t)B * H * nb * nb * 32 * 2;
}

// B*H*block bound of the in-kernel Philox draws (see vb_mask_predict), per device, cached
static int64_t philox_x_only_numel() {
  static int64_t cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
  if (dev < 64 && cache[dev] > 0) return cache[dev];
  int cus = 0, thr = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipDeviceGetAttribute(&thr, hipDeviceAttributeMaxThreadsPerMultiProcessor, dev) != hipSuccess)
    return 0;
  const int64_t n = (int64_t)cus * thr;
  if (dev < 64) cache[dev] = n;
  return n;
}

template <int D, class T>
static int launch_predict(const PredParams& p, hipStream_t stream, hipEvent_t staged) {
  const size_t smem = predict_smem_bytes(p.nb, D);
  auto kern = mask_predict_kernel<D, T, !VB_PRED_SPLIT_ENERGY>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)smem) != hipSuccess)
    return fail(VB_ERR_LAUNCH, "mask_predict: cannot reserve LDS");
  hipLaunchKernelGGL(sample_rows_kernel<T>, dim3((unsigned)((p.nb * 32 + 255) / 256), (unsigned)(p.B * p.H)), dim3(256),
                     0, stream, p);
  if (int rc = check_launch("sample_rows_kernel")) return rc;
  if (staged && hipEventRecord(staged, stream) != hipSuccess) return fail(VB_ERR_LAUNCH, "vb_mask_predict: hipEventRecord failed");
  constexpr int qpw = kPWaves * kQPW<D>;   // sampled q-blocks per workgroup
  const dim3 grid(((p.nb + qpw - 1) / qpw) * p.B * p.H + p.n_pool);
  hipLaunchKernelGGL(kern, grid, dim3(kPThreads), smem, stream, p);
  if (int rc = check_launch("mask_predict_kernel")) return rc;
  if (VB_PRED_SPLIT_ENERGY && p.mask) {
    const int rows = p.B * p.H * p.nb;
    hipLaunchKernelGGL(energy_mask_kernel<T>, dim3((rows + 3) / 4), dim3(256), 0, stream, p.po, rows, p.nb, p.thr,
                       p.min_keep, p.max_keep, p.force_tail, p.nb, p.mask, p.count);
    return check_launch("energy_mask_kernel");
  }
  return 0;
}

}  // namespace vb

#if VB_PRED_TRACE
VB_TRACE_GETTER(vb_debug_pred_trace, vb::g_pred_trace)
#endif
#if VB_PRED_STAMPS
// diagnostic builds only: read and clear the score kernel's phase sums
extern "C" int vb_debug_pred_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vb::g_pred_stamp), 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(vb::g_pred_stamp), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" uint64_t vb_mask_predict_workspace_size(const vb_predict_args* a) {
  if (!a || a->B <= 0 || a->H <= 0 || a->L <= 0 || a->D <= 0) return 0;
  return vb::predict_ws_bytes(a->B, a->H, a->L, a->D);
}

extern "C" int vb_mask_predict(const vb_predict_args* a, void* stream) {
  using namespace vb;
  if (!a || !a->q || !a->k || !a->q_off || !a->k_off || !a->po)
    return fail(VB_ERR_INVALID, "vb_mask_predict: null argument");
  if (a->B <= 0 || a->H <= 0 || a->L <= 0) return fail(VB_ERR_INVALID, "vb_mask_predict: bad sizes");
  if (a->block != 128 || a->num_keep != 32)
    return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: block must be 128 and num_keep 32 (the reference's values)");
  const int nb = (a->L + a->block - 1) / a->block;
  if (nb > kMaxNb) return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: sequence too long");
  if (a->L > 65535) return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: L must be < 65536");
  if (a->min_keep < 1 || a->max_keep < 1) return fail(VB_ERR_INVALID, "vb_mask_predict: keep counts must be >= 1");
  if (a->D != 64 && a->D != 128) return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: head_dim must be 64 or 128");
  const uint64_t ws = predict_ws_bytes(a->B, a->H, a->L, a->D);
  if (!a->workspace || a->workspace_bytes < ws || (reinterpret_cast<uintptr_t>(a->workspace) & 15))
    return fail(VB_ERR_INVALID, "vb_mask_predict: workspace missing or smaller than vb_mask_predict_workspace_size()");
  const uint64_t rows_b = predict_rows_bytes(a->B, a->H, a->L, a->D);
  if (rows_b / a->B / a->H >= (uint64_t(1) << 31)) return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: sampled stream too large");
  if ((int64_t)(a->L - 1) * a->k_stride[2] * 2 + 2 * a->D >= (int64_t(1) << 31))
    return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: a k (b,h) slice spans >= 2 GiB");
  for (int i = 0; i < 3; ++i)
    if ((a->q_stride[i] | a->k_stride[i]) & 7) return fail(VB_ERR_INVALID, "vb_mask_predict: strides must be multiples of 8");
  PredParams p{};
  p.q = a->q; p.k = a->k;
  for (int i = 0; i < 3; ++i) { p.qs[i] = a->q_stride[i]; p.ks[i] = a->k_stride[i]; }
  p.rows = a->rows; p.q_off = a->q_off; p.k_off = a->k_off;
  p.B = a->B; p.H = a->H; p.L = a->L; p.D = a->D; p.block = a->block; p.nb = nb;
  const float scale = a->scale > 0.f ? a->scale : (float)(1.0 / sqrt((double)a->D));
  p.c = scale * 1.44269504f;
  p.thr = a->energy_threshold;
  p.min_keep = a->min_keep; p.max_keep = a->max_keep; p.force_tail = a->force_tail;
  p.po = a->po; p.mask = a->mask; p.count = a->mask_count;
  // the kept counts come from the energy rule of the fused epilogue: refused where it does not run
  if (a->mask_rows_kept && (a->mask_level || !a->mask || VB_PRED_SPLIT_ENERGY))
    return fail(VB_ERR_INVALID, "vb_mask_predict: mask_rows_kept needs the energy mask (mask set, mask_level 0)");
  p.rows_kept = a->mask_rows_kept;
  p.q_s = nullptr;
  p.k_s = reinterpret_cast<uint8_t*>(a->workspace);
  p.rbuf = reinterpret_cast<uint16_t*>(p.k_s + rows_b);
  if ((a->rand_q == nullptr) != (a->rand_k == nullptr))
    return fail(VB_ERR_INVALID, "vb_mask_predict: give both rand_q and rand_k or neither");
  p.rand_q = a->rand_q; p.rand_k = a->rand_k;
  if (a->level_bands < 0 || a->level_bands > 8 ||
      (a->level_bands > 0 && (!a->level_band_value || !a->level_band_start || !a->level_band_end)))
    return fail(VB_ERR_INVALID, "vb_mask_predict: 0..8 level bands with value/start/end arrays");
  if (a->mask_level) {
    if (!a->mask) return fail(VB_ERR_INVALID, "vb_mask_predict: mask_level needs a mask output");
    if (VB_PRED_SPLIT_ENERGY)   // that diagnostic build's epilogue writes the energy mask only
      return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: mask_level needs the fused epilogue (VB_PRED_SPLIT_ENERGY=0)");
    p.level = 1;
    p.lv.n = a->level_bands;
    for (int i = 0; i < a->level_bands; ++i) {
      const int val = a->level_band_value[i];
      if (val != 0 && val != 1 && val != 2 && val != 4 && val != 8)
        return fail(VB_ERR_INVALID, "vb_mask_predict: band values must be 0, 1, 2, 4 or 8");
      // max(0, int(nb * start)), min(nb, int(nb * end)) in double, as vb_level_mask
      const int ia = (int)((double)nb * a->level_band_start[i]), ib = (int)((double)nb * a->level_band_end[i]);
      p.lv.value[i] = val;
      p.lv.start[i] = ia < 0 ? 0 : ia;
      p.lv.end[i] = ib > nb ? nb : ib;
    }
  }
  if (a->philox) {
    if (a->rand_q || a->rand_k) return fail(VB_ERR_INVALID, "vb_mask_predict: philox and rand_q/rand_k are exclusive");
    // torch.rand's grid-stride launch gives element i the x value of thread i only while every
    // element has a thread of its own: numel <= CUs * max threads per CU of THIS device (524288 on
    // an unpartitioned MI355X; fewer in a CPX partition)
    const int64_t one_pass = philox_x_only_numel();
    if (one_pass <= 0) return fail(VB_ERR_LAUNCH, "vb_mask_predict: cannot query the device's CU count");
    if ((int64_t)a->B * a->H * a->block > one_pass)
      return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: philox draws need B*H*block <= " + std::to_string(one_pass) +
                                          " (CUs x max threads per CU of this device)");
    p.philox = 1; p.philox_seed = a->philox_seed; p.philox_offset = a->philox_offset;
  }
  if (a->pool_kp) {   // the pooled K/V pass rides in the score kernel's launch
    if (!a->pool_v || !a->pool_vp || a->pool_gap <= 0 || ((a->pool_k_r == nullptr) != (a->pool_v_r == nullptr)))
      return fail(VB_ERR_INVALID, "vb_mask_predict: pool_v, pool_vp, pool_gap > 0 and both or neither of pool_k_r/pool_v_r");
    for (int i = 0; i < 3; ++i)
      if (a->pool_v_stride[i] & 7) return fail(VB_ERR_INVALID, "vb_mask_predict: pool_v strides must be multiples of 8");
    PoolTask& t = p.pool;
    t.k = reinterpret_cast<const uint8_t*>(a->k); t.v = reinterpret_cast<const uint8_t*>(a->pool_v);
    for (int i = 0; i < 3; ++i) { t.ks[i] = a->k_stride[i]; t.vs[i] = a->pool_v_stride[i]; }
    t.rows = a->rows; t.B = a->B; t.H = a->H; t.L = a->L; t.D = a->D; t.gap = a->pool_gap;
    t.Lp = (a->L + a->pool_gap - 1) / a->pool_gap;
    t.kp = reinterpret_cast<uint8_t*>(a->pool_kp); t.vp = reinterpret_cast<uint8_t*>(a->pool_vp);
    t.k_r = reinterpret_cast<uint8_t*>(a->pool_k_r); t.v_r = reinterpret_cast<uint8_t*>(a->pool_v_r);
    const int64_t items = (int64_t)a->B * a->H * t.Lp * (a->D / 8);
    int n = (int)((items + 255) / 256);
    const int cap = a->D == 64 ? kFusedPoolWgs64 : kFusedPoolWgs;
    n = n < cap ? n : cap;
    p.n_pool = (n + 7) / 8 * 8;   // keeps blockIdx % 8 of the score workgroups (their XCD)
  }
  if (a->pyr_k) {   // the KV pyramid pass rides in the score kernel's launch
    if (a->pool_kp) return fail(VB_ERR_INVALID, "vb_mask_predict: pool_* and pyr_* are exclusive");
    if (!a->pyr_v || !a->pool_v) return fail(VB_ERR_INVALID, "vb_mask_predict: pyr_k needs pyr_v and pool_v");
    for (int i = 0; i < 3; ++i)
      if (a->pool_v_stride[i] & 7) return fail(VB_ERR_INVALID, "vb_mask_predict: pool_v strides must be multiples of 8");
    if (((reinterpret_cast<uintptr_t>(a->k) | reinterpret_cast<uintptr_t>(a->pool_v) |
          reinterpret_cast<uintptr_t>(a->pyr_k) | reinterpret_cast<uintptr_t>(a->pyr_v)) & 15) != 0)
      return fail(VB_ERR_INVALID, "vb_mask_predict: pyramid tensors must be 16-byte aligned");
    PyrTask& t = p.pyr;
    t.k = reinterpret_cast<const uint8_t*>(a->k); t.v = reinterpret_cast<const uint8_t*>(a->pool_v);
    for (int i = 0; i < 3; ++i) { t.ks[i] = a->k_stride[i]; t.vs[i] = a->pool_v_stride[i]; }
    t.rows = a->rows; t.B = a->B; t.H = a->H; t.L = a->L; t.Lpad = nb * 128;
    t.kpyr = reinterpret_cast<uint8_t*>(a->pyr_k); t.vpyr = reinterpret_cast<uint8_t*>(a->pyr_v);
    const int64_t items = (int64_t)a->B * a->H * (t.Lpad / 8) * (a->D / 8);
    int n = (int)((items + 255) / 256);
    const int cap = a->D == 64 ? kFusedPoolWgs64 : kFusedPoolWgs;
    n = n < cap ? n : cap;
    p.n_pool = (n + 7) / 8 * 8;   // keeps blockIdx % 8 of the score workgroups (their XCD)
    p.pool_kind = 2;
  }
#if VB_DIAG
  if (const char* d = getenv("VB_DEBUG_PRED")) p.dbg = atoi(d);
#endif
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipEvent_t ev = reinterpret_cast<hipEvent_t>(a->staged_event);
  if (a->dtype == VB_DTYPE_BF16) {
    if (a->D == 64) return launch_predict<64, BF16>(p, s, ev);
    if (a->D == 128) return launch_predict<128, BF16>(p, s, ev);
  } else if (a->dtype == VB_DTYPE_F16) {
    if (a->D == 64) return launch_predict<64, F16>(p, s, ev);
    if (a->D == 128) return launch_predict<128, F16>(p, s, ev);
  } else {
    return fail(VB_ERR_INVALID, "vb_mask_predict: unknown dtype");
  }
  return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: head_dim must be 64 or 128");
}

extern "C" int vb_energy_mask(const void* po, int B, int H, int nr, int nc, float energy_threshold, int min_keep,
                              int max_keep, int force_tail, int dtype, uint8_t* mask,
                              unsigned long long* mask_count, void* stream) {
  using namespace vb;
  if (!po || !mask) return fail(VB_ERR_INVALID, "vb_energy_mask: null argument");
  if (B <= 0 || H <= 0 || nr <= 0 || nc <= 0) return fail(VB_ERR_INVALID, "vb_energy_mask: bad sizes");
  if (nc > kMaxNb) return fail(VB_ERR_UNSUPPORTED, "vb_energy_mask: too many columns");
  if (min_keep < 1 || max_keep < 1) return fail(VB_ERR_INVALID, "vb_energy_mask: keep counts must be >= 1");
  const int rows = B * H * nr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((rows + 3) / 4);
  if (dtype == VB_DTYPE_BF16)
    hipLaunchKernelGGL(energy_mask_kernel<BF16>, grid, dim3(256), 0, s, po, rows, nc, energy_threshold, min_keep,
                       max_keep, force_tail, nr, mask, mask_count);
  else if (dtype == VB_DTYPE_F16)
    hipLaunchKernelGGL(energy_mask_kernel<F16>, grid, dim3(256), 0, s, po, rows, nc, energy_threshold, min_keep,
                       max_keep, force_tail, nr, mask, mask_count);
  else
    return fail(VB_ERR_INVALID, "vb_energy_mask: unknown dtype");
  return check_launch("energy_mask_kernel");
}

extern "C" int vb_sample_offsets(const float* rand_q, const float* rand_k, int rows, int n, int keep,
                                 int32_t* q_off, int32_t* k_off, void* stream) {
  using namespace vb;
  if (!rand_q || !rand_k || !q_off || !k_off) return fail(VB_ERR_INVALID, "vb_sample_offsets: null argument");
  if (rows <= 0 || n <= 0 || keep <= 0 || keep > n) return fail(VB_ERR_INVALID, "vb_sample_offsets: bad sizes");
  if (n > 256) return fail(VB_ERR_UNSUPPORTED, "vb_sample_offsets: at most 256 draws per row");
  hipLaunchKernelGGL(topk_offsets_kernel, dim3((rows + 3) / 4, 2), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     rand_q, rand_k, rows, n, keep, q_off, k_off);
  return check_launch("topk_offsets_kernel");
}

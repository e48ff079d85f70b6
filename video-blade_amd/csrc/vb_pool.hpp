// Mean pooling of K/V over `gap` consecutive reordered tokens (simple_pooling,
// cogvideox/train/special_attentions_local/TrainRelated/cogvideo_blocksparseattn.py:83-88), fused
// with the Gilbert-ordered K/V copies (the reference's index_select, :148-150). Shared by the
// stand-alone pool_kv_kernel (vb_pool.hip) and the pooling workgroups of the mask predictor's launch
// (vb_predict.hip), which run it beside the score kernel without a second stream.
#pragma once
#include "vb_common.hpp"

namespace vb {

struct PoolTask {
  const uint8_t* k; const uint8_t* v;
  int64_t ks[3], vs[3];
  const int32_t* rows;     // reordered -> caller row, or NULL
  int B, H, L, D, gap, Lp;
  uint8_t* kp; uint8_t* vp;    // [B,H,Lp,D] contiguous
  uint8_t* k_r; uint8_t* v_r;  // [B,H,L,D] contiguous Gilbert-order copies, or NULL
};

// Work items idx0, idx0 + step, ...: one 16-byte chunk of one pooled row each. Every reordered row
// is read by exactly one item, which also writes it to the copies. The gap rows are read in groups
// of VB_POOL_GROUP with every load of a group issued before any is used; the fp32 sums keep the
// sequential row order. The pass is HBM-latency bound with few workgroups, so a thread's steps
// (item, group) are pipelined: the `rows` entries of step s+1 are loaded while step s's K/V rows are
// in flight, into the other of two entry sets (the loop is unrolled by two, so no register copy of
// a pending load forces a wait). Round 5: the entries had been loaded one per row, each behind a
// vmcnt(0) that also waited for the previous rows, so a 15-row item took ~16 round trips.
#ifndef VB_POOL_GROUP
#define VB_POOL_GROUP 8
#endif
#ifndef VB_POOL_NT
// 1: the K/V reads non-temporal (each row is read once; the score workgroups beside the pass keep
// more of their L2), 2: the copies' stores too. Per CogVideoX call against the pipelined pass with
// plain loads: 1.017/1.018x vs 1.015/1.012x, 2: 1.008x (profiles/archive/r05_pool_pipeline_ab.log)
#define VB_POOL_NT 1
#endif
__device__ __forceinline__ u32x4 pool_ld(const uint8_t* p) {
#if VB_POOL_NT >= 1
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#else
  return *reinterpret_cast<const u32x4*>(p);
#endif
}
__device__ __forceinline__ void pool_st(uint8_t* p, const u32x4& x) {
#if VB_POOL_NT >= 2
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
#else
  *reinterpret_cast<u32x4*>(p) = x;
#endif
}
template <class T, bool kRows>
__device__ __forceinline__ void pool_kv_steps(const PoolTask& t, int64_t idx0, int64_t step) {
  constexpr int G = VB_POOL_GROUP;
  const int CH = t.D / 8;
  const int64_t total = (int64_t)t.B * t.H * t.Lp * CH;
  if (idx0 >= total) return;
  // caller-order positions of rows g0 .. g0+G-1 of item idx's pooled row (replicate padding)
  auto positions = [&](int64_t idx, int g0, int (&pos)[G]) __attribute__((always_inline)) {
    const int pr = (int)((idx / CH) % t.Lp);
#pragma unroll
    for (int u = 0; u < G; ++u) pos[u] = min(pr * t.gap + min(g0 + u, t.gap - 1), t.L - 1);
    if constexpr (kRows) {
#pragma unroll
      for (int u = 0; u < G; ++u) pos[u] = t.rows[pos[u]];
    }
  };
  int64_t idx = idx0;
  int g0 = 0;
  float ak[8], av[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ak[e] = av[e] = 0.f;
  // one step: the group's K/V rows (entries `cur`), the next step's entries into `nxt`, then the
  // copies and sums of this group. Returns false after the thread's last step.
  auto run = [&](const int (&cur)[G], int (&nxt)[G]) __attribute__((always_inline)) -> bool {
    const int ch = (int)(idx % CH);
    const int64_t prow = idx / CH;   // (b*H + h)*Lp + pr
    const int pr = (int)(prow % t.Lp);
    const int bh = (int)(prow / t.Lp);
    const int b = bh / t.H, h = bh % t.H;
    const uint8_t* kb = t.k + 2 * (b * t.ks[0] + h * t.ks[1]) + ch * 16;
    const uint8_t* vb = t.v + 2 * (b * t.vs[0] + h * t.vs[1]) + ch * 16;
    u32x4 xk[G], xv[G];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      xk[u] = pool_ld(kb + 2 * (int64_t)cur[u] * t.ks[2]);
      xv[u] = pool_ld(vb + 2 * (int64_t)cur[u] * t.vs[2]);
    }
    int64_t nidx = idx;
    int ng0 = g0 + G;
    if (ng0 >= t.gap) { ng0 = 0; nidx += step; }
    const bool more = nidx < total;
    positions(more ? nidx : idx, more ? ng0 : g0, nxt);   // past the last step: reloaded, unused
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (g0 + u >= t.gap) break;
      const int g = pr * t.gap + g0 + u;
      if (t.k_r && g < t.L) {
        const int64_t o = ((int64_t)bh * t.L + g) * t.D * 2 + ch * 16;
        pool_st(t.k_r + o, xk[u]);
        pool_st(t.v_r + o, xv[u]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ak[2 * e] += T::bits_to_f32(xk[u][e] & 0xffff);
        ak[2 * e + 1] += T::bits_to_f32(xk[u][e] >> 16);
        av[2 * e] += T::bits_to_f32(xv[u][e] & 0xffff);
        av[2 * e + 1] += T::bits_to_f32(xv[u][e] >> 16);
      }
    }
    if (g0 + G >= t.gap) {   // the item's last group: its pooled row
      const float f = 1.0f / (float)t.gap;   // mean = sum * (1/N), as ATen's MeanOps
      u32x4 ok, ov;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ok[e] = pack2<T>(ak[2 * e] * f, ak[2 * e + 1] * f);
        ov[e] = pack2<T>(av[2 * e] * f, av[2 * e + 1] * f);
      }
      *reinterpret_cast<u32x4*>(t.kp + (prow * t.D + ch * 8) * 2) = ok;
      *reinterpret_cast<u32x4*>(t.vp + (prow * t.D + ch * 8) * 2) = ov;
#pragma unroll
      for (int e = 0; e < 8; ++e) ak[e] = av[e] = 0.f;
    }
    idx = nidx;
    g0 = ng0;
    return more;
  };
  int pa[G], pb[G];
  positions(idx, 0, pa);
  for (;;) {
    if (!run(pa, pb)) break;
    if (!run(pb, pa)) break;
  }
}

template <class T>
__device__ __forceinline__ void pool_kv_span(const PoolTask& t, int64_t idx0, int64_t step) {
  if (t.rows) pool_kv_steps<T, true>(t, idx0, step);
  else pool_kv_steps<T, false>(t, idx0, step);
}

}  // namespace vb

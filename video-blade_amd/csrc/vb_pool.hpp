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
// of VB_POOL_GROUP with every load of a group issued before any is used (2 * VB_POOL_GROUP loads in
// flight per thread: the pass is HBM-latency bound otherwise); the fp32 sums keep the sequential
// row order.
#ifndef VB_POOL_GROUP
#define VB_POOL_GROUP 8
#endif
template <class T>
__device__ __forceinline__ void pool_kv_span(const PoolTask& t, int64_t idx0, int64_t step) {
  const int CH = t.D / 8;
  const int64_t total = (int64_t)t.B * t.H * t.Lp * CH;
  for (int64_t idx = idx0; idx < total; idx += step) {
    const int ch = idx % CH;
    const int64_t prow = idx / CH;   // (b*H + h)*Lp + pr
    const int pr = prow % t.Lp;
    const int bh = prow / t.Lp;
    const int b = bh / t.H, h = bh % t.H;
    const uint8_t* kb = t.k + 2 * (b * t.ks[0] + h * t.ks[1]) + ch * 16;
    const uint8_t* vb = t.v + 2 * (b * t.vs[0] + h * t.vs[1]) + ch * 16;
    float ak[8], av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) ak[e] = av[e] = 0.f;
    constexpr int G = VB_POOL_GROUP;
    for (int g0 = 0; g0 < t.gap; g0 += G) {
      u32x4 xk[G], xv[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int g = pr * t.gap + min(g0 + u, t.gap - 1);
        int pos = min(g, t.L - 1);   // replicate padding
        if (t.rows) pos = t.rows[pos];
        xk[u] = *reinterpret_cast<const u32x4*>(kb + 2 * (int64_t)pos * t.ks[2]);
        xv[u] = *reinterpret_cast<const u32x4*>(vb + 2 * (int64_t)pos * t.vs[2]);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        if (g0 + u >= t.gap) break;
        const int g = pr * t.gap + g0 + u;
        if (t.k_r && g < t.L) {
          const int64_t o = ((int64_t)bh * t.L + g) * t.D * 2 + ch * 16;
          *reinterpret_cast<u32x4*>(t.k_r + o) = xk[u];
          *reinterpret_cast<u32x4*>(t.v_r + o) = xv[u];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ak[2 * e] += T::bits_to_f32(xk[u][e] & 0xffff);
          ak[2 * e + 1] += T::bits_to_f32(xk[u][e] >> 16);
          av[2 * e] += T::bits_to_f32(xv[u][e] & 0xffff);
          av[2 * e + 1] += T::bits_to_f32(xv[u][e] >> 16);
        }
      }
    }
    const float f = 1.0f / (float)t.gap;   // mean = sum * (1/N), as ATen's MeanOps
    u32x4 ok, ov;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ok[e] = pack2<T>(ak[2 * e] * f, ak[2 * e + 1] * f);
      ov[e] = pack2<T>(av[2 * e] * f, av[2 * e + 1] * f);
    }
    *reinterpret_cast<u32x4*>(t.kp + (prow * t.D + ch * 8) * 2) = ok;
    *reinterpret_cast<u32x4*>(t.vp + (prow * t.D + ch * 8) * 2) = ov;
  }
}

}  // namespace vb

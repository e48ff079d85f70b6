// KV pyramid of the multi-level path (the reference kernel's _forward, kernels/
// block_sparse_attn_kernel_with_backward_9_10.py:1311-1320: k_2/k_4/k_8 via pad_to_multiple
// :1239-1250 and pooling :1252-1270). Shared by the stand-alone kv_pyramid_kernel (vb_ml.hip) and
// the pyramid workgroups of the mask predictor's launch (vb_predict.hip).
#pragma once
#include "vb_common.hpp"

namespace vb {

struct PyrTask {
  const uint8_t* k; const uint8_t* v;
  int64_t ks[3], vs[3];
  const int32_t* rows;   // reordered -> caller row, or NULL
  int B, H, L, Lpad;
  uint8_t* kpyr; uint8_t* vpyr;   // [B,H,15*Lpad/8,D]
};

// Work items idx0, idx0 + step, ...: one 16-byte chunk (8 elements) of 8 consecutive reordered
// rows g0..g0+7, for K and V: the 8 rows are read once (replicate padding: rows >= L read row
// L-1) and 8 level-1 rows (zero beyond L), 4 level-2, 2 level-4 and 1 level-8 rows are written.
// Each level is the mean of the previous level's pairs in fp32, rounded to the storage dtype, as
// torch.mean on a bf16/fp16 view does. Consecutive items take consecutive chunks of a row, so
// every row read/write is coalesced. Layout per (b,h): [Lpad level-1 | Lpad/2 | Lpad/4 | Lpad/8].
// The `rows` entries of a thread's next item are loaded while the current item's K/V rows are in
// flight (two entry sets, loop unrolled by two), and K and V share them: one memory round trip per
// item (round 5; each entry had been loaded behind a wait for the previous row's data).
template <int D, class T, bool kRows>
__device__ __forceinline__ void kv_pyramid_steps(const PyrTask& t, int64_t idx0, int64_t step) {
  constexpr int kCh = D / 8;   // 16-byte chunks per row
  const int ngroups = t.Lpad / 8;
  const int64_t total = (int64_t)t.B * t.H * ngroups * kCh;
  if (idx0 >= total) return;
  const int R = 15 * (t.Lpad / 8);
  const int off2 = t.Lpad, off4 = t.Lpad + t.Lpad / 2, off8 = off4 + t.Lpad / 4;
  auto positions = [&](int64_t tid, int (&pos)[8]) __attribute__((always_inline)) {
    const int g = (int)((tid / kCh) % ngroups);
#pragma unroll
    for (int r = 0; r < 8; ++r) pos[r] = min(g * 8 + r, t.L - 1);
    if constexpr (kRows) {
#pragma unroll
      for (int r = 0; r < 8; ++r) pos[r] = t.rows[pos[r]];
    }
  };
  int64_t tid = idx0;
  auto run = [&](const int (&cur)[8], int (&nxt)[8]) __attribute__((always_inline)) -> bool {
    const int ch = (int)(tid % kCh);
    const int64_t rest = tid / kCh;
    const int g = (int)(rest % ngroups);
    const int bh = (int)(rest / ngroups);
    const int b = bh / t.H, h = bh % t.H;
    u32x4 xs[2][8];
#pragma unroll
    for (int mat = 0; mat < 2; ++mat) {
      const uint8_t* src = mat == 0 ? t.k : t.v;
      const int64_t s0 = mat == 0 ? t.ks[0] : t.vs[0], s1 = mat == 0 ? t.ks[1] : t.vs[1];
      const int64_t s2 = mat == 0 ? t.ks[2] : t.vs[2];
      const uint8_t* base = src + (b * s0 + h * s1 + ch * 8) * 2;
#pragma unroll
      for (int r = 0; r < 8; ++r) xs[mat][r] = *reinterpret_cast<const u32x4*>(base + (int64_t)cur[r] * s2 * 2);
    }
    const int64_t ntid = tid + step;
    const bool more = ntid < total;
    positions(more ? ntid : tid, nxt);   // past the last item: reloaded, unused
#pragma unroll
    for (int mat = 0; mat < 2; ++mat) {
      const u32x4* x = xs[mat];
      uint8_t* dst = (mat == 0 ? t.kpyr : t.vpyr) + ((int64_t)bh * R * D + ch * 8) * 2;
      uint8_t* dst1 = dst + (int64_t)(g * 8) * D * 2;
      uint8_t* dst2 = dst + (int64_t)(off2 + g * 4) * D * 2;
      uint8_t* dst4 = dst + (int64_t)(off4 + g * 2) * D * 2;
      uint8_t* dst8 = dst + (int64_t)(off8 + g) * D * 2;
      // level 1 (zero beyond L: the reference kernel's masked loads of the tail block)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        u32x4 w = x[r];
        if (g * 8 + r >= t.L) w = u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(dst1 + r * D * 2) = w;   // one base, immediate row offsets
      }
      // levels 2, 4, 8: each level kept as fp32 values of storage-rounded means (x -> f2 -> f4 -> f8)
      float f2[4][8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        u32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t a = x[2 * r][e], b = x[2 * r + 1][e];
          f2[r][2 * e] = round_to<T>((T::bits_to_f32((uint16_t)(a & 0xFFFF)) + T::bits_to_f32((uint16_t)(b & 0xFFFF))) * 0.5f);
          f2[r][2 * e + 1] = round_to<T>((T::bits_to_f32((uint16_t)(a >> 16)) + T::bits_to_f32((uint16_t)(b >> 16))) * 0.5f);
          w[e] = pack2<T>(f2[r][2 * e], f2[r][2 * e + 1]);
        }
        *reinterpret_cast<u32x4*>(dst2 + r * D * 2) = w;
      }
      float f4[2][8];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        u32x4 w;
#pragma unroll
        for (int e = 0; e < 8; ++e) f4[r][e] = round_to<T>((f2[2 * r][e] + f2[2 * r + 1][e]) * 0.5f);
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = pack2<T>(f4[r][2 * e], f4[r][2 * e + 1]);
        *reinterpret_cast<u32x4*>(dst4 + r * D * 2) = w;
      }
      {
        u32x4 w;
        float f8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) f8[e] = round_to<T>((f4[0][e] + f4[1][e]) * 0.5f);
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = pack2<T>(f8[2 * e], f8[2 * e + 1]);
        *reinterpret_cast<u32x4*>(dst8) = w;
      }
    }
    tid = ntid;
    return more;
  };
  int pa[8], pb[8];
  positions(tid, pa);
  for (;;) {
    if (!run(pa, pb)) break;
    if (!run(pb, pa)) break;
  }
}

template <int D, class T>
__device__ __forceinline__ void kv_pyramid_span(const PyrTask& t, int64_t idx0, int64_t step) {
  if (t.rows) kv_pyramid_steps<D, T, true>(t, idx0, step);
  else kv_pyramid_steps<D, T, false>(t, idx0, step);
}

}  // namespace vb

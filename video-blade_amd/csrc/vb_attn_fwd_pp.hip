// Ping-pong variant of the block-sparse FMHA forward for head_dim 64 (CogVideoX), inference launches
// (no LSE output), bf16/f16. Same semantics and inputs as attn_fwd_kernel<64, T, kPool, false, false,
// true> (vb_attn_fwd.hip): one workgroup per (b, h, 128-row q-block), kept 128-key blocks as two
// 64-key tiles each (diagonal block first), then the pooled keys with a +log2(gap) bias, one lazy
// exp2-domain softmax over all of them, Q gathered and O scattered through q_rows.
//
// Why a second kernel: at D=64 a 64-key tile costs a wave 16 MFMAs (512 matrix cycles) and ~600
// cycles of vector issue (32 v_exp, the row sums, the bf16 packs, the MFMA issue holds). In the
// 4-wave kernel the three co-resident waves of a SIMD come from different workgroups and drift into
// the same phase, so the matrix pipe and the exp VALU rarely overlap (PMC: MFMA busy 49 %, VALU
// active 60 %, ~1050 SIMD cycles per wave-tile against a 600-cycle issue bound).
//
// Here a workgroup is 8 waves, two per SIMD (waves w and w+4 share a SIMD and own the same 32 query
// rows). Group A (waves 0-3) takes the even tiles of the q-block's tile list, group B (waves 4-7)
// the odd ones, each with its own running max, row sum and O (split-K). Segments separated by one
// workgroup barrier alternate the groups' roles, so on every SIMD one wave issues MFMAs while its
// partner runs the softmax VALU:
//
//   segment s:  group (s & 1):  P.V of tile s-2, S^T = K.Q^T of tile s, LDS-DMA of tile s+6
//               other group:    softmax of tile s-1 (exp2, row sum, lazy-max check, bf16 pack)
//
// Each group streams its own tiles through an 8-slot LDS ring (tile t in slot t % 8, 16 KiB: K
// image then V image, the XOR-swizzled layouts of vb_attn_fwd.hpp). At the end group B hands its
// (m, l, O) to group A through LDS and A writes the combined, normalised rows. The split changes
// the order of the fp32 sums (results equal the 4-wave kernel's up to rounding; deterministic).
#include <type_traits>

#include "vb_attn_fwd.hpp"

namespace vb {
namespace pp {
constexpr int kD = 64;
constexpr int kKS = kD / 16;              // k-steps of S^T = K.Q^T
constexpr int kDT = kD / 32;              // 32-wide d tiles of O^T
constexpr int kRowB = kD * 2;
constexpr int kMatBytes = kKT * kRowB;    // 8 KiB
constexpr int kBufBytes = 2 * kMatBytes;  // K image, V image
constexpr int kRing = 8;
constexpr int kAhead = 3;                 // own tiles in flight ahead of the one being computed
constexpr int kChunks = kRowB / 16;
constexpr int kRowsPerInst = 1024 / kRowB;
constexpr int kInstPerWave = 4;           // 16 KiB per tile / 4 waves / 1 KiB
}  // namespace pp

#ifndef VB_PP_PRIO
#define VB_PP_PRIO 1   // static s_setprio 1 for group B (the second-dispatched half)
#endif

template <class T, bool kPool>
__global__ void __launch_bounds__(512, 1) attn_fwd_pp_kernel(const FwdParams p) {
  using namespace pp;
  constexpr float kLazyBound = std::is_same<T, BF16>::value ? kLazyBoundBF16 : kLazyBoundF16;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kRing * kBufBytes + kMaxBlocks * 2 + 16];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + kRing * kBufBytes);
  int* list_n = reinterpret_cast<int*>(smem + kRing * kBufBytes + kMaxBlocks * 2);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wave >> 2;       // 0: even tiles, 1: odd tiles
  const int wq = wave & 3;         // query-row group (shared by waves wq and wq + 4)
  const int half = lane >> 5;
  const int l32 = lane & 31;
  if (VB_PP_PRIO && grp == 1) __builtin_amdgcn_s_setprio(1);

  // work order: as attn_fwd_kernel (heavy rows first, then XCD-contiguous head-major ranges)
  const int BH = p.B * p.H;
  const int hr = min(p.heavy_rows, p.nbq);
  const int n_heavy = hr * BH;
  int qblk, bh;
  if ((int)blockIdx.x < n_heavy) {
    qblk = p.nbq - 1 - (int)(blockIdx.x / BH);
    bh = blockIdx.x % BH;
  } else {
    const int rows_left = p.nbq - hr;
    const int lin = xcd_linear(blockIdx.x - n_heavy, rows_left * BH);
    bh = lin / rows_left;
    qblk = rows_left - 1 - lin % rows_left;
  }
  const int b = bh / p.H, h = bh % p.H;
  const int Lq = p.Lq, Lk = p.Lk;
  const int q0 = qblk * kQBlk;
  const int nbk = (Lk + kQBlk - 1) / kQBlk;

  // ---- kept key blocks of this q-block (diagonal first), as attn_fwd_kernel --------------------
  const uint8_t* mrow = p.mask ? p.mask + b * p.ms[0] + (int64_t)h * p.ms[1] + (int64_t)qblk * p.ms[2] : nullptr;
  if (threadIdx.x < 64) {
    int n = 0, dpos = -1;
    for (int j0 = 0; j0 < nbk; j0 += 64) {
      const int j = j0 + lane;
      const bool keep = (j < nbk) && (mrow == nullptr || mrow[j] != 0);
      const unsigned long long bal = __ballot(keep);
      if (keep) {
        const int pos = n + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
        list[pos] = (uint16_t)j;
        if (j == qblk) dpos = pos;
      }
      n += __popcll(bal);
    }
    const unsigned long long db = __ballot(dpos > 0);
    if (db != 0 && qblk != nbk - 1) {
      const int dp = __builtin_amdgcn_readlane(dpos, (int)__builtin_ctzll(db));
      if (lane == 0) {
        const uint16_t t = list[0];
        list[0] = (uint16_t)qblk;
        list[dp] = t;
      }
    }
    if (lane == 0) *list_n = n;
  }

  // ---- Q fragment (pre-scaled by scale*log2e: scores leave the MFMA in the exp2 domain) ---------
  const int qg = q0 + wq * 32 + l32;
  const bool qvalid = qg < Lq;
  int qrow = qvalid ? qg : Lq - 1;
  if (p.q_rows) qrow = p.q_rows[qrow];
  typename T::vec8 qf[kKS];
  {
    const uint8_t* qp = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + (int64_t)qrow * p.qs[2]);
#pragma unroll
    for (int s = 0; s < kKS; ++s) qf[s] = *reinterpret_cast<const typename T::vec8*>(qp + (16 * s + 8 * half) * 2);
#pragma unroll
    for (int s = 0; s < kKS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[s][e] = T::from_f32(T::to_f32(qf[s][e]) * p.c);
#pragma unroll
    for (int s = 0; s < kKS; ++s) asm volatile("" : "+v"(qf[s]));
  }
  __syncthreads();
  const int nkept = __builtin_amdgcn_readfirstlane(*list_n);
  int ntm = 2 * nkept;
  if (nkept > 0 && list[nkept - 1] == nbk - 1 && (nbk - 1) * kQBlk + kKT >= Lk) ntm -= 1;
  const int ntp = kPool ? (p.Lkp + kKT - 1) / kKT : 0;
  const int ntiles = ntm + ntp;

  // ---- LDS-DMA of a tile: waves wq 0-1 fill K, 2-3 fill V (4 x 1 KiB each), swizzle on the source --
  const int my_mat = wq >> 1;
  const uint8_t* kbase = reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1]);
  const uint8_t* vbase = reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1]);
  const int my_rowb = 2 * (int)(my_mat == 0 ? p.ks[2] : p.vs[2]);
  const srd_t my_rsrc = make_srd(my_mat == 0 ? kbase : vbase, (int)((int64_t)(Lk - 1) * my_rowb + kRowB));
  int my_prowb = 0;
  srd_t my_prsrc = my_rsrc;
  if (kPool) {
    const uint8_t* kp = reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1]);
    const uint8_t* vp = reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1]);
    my_prowb = 2 * (int)(my_mat == 0 ? p.kps[2] : p.vps[2]);
    my_prsrc = make_srd(my_mat == 0 ? kp : vp, (int)((int64_t)(p.Lkp - 1) * my_prowb + kRowB));
  }
  int my_rc[kInstPerWave];
  const int my_row0 = (wq & 1) * kInstPerWave * kRowsPerInst + lane / kChunks;
#pragma unroll
  for (int i = 0; i < kInstPerWave; ++i) {
    const int r = my_row0 + i * kRowsPerInst;
    const int sl = lane % kChunks;
    my_rc[i] = 16 * (my_mat == 0 ? (sl ^ ((r >> 1) & 7)) : ((((sl >> 2) ^ ((r >> 1) & 1)) << 2) | (sl & 3)));
  }
  const int voff_m0 = my_row0 * my_rowb, voff_p0 = my_row0 * my_prowb;
  // tile t's keys: (pooled?, first key, valid keys)
  auto tile_keys = [&](int t, int& pooled, int& kstart, int& klen) __attribute__((always_inline)) {
    if (t < ntm) {
      const int blk = __builtin_amdgcn_readfirstlane((int)list[min(t >> 1, kMaxBlocks - 1)]);
      pooled = 0;
      kstart = blk * kQBlk + (t & 1) * kKT;
      klen = min(kKT, Lk - kstart);
    } else {
      pooled = 1;
      kstart = (t - ntm) * kKT;
      klen = min(kKT, p.Lkp - kstart);
    }
  };
  auto issue = [&](int t) __attribute__((always_inline)) {
    int pooled, kstart, klen;
    tile_keys(t, pooled, kstart, klen);
    uint8_t* dst = smem + (t & (kRing - 1)) * kBufBytes + my_mat * kMatBytes + (wq & 1) * kInstPerWave * 1024;
    const bool pl = kPool && pooled;
    const int rowb = pl ? my_prowb : my_rowb;
    const int soff = __builtin_amdgcn_readfirstlane(kstart * rowb);
    if (klen == kKT) {
      const int vb0 = pl ? voff_p0 : voff_m0;
#pragma unroll
      for (int i = 0; i < kInstPerWave; ++i)
        dma16(pl ? my_prsrc : my_rsrc, dst + i * 1024, vb0 + my_rc[i],
              __builtin_amdgcn_readfirstlane(soff + i * kRowsPerInst * rowb));
    } else {   // tail tile: rows past the last key replicate it (masked in the softmax)
#pragma unroll
      for (int i = 0; i < kInstPerWave; ++i) {
        const int r = min(my_row0 + i * kRowsPerInst, klen - 1);
        dma16(pl ? my_prsrc : my_rsrc, dst + i * 1024, r * rowb + my_rc[i], soff);
      }
    }
  };

  // ---- per-wave softmax state (exp2 domain, lazy running max: see attn_fwd_kernel) ---------------
  f32x16 o[kDT];
#pragma unroll
  for (int i = 0; i < kDT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = 0.f, l = 0.f;
  f32x16 cb;   // bias - m: the C seed of every S^T chain
#pragma unroll
  for (int r = 0; r < 16; ++r) cb[r] = 0.f;
  float cur_bias = 0.f;
  bool first = true;
  f32x16 s[2];                        // S^T of the tile awaiting its softmax
  typename T::vec8 pf[4];             // packed P of the tile awaiting its P.V
  int s_klen = kKT;

  const uint32_t smem_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)smem));
  int k_lane[kKS];
#pragma unroll
  for (int ks = 0; ks < kKS; ++ks) k_lane[ks] = k_off<kD>(l32, 2 * ks + half);
  const int vrow = 4 * half + (lane & 15) / 4;
  const int vcol = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  uint32_t v_lane[kDT];
#pragma unroll
  for (int dt = 0; dt < kDT; ++dt) v_lane[dt] = smem_base + kMatBytes + v_off_bytes<kD>(vrow, dt * 32 + vcol);

  auto half_max = [&](const f32x16& x) __attribute__((always_inline)) -> float {
    const float a = max3f(max3f(max3f(x[0], x[1], x[2]), x[3], x[4]), x[5], x[6]);
    const float c = max3f(max3f(max3f(x[8], x[9], x[10]), x[11], x[12]), x[13], x[14]);
    return max3f(a, c, fmaxf(x[7], x[15]));
  };
  auto exp_pack = [&](const f32x16& x, typename T::vec8& p0, typename T::vec8& p1) __attribute__((always_inline)) -> float {
    float e[16], h4[4];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      e[r] = exp2_fast(x[r]);
      h4[r & 3] = r < 4 ? e[r] : h4[r & 3] + e[r];
    }
    u32x4 u0, u1;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      u0[w] = pack2<T>(e[2 * w], e[2 * w + 1]);
      u1[w] = pack2<T>(e[8 + 2 * w], e[8 + 2 * w + 1]);
    }
    p0 = __builtin_bit_cast(typename T::vec8, u0);
    p1 = __builtin_bit_cast(typename T::vec8, u1);
    return (h4[0] + h4[1]) + (h4[2] + h4[3]);
  };
  // raise m by the rows' max mt (if > 0): rescale O, l, the C seed and S half kt (and the second half)
  auto raise_m = [&](float mt, int kt) __attribute__((always_inline)) {
    const float delta = fmaxf(max_xor32(mt), 0.f);
    const float alpha = exp2_fast(-delta);
    m += delta;
    l *= alpha;
#pragma unroll
    for (int i = 0; i < kDT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      cb[r] -= delta;
      if (kt == 0) s[0][r] -= delta;
      s[1][r] -= delta;
    }
  };

  // MFMA segment, part 1: O^T += V^T . P^T of tile t (slot t % 8; P packed by its softmax). The
  // transposed V reads are asm (the builtin would make hipcc drain the LDS-DMA queue before each,
  // see vb_tiles.hpp) with explicit counted waits: k-steps 0-1 after lgkmcnt(8), 2-3 after 0.
  auto pv = [&](int t) __attribute__((always_inline)) {
    const uint32_t so = (t & (kRing - 1)) * kBufBytes;
    s16x4 vlo[4][kDT], vhi[4][kDT];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
      for (int dt = 0; dt < kDT; ++dt) {
        const uint32_t a = v_lane[dt] + so;
        switch (kk) {   // compile-time row offsets (instruction immediates)
          case 0: vlo[0][dt] = lds_tr4_asm(a, 0 * kRowB); vhi[0][dt] = lds_tr4_asm(a, 8 * kRowB); break;
          case 1: vlo[1][dt] = lds_tr4_asm(a, 16 * kRowB); vhi[1][dt] = lds_tr4_asm(a, 24 * kRowB); break;
          case 2: vlo[2][dt] = lds_tr4_asm(a, 32 * kRowB); vhi[2][dt] = lds_tr4_asm(a, 40 * kRowB); break;
          default: vlo[3][dt] = lds_tr4_asm(a, 48 * kRowB); vhi[3][dt] = lds_tr4_asm(a, 56 * kRowB); break;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(vlo[0][0]), "+v"(vhi[0][0]), "+v"(vlo[0][1]), "+v"(vhi[0][1]),
                 "+v"(vlo[1][0]), "+v"(vhi[1][0]), "+v"(vlo[1][1]), "+v"(vhi[1][1]));
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int dt = 0; dt < kDT; ++dt) o[dt] = T::mfma32(join8<T>(vlo[kk][dt], vhi[kk][dt]), pf[kk], o[dt]);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[2][0]), "+v"(vhi[2][0]), "+v"(vlo[2][1]), "+v"(vhi[2][1]),
                 "+v"(vlo[3][0]), "+v"(vhi[3][0]), "+v"(vlo[3][1]), "+v"(vhi[3][1]));
#pragma unroll
    for (int kk = 2; kk < 4; ++kk)
#pragma unroll
      for (int dt = 0; dt < kDT; ++dt) o[dt] = T::mfma32(join8<T>(vlo[kk][dt], vhi[kk][dt]), pf[kk], o[dt]);
  };
  // MFMA segment, part 2: S^T = K.Q^T of tile t, seeded with (bias - m)
  auto qk = [&](int t) __attribute__((always_inline)) {
    int pooled, kstart, klen;
    tile_keys(t, pooled, kstart, klen);
    const float bias = (kPool && pooled) ? p.pool_bias_l2 : 0.f;
    if (bias != cur_bias) {   // wave-uniform; once, where the pooled keys begin
      asm volatile("");
      const float db = bias - cur_bias;
#pragma unroll
      for (int r = 0; r < 16; ++r) cb[r] += db;
      cur_bias = bias;
    }
    s_klen = klen;
    const uint8_t* kl = smem + (t & (kRing - 1)) * kBufBytes;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      typename T::vec8 kf[kKS];
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) kf[ks] = lds_b128<T>(kl + kt * 32 * kRowB, k_lane[ks]);
      s[kt] = T::mfma32(kf[0], qf[0], cb);
#pragma unroll
      for (int ks = 1; ks < kKS; ++ks) s[kt] = T::mfma32(kf[ks], qf[ks], s[kt]);
    }
  };
  // VALU segment: lazy softmax of the tile in s -> pf, l (m and O only on the rare slow path)
  auto softmax = [&]() __attribute__((always_inline)) {
    if (s_klen < kKT) {
      asm volatile("");
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= s_klen) s[kt][r] = -INFINITY;
    }
    if (first) {
      asm volatile("");
      const float mt = max_xor32(fmaxf(half_max(s[0]), half_max(s[1])));
      m += mt;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[0][r] -= mt;
        s[1][r] -= mt;
        cb[r] -= mt;
      }
      first = false;
    }
    float h0 = exp_pack(s[0], pf[0], pf[1]);
    float h1 = exp_pack(s[1], pf[2], pf[3]);
    if (!__all(fmaxf(h0, h1) <= kLazyBound)) {
      asm volatile("");
      // O holds no P of this tile yet (its P.V runs in the next segment): raise m to the tile's
      // row max, rescale O and l, and redo both halves
      raise_m(fmaxf(half_max(s[0]), half_max(s[1])), 0);
      h0 = exp_pack(s[0], pf[0], pf[1]);
      h1 = exp_pack(s[1], pf[2], pf[3]);
    }
    l += h0 + h1;
  };

  // ---- the segment loop ----------------------------------------------------------------------------
  // Segment seg: the group with (seg & 1) == grp runs P.V(seg-2) + S(seg) + DMA(seg+6), the other the
  // softmax of tile seg-1. The steady state (every tile index in range) is a loop specialised per
  // group and unrolled by two, so the role of each segment is a compile-time constant and the big
  // loop-carried values (S, P, O) pass no branch joins (which made hipcc copy them at every join).
#pragma unroll
  for (int k = 0; k < kAhead; ++k) {
    const int t = grp + 2 * k;
    if (t < ntiles) issue(t);
  }
  const int nseg = ntiles + 2;
  auto sync = [&](int seg, bool mfma) __attribute__((always_inline)) {
    if (mfma && seg < ntiles) {
      // own DMAs of tile seg must have landed; own tiles seg+2, seg+4 may stay in flight
      const int younger = (seg + 2 < ntiles) + (seg + 4 < ntiles);
      if (younger == 2) VB_WAIT_VMCNT(2 * kInstPerWave);
      else if (younger == 1) VB_WAIT_VMCNT(kInstPerWave);
      else VB_WAIT_VMCNT(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // any segment, every condition checked (the ends of the schedule)
  auto seg_generic = [&](int seg) __attribute__((always_inline)) {
    const bool mfma = (seg & 1) == grp;
    sync(seg, mfma);
    if (mfma) {
      if (seg >= 2 && seg - 2 < ntiles) pv(seg - 2);
      if (seg < ntiles) qk(seg);
      if (seg + 2 * kAhead < ntiles) issue(seg + 2 * kAhead);
    } else if (seg >= 1 && seg - 1 < ntiles) {
      softmax();
    }
  };
  // steady state for group G from segment `first_mfma` (its first MFMA segment with a P.V to do)
  auto steady = [&](int seg) __attribute__((always_inline)) -> int {
    for (; seg + 1 < ntiles; seg += 2) {   // seg: MFMA (seg-2, seg in range); seg+1: softmax of seg
      sync(seg, true);
      pv(seg - 2);
      qk(seg);
      if (seg + 2 * kAhead < ntiles) issue(seg + 2 * kAhead);
      sync(seg + 1, false);
      softmax();
    }
    return seg;
  };
  int seg = 0;
  // segments 0 .. 1 + grp: A: [S(0)], [softmax(0)]; B: [-], [S(1)], [softmax(1)]
  for (; seg < 2 + grp && seg < nseg; ++seg) seg_generic(seg);
  if (seg == 2 + grp) seg = steady(seg);
  for (; seg < nseg; ++seg) seg_generic(seg);
  VB_WAIT_VMCNT(0);

  // ---- combine the two groups' (m, l, O) and write ----------------------------------------------
  __syncthreads();   // every ring read and DMA is done: the ring is free
  float* xch = reinterpret_cast<float*>(smem) + wq * (34 * 64);
  if (grp == 1) {
#pragma unroll
    for (int dt = 0; dt < kDT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) xch[(dt * 16 + r) * 64 + lane] = o[dt][r];
    xch[32 * 64 + lane] = m;
    xch[33 * 64 + lane] = l;
  }
  __syncthreads();
  if (grp == 1) return;
  const int nB = ntiles >> 1;   // tiles of group B
  const float mB = xch[32 * 64 + lane], lB = xch[33 * 64 + lane];
  const float mm = nB > 0 ? fmaxf(m, mB) : m;
  const float wa = exp2_fast(m - mm);
  const float wb = nB > 0 ? exp2_fast(mB - mm) : 0.f;
#pragma unroll
  for (int dt = 0; dt < kDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = o[dt][r] * wa + xch[(dt * 16 + r) * 64 + lane] * wb;
  const float lt = add_xor32(l * wa + lB * wb);
  const float inv = (lt > 0.f) ? 1.0f / lt : 0.f;
  if (qvalid) {
    uint8_t* obase = reinterpret_cast<uint8_t*>(p.out) + 2 * (b * p.os[0] + h * p.os[1] + (int64_t)qrow * p.os[2]);
#pragma unroll
    for (int dt = 0; dt < kDT; ++dt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        u32x2 a, c;
        a[0] = pack2<T>(o[dt][8 * pr + 0] * inv, o[dt][8 * pr + 1] * inv);
        a[1] = pack2<T>(o[dt][8 * pr + 2] * inv, o[dt][8 * pr + 3] * inv);
        c[0] = pack2<T>(o[dt][8 * pr + 4] * inv, o[dt][8 * pr + 5] * inv);
        c[1] = pack2<T>(o[dt][8 * pr + 6] * inv, o[dt][8 * pr + 7] * inv);
        const auto sx = __builtin_amdgcn_permlane32_swap(a[0], c[0], false, false);
        const auto sy = __builtin_amdgcn_permlane32_swap(a[1], c[1], false, false);
        const u32x4 w = {sx[0], sy[0], sx[1], sy[1]};
        *reinterpret_cast<u32x4*>(obase + (dt * 32 + 16 * pr + 8 * half) * 2) = w;
      }
  }
}

// Launch if the ping-pong kernel covers this call (D=64, no LSE, Gilbert-copy or plain K/V, no
// varlen, no head_mask_type); returns -1 when it does not, so the caller launches attn_fwd_kernel.
int launch_fwd_pp(const FwdParams& p, int dtype, bool pool, hipStream_t stream) {
  if (p.lse || p.kv_rows || p.cu_q || p.head_mask_type || !p.use_main) return -1;
  const dim3 grid(p.nbq * p.B * p.H);
  if (dtype == VB_DTYPE_BF16) {
    if (pool) hipLaunchKernelGGL((attn_fwd_pp_kernel<BF16, true>), grid, dim3(512), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_pp_kernel<BF16, false>), grid, dim3(512), 0, stream, p);
  } else {
    if (pool) hipLaunchKernelGGL((attn_fwd_pp_kernel<F16, true>), grid, dim3(512), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_pp_kernel<F16, false>), grid, dim3(512), 0, stream, p);
  }
  return check_launch("attn_fwd_pp_kernel");
}

}  // namespace vb

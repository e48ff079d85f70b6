// Software-pipelined block-sparse FMHA forward for head_dim 64, inference launches (no LSE), K/V in
// Gilbert-ordered contiguous copies (the CogVideoX module path). Same semantics, inputs and results
// (up to rounding order: none, the sums are the same) as attn_fwd_kernel<64, T, kPool, false, false,
// true> (vb_attn_fwd.hip): one 4-wave workgroup per (b, h, 128-row q-block), kept 128-key blocks as
// two 64-key tiles (diagonal first), then the pooled keys with a +log2(gap) bias, one lazy
// exp2-domain softmax, Q gathered and O scattered through q_rows.
//
// Why: on gfx950 the MFMAs of one wave and the VALU of another wave on the same SIMD barely overlap
// (tools/microbench/mfma_valu_overlap.hip: 0.96 of the sum of the two alone), while the same two
// streams interleaved inside ONE wave run at 0.71 of the sum. attn_fwd_kernel computes S(t), then
// the softmax of S(t), then P(t).V(t): every MFMA group waits on the VALU group before it. Here the
// wave computes S(t+1) while it runs the softmax of tile t, so its 8 S MFMAs have independent VALU
// work beside them, and the P.V MFMAs of the first 32 keys run beside the exp of the second 32:
//
//   iteration t:  [S(t+1) = K(t+1).Q^T]  x  [exp/sum/pack of S(t) keys 0-31]   (check)
//                 [P.V(t) keys 0-31]     x  [exp/sum/pack of S(t) keys 32-63]  (check)
//                 [P.V(t) keys 32-63]
//
// S(t+1) needs K(t+1) one tile earlier than the plain loop, so the LDS ring has 4 slots (64 KiB:
// two workgroups per CU, two waves per SIMD, which also gives the ~230 registers the two live S
// tiles need): tile t+3 is loaded while t+1 is consumed.
#include <type_traits>

#include "vb_attn_fwd.hpp"

namespace vb {

template <class T, bool kPool>
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_swp_kernel(const FwdParams p) {
  constexpr int D = 64, KS = D / 16, DT = D / 32;
  constexpr int kRowB = D * 2;
  constexpr int kMatBytes = kKT * kRowB;       // 8 KiB
  constexpr int kBufBytes = 2 * kMatBytes;     // K image, V image
  constexpr int kBufs = 4;
  constexpr int kChunks = kRowB / 16;
  constexpr int kRowsPerInst = 1024 / kRowB;
  constexpr int kInstPerWave = 2 * (kMatBytes / 1024) / 4;   // 4
  constexpr float kLazyBound = std::is_same<T, BF16>::value ? kLazyBoundBF16 : kLazyBoundF16;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kBufs * kBufBytes + kMaxBlocks * 2 + 16];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + kBufs * kBufBytes);
  int* list_n = reinterpret_cast<int*>(smem + kBufs * kBufBytes + kMaxBlocks * 2);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;

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

  // ---- kept key blocks (diagonal first), as attn_fwd_kernel ------------------------------------
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

  // ---- Q fragment, pre-scaled by scale*log2e (scores leave the MFMA in the exp2 domain) ---------
  const int qg = q0 + wave * 32 + l32;
  const bool qvalid = qg < Lq;
  int qrow = qvalid ? qg : Lq - 1;
  if (p.q_rows) qrow = p.q_rows[qrow];
  typename T::vec8 qf[KS];
  {
    const uint8_t* qp = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + (int64_t)qrow * p.qs[2]);
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const typename T::vec8*>(qp + (16 * s + 8 * half) * 2);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[s][e] = T::from_f32(T::to_f32(qf[s][e]) * p.c);
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(qf[s]));
  }
  __syncthreads();
  const int nkept = __builtin_amdgcn_readfirstlane(*list_n);
  int ntm = 2 * nkept;
  if (nkept > 0 && list[nkept - 1] == nbk - 1 && (nbk - 1) * kQBlk + kKT >= Lk) ntm -= 1;
  const int ntp = kPool ? (p.Lkp + kKT - 1) / kKT : 0;
  const int ntiles = ntm + ntp;

  // ---- LDS-DMA (as attn_fwd_kernel): waves 0-1 fill K, 2-3 fill V, swizzle applied on the source --
  const int my_mat = wave >> 1;
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
  const int my_row0 = (wave & 1) * kInstPerWave * kRowsPerInst + lane / kChunks;
#pragma unroll
  for (int i = 0; i < kInstPerWave; ++i) {
    const int r = my_row0 + i * kRowsPerInst;
    const int sl = lane % kChunks;
    my_rc[i] = 16 * (my_mat == 0 ? (sl ^ ((r >> 1) & 7)) : ((((sl >> 2) ^ ((r >> 1) & 1)) << 2) | (sl & 3)));
  }
  // tile t's keys: pooled flag, first key, valid keys; `blk_raw` = list[t >> 1]
  auto tile_src = [&](int t, int blk_raw) __attribute__((always_inline)) -> TileSrc {
    TileSrc s;
    if (t < ntm) {
      const int blk = __builtin_amdgcn_readfirstlane(blk_raw);
      s.pooled = 0;
      s.kstart = blk * kQBlk + (t & 1) * kKT;
      s.klen = min(kKT, Lk - s.kstart);
    } else {
      s.pooled = 1;
      s.kstart = (t - ntm) * kKT;
      s.klen = min(kKT, p.Lkp - s.kstart);
    }
    return s;
  };
  auto list_at = [&](int t) __attribute__((always_inline)) -> int {
    return t < ntm ? (int)list[min(t >> 1, kMaxBlocks - 1)] : 0;
  };
  auto issue = [&](const TileSrc src, int slot) __attribute__((always_inline)) {
    uint8_t* dst = smem + slot * kBufBytes + my_mat * kMatBytes + (wave & 1) * kInstPerWave * 1024;
    const bool pl = kPool && src.pooled;
    const int rowb = pl ? my_prowb : my_rowb;
    const int soff = __builtin_amdgcn_readfirstlane(src.kstart * rowb);
    if (src.klen == kKT) {
      const int vb0 = my_row0 * rowb;
#pragma unroll
      for (int i = 0; i < kInstPerWave; ++i)
        dma16(pl ? my_prsrc : my_rsrc, dst + i * 1024, vb0 + my_rc[i],
              __builtin_amdgcn_readfirstlane(soff + i * kRowsPerInst * rowb));
    } else {   // tail tile: rows past the last key replicate it (masked in the softmax)
#pragma unroll
      for (int i = 0; i < kInstPerWave; ++i) {
        const int r = min(my_row0 + i * kRowsPerInst, src.klen - 1);
        dma16(pl ? my_prsrc : my_rsrc, dst + i * 1024, r * rowb + my_rc[i], soff);
      }
    }
  };

  // ---- softmax state (exp2 domain, lazy running max: see attn_fwd_kernel) -------------------------
  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = 0.f, l = 0.f;   // m: the running max (kept for clarity; the output needs only l)
  (void)m;
  f32x16 cb;   // bias - m: the C seed of every S^T chain
#pragma unroll
  for (int r = 0; r < 16; ++r) cb[r] = 0.f;
  int cur_bias_bits = 0;
  bool first = true;
  f32x16 sA[2], sB[2];   // S^T of two consecutive tiles (even t in sA, odd t in sB)

  int k_lane[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) k_lane[ks] = k_off<D>(l32, 2 * ks + half);
  const int vrow = 4 * half + (lane & 15) / 4;
  const int vcol = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  uint32_t v_lane[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
    v_lane[dt] = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)smem)) +
                 v_off_bytes<D>(vrow, dt * 32 + vcol);

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

  // S^T of tile t (slot u) into s, seeded with the C operand cb (= its bias - m)
  auto compute_s = [&](f32x16 (&s)[2], int u) __attribute__((always_inline)) {
    const uint8_t* kl = smem + u * kBufBytes;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      typename T::vec8 kf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[ks] = lds_b128<T>(kl + kt * 32 * kRowB, k_lane[ks]);
      s[kt] = T::mfma32(kf[0], qf[0], cb);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) s[kt] = T::mfma32(kf[ks], qf[ks], s[kt]);
    }
  };
  auto set_bias = [&](float bias) __attribute__((always_inline)) {
    const int bias_bits = __builtin_amdgcn_readfirstlane(__float_as_int(bias));
    if (bias_bits != cur_bias_bits) {   // wave-uniform; where the pooled keys begin
      asm volatile("");
      const float db = bias - __int_as_float(cur_bias_bits);
#pragma unroll
      for (int r = 0; r < 16; ++r) cb[r] += db;
      cur_bias_bits = bias_bits;
    }
  };
  auto src_bias = [&](const TileSrc& src) __attribute__((always_inline)) -> float {
    return (kPool && src.pooled) ? p.pool_bias_l2 : 0.f;
  };

  // ---- pipeline ------------------------------------------------------------------------------------
  // Tile t sits in slot t % 4. Prologue: tiles 0-2 in flight, S(0) once tile 0 has landed.
  // Iteration t: wait for tile t+1, barrier (tile t+1 visible; slot (t-1) % 4 free: P.V(t-1) and
  // S(t) have read it... all waves finished iteration t-1), DMA tile t+3, S(t+1), softmax + P.V(t).
  TileSrc src_cur = tile_src(0, list_at(0));
  {
    TileSrc s1 = tile_src(1, list_at(1)), s2 = tile_src(2, list_at(2));
    if (ntiles > 0) issue(src_cur, 0);
    if (ntiles > 1) issue(s1, 1);
    if (ntiles > 2) issue(s2, 2);
    const int younger = min(ntiles - 1, 2);
    if (younger >= 2) VB_WAIT_VMCNT(2 * kInstPerWave);
    else if (younger == 1) VB_WAIT_VMCNT(kInstPerWave);
    else VB_WAIT_VMCNT(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    set_bias(src_bias(src_cur));
    if (ntiles > 0) compute_s(sA, 0);
  }
  int next_blk = list_at(3);   // list entry of the tile issued in iteration 0

  auto iteration = [&](int t, auto U, f32x16 (&s_cur)[2], f32x16 (&s_nxt)[2]) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;             // slot of tile t
    constexpr int u1 = (u + 1) % kBufs, u3 = (u + 3) % kBufs;
    const bool has_next = t + 1 < ntiles;
    // wait for this wave's part of tile t+1 (tile t+2 may stay in flight), then the barrier
    if (t + 2 < ntiles) VB_WAIT_VMCNT(kInstPerWave);
    else VB_WAIT_VMCNT(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + 3 < ntiles) {
      issue(tile_src(t + 3, next_blk), u3);
      next_blk = list_at(t + 4);
    }
    const TileSrc src_nxt = has_next ? tile_src(t + 1, list_at(t + 1)) : src_cur;
    // K fragments of tile t+1 (past the last tile: a stale slot, computed and never used, so the
    // S(t+1) MFMAs below need no branch)
    typename T::vec8 kf[2][KS];
    {
      const uint8_t* kl = smem + u1 * kBufBytes;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kf[kt][ks] = lds_b128<T>(kl + kt * 32 * kRowB, k_lane[ks]);
    }
    // V^T fragments of tile t, one 32-key half at a time; the asm reads are waited for explicitly
    s16x4 vlo[2][DT], vhi[2][DT];
    auto read_v = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int kk = 2 * kt + j;
        const int row0 = (kk >> 1) * 32 + 16 * (kk & 1);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          vlo[j][dt] = lds_tr4_asm(v_lane[dt], u * kBufBytes + kMatBytes + row0 * kRowB);
          vhi[j][dt] = lds_tr4_asm(v_lane[dt], u * kBufBytes + kMatBytes + (row0 + 8) * kRowB);
        }
      }
    };
    // tile t's tail mask and (first tile) exact max, before S(t+1) is seeded from cb
    const int klen = src_cur.klen;
    if (klen < kKT) {
      asm volatile("");
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= klen) s_cur[kt][r] = -INFINITY;
    }
    if (first) {
      asm volatile("");
      const float mt = max_xor32(fmaxf(half_max(s_cur[0]), half_max(s_cur[1])));
      m += mt;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s_cur[0][r] -= mt;
        s_cur[1][r] -= mt;
        cb[r] -= mt;
      }
      first = false;
    }
    set_bias(src_bias(src_nxt));
    read_v(0);
    // S(t+1) interleaved with the exp/sum/pack of tile t's first 32 keys: one MFMA, then a block of
    // the independent VALU, eight times
    typename T::vec8 pf[4];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s_nxt[kt] = T::mfma32(kf[kt][0], qf[0], cb);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) s_nxt[kt] = T::mfma32(kf[kt][ks], qf[ks], s_nxt[kt]);
    }
    float hs0 = exp_pack(s_cur[0], pf[0], pf[1]);
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);   // 5 VALU
    }
    // raise m by the rows' max mt of S half kt0.. (rare): rescale O, l, the seed, S(t) halves >= kt0
    // and S(t+1) (seeded before the raise)
    auto raise_m = [&](float mt, auto KT0) __attribute__((always_inline)) {
      constexpr int kt0 = decltype(KT0)::value;
      const float delta = fmaxf(max_xor32(mt), 0.f);
      const float alpha = exp2_fast(-delta);
      m += delta;
      l *= alpha;
#pragma unroll
      for (int i = 0; i < DT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        cb[r] -= delta;
        if (kt0 == 0) s_cur[0][r] -= delta;
        s_cur[1][r] -= delta;
        s_nxt[0][r] -= delta;
        s_nxt[1][r] -= delta;
      }
    };
    if (!__all(hs0 <= kLazyBound)) {
      asm volatile("");
      raise_m(half_max(s_cur[0]), std::integral_constant<int, 0>{});
      hs0 = exp_pack(s_cur[0], pf[0], pf[1]);
    }
    l += hs0;
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[0][0]), "+v"(vhi[0][0]), "+v"(vlo[0][1]), "+v"(vhi[0][1]),
                 "+v"(vlo[1][0]), "+v"(vhi[1][0]), "+v"(vlo[1][1]), "+v"(vhi[1][1]));
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] = T::mfma32(join8<T>(vlo[j][dt], vhi[j][dt]), pf[j], o[dt]);
    read_v(1);
    float hs1 = exp_pack(s_cur[1], pf[2], pf[3]);
    if (!__all(hs1 <= kLazyBound)) {
      asm volatile("");
      raise_m(half_max(s_cur[1]), std::integral_constant<int, 1>{});
      hs1 = exp_pack(s_cur[1], pf[2], pf[3]);
    }
    l += hs1;
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[0][0]), "+v"(vhi[0][0]), "+v"(vlo[0][1]), "+v"(vhi[0][1]),
                 "+v"(vlo[1][0]), "+v"(vhi[1][0]), "+v"(vlo[1][1]), "+v"(vhi[1][1]));
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] = T::mfma32(join8<T>(vlo[j][dt], vhi[j][dt]), pf[2 + j], o[dt]);
    src_cur = src_nxt;
  };
  // unrolled by the ring size: compile-time slots, and the two S tiles alternate between sA and sB
  for (int t0 = 0; t0 < ntiles; t0 += kBufs) {
    iteration(t0, std::integral_constant<int, 0>{}, sA, sB);
    if (t0 + 1 < ntiles) iteration(t0 + 1, std::integral_constant<int, 1>{}, sB, sA);
    if (t0 + 2 < ntiles) iteration(t0 + 2, std::integral_constant<int, 2>{}, sA, sB);
    if (t0 + 3 < ntiles) iteration(t0 + 3, std::integral_constant<int, 3>{}, sB, sA);
  }

  // ---- epilogue (as attn_fwd_kernel) ----------------------------------------------------------------
  const float lt = add_xor32(l);
  const float inv = (lt > 0.f) ? 1.0f / lt : 0.f;
  if (qvalid) {
    uint8_t* obase = reinterpret_cast<uint8_t*>(p.out) + 2 * (b * p.os[0] + h * p.os[1] + (int64_t)qrow * p.os[2]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
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

int launch_fwd_swp(const FwdParams& p, int dtype, bool pool, hipStream_t stream) {
  if (p.lse || p.kv_rows || p.cu_q || p.head_mask_type || !p.use_main) return -1;
  const dim3 grid(p.nbq * p.B * p.H);
  if (dtype == VB_DTYPE_BF16) {
    if (pool) hipLaunchKernelGGL((attn_fwd_swp_kernel<BF16, true>), grid, dim3(kThreads), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_swp_kernel<BF16, false>), grid, dim3(kThreads), 0, stream, p);
  } else {
    if (pool) hipLaunchKernelGGL((attn_fwd_swp_kernel<F16, true>), grid, dim3(kThreads), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_swp_kernel<F16, false>), grid, dim3(kThreads), 0, stream, p);
  }
  return check_launch("attn_fwd_swp_kernel");
}

}  // namespace vb

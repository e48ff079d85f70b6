// Block-sparse FMHA forward for head_dim 64 on v_mfma_f32_16x16x32 (inference launches: no LSE; K/V
// in Gilbert-ordered contiguous copies, the CogVideoX module path). Same semantics and inputs as
// attn_fwd_kernel<64, T, kPool, false, false, true> (vb_attn_fwd.hip): one 4-wave workgroup per
// (b, h, 128-row q-block), kept 128-key blocks as two 64-key tiles (diagonal first), then the pooled
// keys with a +log2(gap) bias, one lazy exp2-domain softmax, Q gathered and O scattered through
// q_rows; the same 3-slot LDS-DMA ring and K/V images.
//
// Why: on gfx950 the same bf16 FLOPs issued as v_mfma_f32_16x16x32 run 21 % faster than as
// v_mfma_f32_32x32x16 alone, and 13 % faster beside another wave's exp/add/pack stream
// (tools/microbench/mfma_valu_overlap.hip, profiles/r02_mfma_valu_overlap_m16.json).
//
// Operand maps (wave64; c = lane & 15, g = lane >> 4):
//   A [16 x 32]: lane supplies row c, k = 8g .. 8g+7;  B [32 x 16]: column c, k = 8g .. 8g+7;
//   C [16 x 16]: lane holds column c, rows 4g .. 4g+3.
// Per wave: 32 queries = two q-tiles (qt) of 16, a 64-key tile = four key-tiles (kt) of 16.
//   S^T(kt, qt) = K(kt) . Q(qt)^T: A = K rows 16kt + c, d chunk 4ks + g (ds_read_b128 of the K
//     image), B = Q fragment (query 16qt + c, d 32ks + 8g..); C: lane holds query 16qt + c, keys
//     16kt + 4g + r. A query's 64 keys are spread over the four lanes c, c+16, c+32, c+48.
//   O^T(dt, qt) += V^T(dt) . P^T(qt) per 32-key half h: B = P packed from S^T(2h, qt) and
//     S^T(2h+1, qt) (k = 8g + e <-> key 32h + 4g + e (e < 4), 32h + 16 + 4g + e - 4 (e >= 4)), A = V^T
//     rows d = 16dt + c at the same key order, two ds_read_b64_tr_b16 per operand (key rows
//     32h + 4g .. +3 and 32h + 16 + 4g .. +3). No LDS round trip for P.
#include <type_traits>

#include "vb_attn_fwd.hpp"

namespace vb {

// V image of this kernel: [64 keys][64 d], 32-byte granules XOR-swizzled by (row >> 1) & 3. A
// 32-lane half of a transposed read covers rows 4g + 0..3 for g in {0,1} (8 rows) at the same 16
// columns: rows of one parity then land in four distinct granules and the two parities in the two
// 128-byte halves, so the 32 lanes' 8-byte pieces cover the 256-byte bank row once (the
// attn_fwd_kernel image, built for a 4-row footprint, puts rows r and r+4 on the same banks).
// Rows +16 / +32 keep the swizzle, so those offsets stay instruction immediates.
__device__ __forceinline__ int v16_off(int row, int col) {
  return row * 128 + 32 * ((col >> 4) ^ ((row >> 1) & 3)) + (col & 15) * 2;
}

// max / sum over the four lanes of a query (c, c+16, c+32, c+48)
__device__ __forceinline__ float max_xor48(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float y = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(y), __float_as_uint(y), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float add_xor48(float x) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  const float y = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(y), __float_as_uint(y), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

template <class T, bool kPool>
__global__ void __launch_bounds__(kThreads, 3) attn_fwd_m16_kernel(const FwdParams p) {
  constexpr int D = 64;
  constexpr int kRowB = D * 2;
  constexpr int kMatBytes = kKT * kRowB;       // 8 KiB
  constexpr int kBufBytes = 2 * kMatBytes;     // K image, V image
  constexpr int kBufs = 3;
  constexpr int kChunks = kRowB / 16;
  constexpr int kRowsPerInst = 1024 / kRowB;
  constexpr int kInstPerWave = 2 * (kMatBytes / 1024) / 4;   // 4
  constexpr float kLazyBound = std::is_same<T, BF16>::value ? kLazyBoundBF16 : kLazyBoundF16;
  typedef f32x4 f32x4_t;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kBufs * kBufBytes + kMaxBlocks * 2 + 16];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + kBufs * kBufBytes);
  int* list_n = reinterpret_cast<int*>(smem + kBufs * kBufBytes + kMaxBlocks * 2);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15;
  const int g = lane >> 4;

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

  // ---- Q fragments (B operands), pre-scaled by scale*log2e: query 16qt + c, d 32ks + 8g .. +7 ----
  int qrow[2];
  bool qvalid[2];
  typename T::vec8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qg = q0 + wave * 32 + 16 * qt + c;
    qvalid[qt] = qg < Lq;
    int r = qvalid[qt] ? qg : Lq - 1;
    if (p.q_rows) r = p.q_rows[r];
    qrow[qt] = r;
    const uint8_t* qp = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + (int64_t)r * p.qs[2]);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[qt][ks] = *reinterpret_cast<const typename T::vec8*>(qp + (32 * ks + 8 * g) * 2);
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[qt][ks][e] = T::from_f32(T::to_f32(qf[qt][ks][e]) * p.c);
      asm volatile("" : "+v"(qf[qt][ks]));
    }
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
    // K: the attn_fwd_kernel image; V: 32-byte granules XOR (row >> 1) & 3 (v16_off below)
    my_rc[i] = 16 * (my_mat == 0 ? (sl ^ ((r >> 1) & 7)) : ((((sl >> 1) ^ ((r >> 1) & 3)) << 1) | (sl & 1)));
  }
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

  // ---- per-lane softmax state (two queries: 16qt + c) ------------------------------------------------
  f32x4_t o[4][2];   // O^T tiles: d 16dt + 4g + r, query 16qt + c
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) o[dt][qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float l[2] = {0.f, 0.f};
  f32x4_t cb[2];     // bias - m of each query: the C seed of its S^T chains
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) cb[qt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  int cur_bias_bits = 0;
  bool first = true;

  // loop-invariant lane addresses: K rows 16kt + c, chunk 4ks + g; V^T transposed reads at key row
  // 4g + (c >> 2) (+16 / +32 / +48 via the immediate), columns 16dt + 4 (c & 3)
  int k_lane[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) k_lane[ks] = k_off<D>(c, 4 * ks + g);   // row 16kt + c: same swizzle, + 16kt rows
  const uint32_t smem_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)smem));

  auto tile_step = [&](auto U, float bias, int klen) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    const uint8_t* kl = smem + u * kBufBytes;
    {
      const int bias_bits = __builtin_amdgcn_readfirstlane(__float_as_int(bias));
      if (bias_bits != cur_bias_bits) {   // wave-uniform; where the pooled keys begin
        asm volatile("");
        const float db = bias - __int_as_float(cur_bias_bits);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) cb[qt] += db;
        cur_bias_bits = bias_bits;
      }
    }
    // S^T: 4 key-tiles x 2 q-tiles, two k-steps each (16 MFMAs); a K fragment serves both q-tiles
    f32x4_t s[4][2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      typename T::vec8 kf[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        kf[ks] = *reinterpret_cast<const typename T::vec8*>(kl + 16 * kt * kRowB + k_lane[ks]);
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        s[kt][qt] = T::mfma16(kf[0], qf[qt][0], cb[qt]);
        s[kt][qt] = T::mfma16(kf[1], qf[qt][1], s[kt][qt]);
      }
    }
    // V^T operands of one 32-key half: per d-tile, rows (keys) 32h + 4g.. and 32h + 16 + 4g..
    s16x4 vlo[4], vhi[4];
    auto read_v = [&](int hh) __attribute__((always_inline)) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const uint32_t a = smem_base + u * kBufBytes + kMatBytes + v16_off(32 * hh + 4 * g + (c >> 2), 16 * dt + 4 * (c & 3));
        vlo[dt] = lds_tr4_asm(a, 0);
        vhi[dt] = lds_tr4_asm(a, 16 * kRowB);
      }
    };
    read_v(0);
    if (klen < kKT) {
      asm volatile("");
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * kt + 4 * g + r >= klen) s[kt][0][r] = s[kt][1][r] = -INFINITY;
    }
    if (first) {   // m := the first tile's exact row max
      asm volatile("");
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        float mx = s[0][qt][0];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
        const float mt = max_xor48(mx);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) s[kt][qt] -= mt;
        cb[qt] -= mt;
      }
      first = false;
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      typename T::vec8 pb[2];
      float hs[2];
      auto exps = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          float e[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            e[r] = exp2_fast(s[2 * hh][qt][r]);
            e[4 + r] = exp2_fast(s[2 * hh + 1][qt][r]);
          }
          hs[qt] = ((e[0] + e[4]) + (e[1] + e[5])) + ((e[2] + e[6]) + (e[3] + e[7]));
          u32x4 w;
#pragma unroll
          for (int k = 0; k < 4; ++k) w[k] = pack2<T>(e[2 * k], e[2 * k + 1]);
          pb[qt] = __builtin_bit_cast(typename T::vec8, w);
        }
      };
      exps();
      if (!__all(fmaxf(hs[0], hs[1]) <= kLazyBound)) {
        asm volatile("");
        // raise each query's m to its rows' max over this half and the rest of the tile
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          float mx = s[2 * hh][qt][0];
#pragma unroll
          for (int kt = 2 * hh; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kt][qt][r]);
          const float delta = fmaxf(max_xor48(mx), 0.f);
          const float alpha = exp2_fast(-delta);
          l[qt] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt) o[dt][qt] *= alpha;
          cb[qt] -= delta;
#pragma unroll
          for (int kt = 2 * hh; kt < 4; ++kt) s[kt][qt] -= delta;
        }
        exps();
      }
      l[0] += hs[0];
      l[1] += hs[1];
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[0]), "+v"(vhi[0]), "+v"(vlo[1]), "+v"(vhi[1]),
                   "+v"(vlo[2]), "+v"(vhi[2]), "+v"(vlo[3]), "+v"(vhi[3]));
      s16x4 wlo[4], whi[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        wlo[dt] = vlo[dt];
        whi[dt] = vhi[dt];
      }
      if (hh == 0) read_v(1);   // the second half's V^T reads land while these MFMAs run
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) o[dt][qt] = T::mfma16(join8<T>(wlo[dt], whi[dt]), pb[qt], o[dt][qt]);
    }
  };

  // ---- 3-slot ring, slot-unrolled loop (as attn_fwd_kernel's Gilbert-copy path) --------------------
  TileSrc slot_src[kBufs];
  slot_src[0] = tile_src(0, list_at(0));
  if (ntiles > 0) issue(slot_src[0], 0);
  slot_src[1] = tile_src(1, list_at(1));
  if (ntiles > 1) issue(slot_src[1], 1);
  int next_blk = list_at(2);
  auto body = [&](int t, auto U) __attribute__((always_inline)) {
    constexpr int uu = decltype(U)::value;
    constexpr int un = (uu + kBufs - 1) % kBufs;
    const int ti = t + kBufs - 1;
    const int younger = min(ntiles - 1 - t, kBufs - 2);
    if (younger >= 1) VB_WAIT_VMCNT(kInstPerWave);
    else VB_WAIT_VMCNT(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (ti < ntiles) {
      slot_src[un] = tile_src(ti, next_blk);
      issue(slot_src[un], un);
      next_blk = list_at(ti + 1);
    }
    const TileSrc src = slot_src[uu];
    tile_step(U, (kPool && src.pooled) ? p.pool_bias_l2 : 0.f, src.klen);
  };
  for (int t0 = 0; t0 < ntiles; t0 += kBufs) {
    body(t0, std::integral_constant<int, 0>{});
    if (t0 + 1 < ntiles) body(t0 + 1, std::integral_constant<int, 1>{});
    if (t0 + 2 < ntiles) body(t0 + 2, std::integral_constant<int, 2>{});
  }

  // ---- epilogue: lane writes d 16dt + 4g .. +3 of queries 16qt + c ---------------------------------
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const float lt = add_xor48(l[qt]);
    const float inv = (lt > 0.f) ? 1.0f / lt : 0.f;
    if (!qvalid[qt]) continue;
    uint8_t* obase = reinterpret_cast<uint8_t*>(p.out) + 2 * (b * p.os[0] + h * p.os[1] + (int64_t)qrow[qt] * p.os[2]);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      u32x2 w;
      w[0] = pack2<T>(o[dt][qt][0] * inv, o[dt][qt][1] * inv);
      w[1] = pack2<T>(o[dt][qt][2] * inv, o[dt][qt][3] * inv);
      *reinterpret_cast<u32x2*>(obase + (16 * dt + 4 * g) * 2) = w;
    }
  }
}

int launch_fwd_m16(const FwdParams& p, int dtype, bool pool, hipStream_t stream) {
  if (p.lse || p.kv_rows || p.cu_q || p.head_mask_type || !p.use_main) return -1;
  const dim3 grid(p.nbq * p.B * p.H);
  if (dtype == VB_DTYPE_BF16) {
    if (pool) hipLaunchKernelGGL((attn_fwd_m16_kernel<BF16, true>), grid, dim3(kThreads), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_m16_kernel<BF16, false>), grid, dim3(kThreads), 0, stream, p);
  } else {
    if (pool) hipLaunchKernelGGL((attn_fwd_m16_kernel<F16, true>), grid, dim3(kThreads), 0, stream, p);
    else hipLaunchKernelGGL((attn_fwd_m16_kernel<F16, false>), grid, dim3(kThreads), 0, stream, p);
  }
  return check_launch("attn_fwd_m16_kernel");
}

}  // namespace vb

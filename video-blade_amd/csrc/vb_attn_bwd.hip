// Block-sparse FMHA backward for gfx950 (MI355X): FlashAttention-2 gradient semantics, deterministic.
//
// Replaces the backward of the external block_sparse_attn_func (mit-han-lab/Block-Sparse-Attention)
// as the reference's autograd reaches it (cogvideox/train/special_attentions_local/TrainRelated/
// cogvideo_blocksparseattn.py:316-320 sparse call, :106-109 dense pooled call) together with the
// autograd of the surrounding adaptive_block_sparse_attn ops (:366-393):
//   * the softmax LSE is a constant (the library's backward ignores its gradient), hence the combine
//     weight a = exp(lse1 - M)/(...) is a constant too: dO1 = a*dO, dO2 = (1-a)*dO;
//   * each branch back-propagates with its own output and LSE;
//   * pooled-branch K/V gradients flow back through the mean pool (replicate padding folds onto the
//     last token) and the Gilbert gather (a scatter to the caller's rows).
// The branch weight is folded into the row statistic: a*P1 = exp2(S*c - (lse1*log2e - log2 a)),
// so dO itself is used unscaled and Delta = rowsum(dO * O_branch) (FA2's D_i) per branch.
//
// Kernels (all 256 threads = 4 waves, v_mfma_f32_32x32x16, operand maps in vb_tiles.hpp):
//   bwd_prep_kernel   per row: -Delta1/2, L'1/2 -> stats [B*H][ntile64][4][64] fp32 (Delta negated:
//                     it seeds the dP accumulators, see below); optional
//                     reordered contiguous copies of q and dO (one gather pass instead of one per
//                     key block that reads them)
//   bwd_dkdv_kernel   one workgroup per (b, h, 128-key block); wave = 32 keys held in registers;
//                     streams the 64-row Q / dO tiles of every q-block that keeps this key block
//                     (mask column; all q-blocks for pooled keys) through LDS by LDS-DMA:
//                       S = Q.K^T, dP = dO.V^T         (C: lane = key, registers = q rows)
//                       P = exp2(S c - L'), dS = P (dP - Delta)
//                       dV^T += dO^T.P, dK^T += Q^T.dS (A = ds_read_b64_tr_b16 of the Q/dO tiles)
//                     pooled keys -> fp32 workspace; full-resolution keys -> dk/dv rows (kv_rows),
//                     adding the mean-pool adjoint of the pooled grads
//   bwd_dq_kernel     one workgroup per (b, h, 128-row q-block), the forward's geometry: streams the
//                     kept K/V tiles then the pooled ones:
//                       S^T = K.Q^T, dP^T = V.dO^T      (C: lane = query, registers = keys)
//                       dQ^T += K^T.dS^T                (A = transposed read of the K tile)
// No atomics: every gradient element is written by exactly one workgroup, so results are
// bit-reproducible run to run (the reference's deterministic=True).
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>

#include "vb_attn_bwd.hpp"

namespace vb {

// ------------------------------------------------------------------------------------------------
// prep: one thread per 16-byte chunk of a row
// ------------------------------------------------------------------------------------------------
template <class T>
__global__ void __launch_bounds__(256) bwd_prep_kernel(const PrepParams p) {
  const int CH = p.D / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t rows_per_bh = (int64_t)p.ntile * 64;
  const int64_t total = (int64_t)p.B * p.H * rows_per_bh * CH;
  if (idx >= total) return;  // CH divides 64: whole row groups leave together
  const int ch = idx % CH;
  const int64_t rid = idx / CH;
  const int g = rid % rows_per_bh;
  const int bh = rid / rows_per_bh;
  const int b = bh / p.H, h = bh % p.H;
  int Lq = p.Lq, qrow0 = 0;
  if (p.cu_q) { qrow0 = p.cu_q[b]; Lq = p.cu_q[b + 1] - qrow0; }
  const bool valid = g < Lq;
  const int row = valid ? (p.q_rows ? p.q_rows[g] : g) : 0;
  float d1 = 0.f, d2 = 0.f;
  if (valid) {
    const int64_t r = qrow0 + row;
    const u32x4 dov = *reinterpret_cast<const u32x4*>(
        reinterpret_cast<const uint8_t*>(p.dout) + 2 * (b * p.dos[0] + h * p.dos[1] + r * p.dos[2] + ch * 8));
    const u32x4 ov = *reinterpret_cast<const u32x4*>(
        reinterpret_cast<const uint8_t*>(p.out) + 2 * (b * p.os[0] + h * p.os[1] + r * p.os[2] + ch * 8));
    u32x4 o2v = {0, 0, 0, 0};
    if (p.out2)
      o2v = *reinterpret_cast<const u32x4*>(
          reinterpret_cast<const uint8_t*>(p.out2) + 2 * (b * p.o2s[0] + h * p.o2s[1] + r * p.o2s[2] + ch * 8));
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const float x = T::bits_to_f32((dov[e] >> (16 * s)) & 0xffff);
        d1 += x * T::bits_to_f32((ov[e] >> (16 * s)) & 0xffff);
        d2 += x * T::bits_to_f32((o2v[e] >> (16 * s)) & 0xffff);
      }
    if (p.q_r) {
      const u32x4 qv = *reinterpret_cast<const u32x4*>(
          reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + r * p.qs[2] + ch * 8));
      const int64_t dst = 2 * (((int64_t)bh * p.Lq + g) * p.D + ch * 8);
      *reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(p.q_r) + dst) = qv;
      *reinterpret_cast<u32x4*>(reinterpret_cast<uint8_t*>(p.do_r) + dst) = dov;
    }
  }
  // reduce over the CH consecutive lanes of this row (CH in {8, 16}, aligned groups)
  for (int o = 1; o < CH; o <<= 1) {
    d1 += __shfl_xor(d1, o);
    d2 += __shfl_xor(d2, o);
  }
  if (ch != 0) return;
  float l1 = bwd::kBigL, l2 = bwd::kBigL;
  if (valid) {
    const int64_t li = (int64_t)bh * p.Lq + row;
    const float a = p.alpha ? p.alpha[li] : 1.f;
    const float lse1 = p.lse[li];
    // a * P1 = exp2(S c - (lse1 log2e - log2 a)); rows with no kept key (lse = -inf) or a = 0
    // contribute nothing
    if (lse1 > -INFINITY && a > 0.f) l1 = fminf(lse1 * kLog2e - __log2f(a), bwd::kBigL);
    if (p.lse2) {
      const float w2 = round_to<T>(1.f - a);  // the reference's bf16 (1 - alpha), :393
      const float lse2 = p.lse2[li];
      if (lse2 > -INFINITY && w2 > 0.f) l2 = fminf(lse2 * kLog2e - __log2f(w2), bwd::kBigL);
    }
  } else {
    d1 = d2 = 0.f;
  }
  float* st = p.stats + ((int64_t)bh * p.ntile + g / 64) * 256 + (g & 63);
  st[0] = l1;
  st[64] = -d1;
  st[128] = l2;
  st[192] = -d2;
}

// ------------------------------------------------------------------------------------------------
// dK / dV: one workgroup per (b, h, 128-key block)
// ------------------------------------------------------------------------------------------------
#ifndef VB_BWD_SEED128
#define VB_BWD_SEED128 0    // D=128: dP seeded with -Delta too (measured 6 % slower on Wan's dK/dV)
#endif
#ifndef VB_DKDV_PRIO64
#define VB_DKDV_PRIO64 1   // measured (cog backward): 1 1.013x, 3 1.009x
#endif
#ifndef VB_DKDV_PRIO128
#define VB_DKDV_PRIO128 0  // one wave per SIMD at D=128: nothing to arbitrate
#endif
#ifndef VB_DKDV_WAVES_D64
#define VB_DKDV_WAVES_D64 2   // waves per SIMD the D=64 dK/dV kernel is register-budgeted for
#endif
#ifndef VB_ML_PYR_WAVES
// waves per multi-level pooled dK/dV workgroup at D=64: 2 = 64-row items on a 2-slot ring, four
// workgroups per CU (vb_ml_attn_bwd 1.15x over 4 = 128-row items, dk bit-identical;
// profiles/archive/r05_ml_bwd_pyr2_ab.log). D=128 keeps 4 (two waves spill there).
#define VB_ML_PYR_WAVES 2
#endif
#ifndef VB_ML_LONG_FIRST
#define VB_ML_LONG_FIRST 1   // multi-level pooled dK/dV items in level 8, 4, 2 order (longest first; 0: 2, 4, 8)
#endif
// kW: waves per workgroup (4, or 2 for the multi-level pooled items: an item is 32 kW pyramid rows,
// so a level-2 item covers one key block and walks its own q-list instead of a union, and a level-4
// or level-8 item half as many blocks; the union walk leaves fewer waves idle).
template <int D, class T, bool kPooled, bool kML = false, int kW = 4>
__global__ void __launch_bounds__(kW * 64, D == 128 ? 1 : VB_DKDV_WAVES_D64) bwd_dkdv_kernel(const BwdParams p) {
  using namespace bwd;
  static_assert(kW == 4 || (kML && kPooled), "2-wave workgroups: the multi-level pooled items only");
  constexpr int kRows = 32 * kW;             // keys (pyramid rows) per work item
  // s_setprio 1 around the MFMA chains (bit 0: S and dP, bit 1: the dV/dK steps)
  constexpr int kPrioKV = D == 128 ? VB_DKDV_PRIO128 : VB_DKDV_PRIO64;
  constexpr int KS = D / 16;
  constexpr int DT = D / 32;
  constexpr int RB = D * 2;                 // bytes per row
  constexpr int kTileBytes = kT * RB;       // one 64-row Q (or dO) tile
  constexpr int kInstTile = kTileBytes / 1024;
  constexpr int kRowsPerInst = 1024 / RB;
  constexpr int kCh = RB / 16;
  constexpr int kInst = 2 * kInstTile + 1;  // Q, dO, stats (1 KiB)
  constexpr int kBufBytes = 2 * kTileBytes + 1024;
  // LDS ring: tile t read, t+1 in flight, t+2 being issued; kW = 2: a 2-slot ring (38 KiB with the
  // lists), so four 2-wave workgroups fit a CU (two waves per SIMD, as the 4-wave form)
  constexpr int kBufs = kW == 2 ? 2 : 3;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kBufs * kBufBytes + kMaxBlocks * 3 + 16];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + kBufs * kBufBytes);
  int* list_n = reinterpret_cast<int*>(smem + kBufs * kBufBytes + kMaxBlocks * 2);
  uint8_t* list_bits = smem + kBufs * kBufBytes + kMaxBlocks * 2 + 16;   // multi-level: active blocks

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;

  const int BH = p.B * p.H;
  const int nkb = kPooled ? p.nbkp : p.nbk;
  // pooled-key blocks see every q-block: their work is split into psplit q-block ranges (split
  // innermost, so a key block's workgroups run together); main blocks XCD-contiguous
  // Main blocks: the `heavy_rows` last key blocks of every head (CogVideoX's forced dense text
  // columns, kept by every q-block: ~8x the average column's tiles) go first over all XCDs, then
  // each XCD takes a contiguous head-major range with key blocks in descending order. Ascending
  // order put every head's two heavy columns at the end of its range, so the last head of each
  // XCD's range left a long tail (measured: 1.26 waves per SIMD on average at 2 possible).
  const int split = kPooled ? (int)blockIdx.x % p.psplit : 0;
  int bh, kblk;
  int ml_e = 0, ml_m = 0;   // multi-level pooled items: level exponent and pyramid block
  if (kML && kPooled && VB_ML_LONG_FIRST) {
    // longest items first: a level-8 block's q-list is the union over 8 key blocks (≈4x a level-2
    // item's tiles), so level 8, then 4, then 2, each spread over the heads (consecutive
    // workgroups = different heads, so different XCDs); placement only, the results are the same
    int lin = (int)blockIdx.x;
    ml_e = 3;
    auto nit = [&](int e) { return ((p.Lpad >> e) + kRows - 1) / kRows; };   // items of level e
    while (ml_e > 1 && lin >= nit(ml_e) * BH) { lin -= nit(ml_e) * BH; --ml_e; }
    bh = lin % BH;
    ml_m = lin / BH;
    kblk = 0;
  } else if (kPooled) {
    const int lin = (int)blockIdx.x / p.psplit;
    bh = lin / nkb;
    kblk = lin % nkb;
  } else {
    const int hr = kML ? 0 : min(p.heavy_rows, nkb);
    const int n_heavy = hr * BH;
    if ((int)blockIdx.x < n_heavy) {
      kblk = nkb - 1 - (int)(blockIdx.x / BH);
      bh = blockIdx.x % BH;
    } else {
      const int cols_left = nkb - hr;
      const int lin = xcd_linear(blockIdx.x - n_heavy, cols_left * BH);
      bh = lin / cols_left;
      kblk = cols_left - 1 - lin % cols_left;
    }
  }
  const int b = bh / p.H, h = bh % p.H;

  int Lq = p.Lq, Lk = p.Lk;
  int64_t qrow0 = 0, krow0 = 0;
  if (p.cu_q) {
    qrow0 = p.cu_q[b]; Lq = p.cu_q[b + 1] - p.cu_q[b];
    krow0 = p.cu_k[b]; Lk = p.cu_k[b + 1] - p.cu_k[b];
  }
  int Lkey = kPooled ? p.Lkp : Lk;
  int k0 = kblk * kBlk;
  // multi-level: level e (p = 2^e) of this work item, its pyramid region start and row count;
  // pooled items number the level-2, then level-4, then level-8 pyramid blocks
  int ml_row0 = 0;
  if (!(kML && kPooled && VB_ML_LONG_FIRST)) ml_m = kblk;
  if (kML) {
    const MlGeom gm(p.Lpad);
    if (kPooled && !VB_ML_LONG_FIRST) {
      ml_e = 1;
      auto nit = [&](int e) { return ((p.Lpad >> e) + kRows - 1) / kRows; };
      while (ml_e < 3 && ml_m >= nit(ml_e)) { ml_m -= nit(ml_e); ++ml_e; }
    }
    ml_row0 = gm.off[ml_e];
    Lkey = kPooled ? p.Lpad >> ml_e : Lk;
    k0 = ml_m * (kPooled ? kRows : kBlk);
  }
  if (k0 >= Lkey || Lq <= 0) return;
  const int nbq = (Lq + kBlk - 1) / kBlk;

  bool nan_head = false;
  const uint8_t* mcol = nullptr;
  if (!kPooled || kML) {
    const uint8_t* mh = head_mask_base(p.mask, p.ms, p.head_mask_type, p.H, b, h, nan_head, p.hm_mode);
    if (mh) mcol = mh + (kML ? ((k0 << ml_e) >> 7) : kblk);   // the item's first key block
  }
  const int qlo = (kPooled && !kML) ? split * nbq / p.psplit : 0;
  const int qhi = (kPooled && !kML) ? (split + 1) * nbq / p.psplit : nbq;
  if (kML) {
    // q-blocks where any of this item's 2^e key blocks has level 2^e; bit e' = block ml_m*2^e + e'
    if (threadIdx.x < 64) {
      const int pl = 1 << ml_e;
      const int nblk_here = min((kRows << ml_e) >> 7, p.nbk - ((k0 << ml_e) >> 7));
      int n = 0;
      for (int i0 = 0; i0 < nbq; i0 += 64) {
        const int i = i0 + lane;
        int bits = 0;
        if (i < nbq)
          for (int e = 0; e < nblk_here; ++e) bits |= (mcol[(int64_t)i * p.ms[2] + e] == pl) << e;
        const unsigned long long bal = __ballot(bits != 0);
        if (bits) {
          const int pos = n + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
          list[pos] = (uint16_t)i;
          list_bits[pos] = (uint8_t)bits;
        }
        n += __popcll(bal);
      }
      if (lane == 0) *list_n = n;
    }
  } else if (threadIdx.x < 64) {
    int n = 0;
    for (int i0 = qlo; i0 < qhi; i0 += 64) {
      const int i = i0 + lane;
      const bool keep = (i < qhi) && (mcol == nullptr || mcol[(int64_t)i * p.ms[2]] != 0);
      const unsigned long long bal = __ballot(keep);
      if (keep) {
        const int pos = n + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
        list[pos] = (uint16_t)i;
      }
      n += __popcll(bal);
    }
    if (lane == 0) *list_n = n;
  }

  // this wave's 32 keys as B operands (lane = key, d = 16 ks + 8 half + 0..7)
  const int key = k0 + wave * 32 + l32;
  const bool kvalid = key < Lkey;
  const int keyc = kvalid ? key : Lkey - 1;
  const uint8_t* kb = (kPooled && !kML)
      ? reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1] + (int64_t)keyc * p.kps[2])
      : reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1] + (krow0 + ml_row0 + keyc) * p.ks[2]);
  const uint8_t* vb_ = (kPooled && !kML)
      ? reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1] + (int64_t)keyc * p.vps[2])
      : reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1] + (krow0 + ml_row0 + keyc) * p.vs[2]);
  // multi-level: which of the item's key blocks this lane's key belongs to, and the logit bias
  const int my_blk_bit = kML ? (wave * 32 + l32) / (kBlk >> ml_e) : 0;
  const float lvl_bias = (float)ml_e;
  typename T::vec8 kf[KS], vf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    kf[s] = *reinterpret_cast<const typename T::vec8*>(kb + (16 * s + 8 * half) * 2);
    vf[s] = *reinterpret_cast<const typename T::vec8*>(vb_ + (16 * s + 8 * half) * 2);
  }
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    asm volatile("" : "+v"(kf[s]));
    asm volatile("" : "+v"(vf[s]));
  }
  __syncthreads();
  const int nlist = __builtin_amdgcn_readfirstlane(*list_n);
  int ntiles = 2 * nlist;
  if (nlist > 0 && list[nlist - 1] == nbq - 1 && (nbq - 1) * kBlk + kT >= Lq) ntiles -= 1;

  const uint8_t* qsrc = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + qrow0 * p.qs[2]);
  const uint8_t* dosrc = reinterpret_cast<const uint8_t*>(p.dout) + 2 * (b * p.dos[0] + h * p.dos[1] + qrow0 * p.dos[2]);
  const int qrowb = 2 * (int)p.qs[2], dorowb = 2 * (int)p.dos[2];   // host: every slice < 2 GiB
  const float* stsrc = p.stats + (int64_t)bh * p.ntile * 256;

  // Tile t (64 q rows) -> ring slot t % kBufs by LDS-DMA through buffer descriptors: this wave
  // issues instructions i = wave + 4k (i < kInstTile: Q, then dO, then the stats KiB). A lane's
  // part of each instruction (row within the tile, swizzled chunk) is a fixed voffset; the tile's
  // first row is the scalar soffset. Rows past Lq read as zeros (their stats make P = 0).
  constexpr int kHi = (kInst + kW - 1) / kW, kLo = kInst / kW;  // DMA instructions per wave and tile
  const bool many = wave < (kInst % kW);
  const srd_t q_srd = make_srd(qsrc, (int)((int64_t)(Lq - 1) * qrowb + RB));
  const srd_t do_srd = make_srd(dosrc, (int)((int64_t)(Lq - 1) * dorowb + RB));
  const srd_t st_srd = make_srd(stsrc, p.ntile * 1024);
  int voff[kHi];
#pragma unroll
  for (int k = 0; k < kHi; ++k) {
    const int i = wave + kW * k;
    voff[k] = lane * 16;
    if (i < 2 * kInstTile) {
      const int ii = i < kInstTile ? i : i - kInstTile;
      const int r = ii * kRowsPerInst + lane / kCh;
      const int c = (lane % kCh) ^ dual_swz<D>(r);
      voff[k] = r * (i < kInstTile ? qrowb : dorowb) + c * 16;
    }
  }
  auto issue = [&](int t, int slot) __attribute__((always_inline)) {
    const int qb = __builtin_amdgcn_readfirstlane(list[t >> 1]);
    const int row0 = qb * kBlk + (t & 1) * kT;
    uint8_t* buf = smem + slot * kBufBytes;
#pragma unroll
    for (int k = 0; k < kHi; ++k) {
      const int i = wave + kW * k;
      if (i >= kInst) break;
      if (i < kInstTile) dma16(q_srd, buf + i * 1024, voff[k], row0 * qrowb);
      else if (i < 2 * kInstTile) dma16(do_srd, buf + i * 1024, voff[k], row0 * dorowb);
      else dma16(st_srd, buf + i * 1024, voff[k], (row0 / 64) * 1024);
    }
  };

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[i][r] = dv[i][r] = 0.f;

  const int trr = tr_row(lane), trc = tr_col(lane);
  constexpr int fL = (kPooled && !kML) ? 2 : 0;  // stats fields of this branch
  constexpr bool kSeed = D == 64 || VB_BWD_SEED128;

  if (ntiles > 0) issue(0, 0);
  if (kBufs == 3 && ntiles > 1) issue(1, 1);
  // The loop body is instantiated once per ring slot: every LDS address is a compile-time offset.
  auto body = [&](int t, auto U) __attribute__((always_inline)) {
    constexpr int u_slot = decltype(U)::value;
    // retire this wave's DMAs of tile t (tile t+1 stays in flight); the barrier makes every wave's
    // part visible and proves slot (t-1) % kBufs is no longer being read
    if (kBufs == 3 && t + 1 < ntiles) {
      if (many) VB_WAIT_VMCNT(kHi);
      else VB_WAIT_VMCNT(kLo);
    } else {
      VB_WAIT_VMCNT(0);
    }
    __builtin_amdgcn_s_barrier();
    if constexpr (kBufs == 3) {
      if (t + 2 < ntiles) issue(t + 2, (u_slot + 2) % kBufs);
    } else {
      if (t + 1 < ntiles) issue(t + 1, (u_slot + 1) % kBufs);   // into slot (t-1) % 2, free after the barrier
    }
    const uint8_t* qt = smem + u_slot * kBufBytes;
    const uint8_t* dot = qt + kTileBytes;
    const float* st = reinterpret_cast<const float*>(qt + 2 * kTileBytes);
    // multi-level pooled items: keys of blocks without level 2^e for this q-block take no part
    bool act = true;
    if (kML && kPooled) {
      act = (list_bits[t >> 1] >> my_blk_bit) & 1;
      // The item's q-block list is the union over its 2^e key blocks; a wave whose own key
      // blocks are not at level 2^e for this q-block has nothing to add (P = 0 for all its keys)
      // and skips the tile's MFMAs, leaving its SIMD to the co-resident waves. A wave holds one
      // block's keys at levels 2 and 4, two blocks' at level 8. Its tile would add exact zeros,
      // so the sums are unchanged.
      if (!__any(act)) return;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      // dP's accumulator starts at -Delta of its row (register r = row 4j+e of this u half; the
      // stats hold -Delta, read straight into the accumulator), so dS = P * (dO.V^T - Delta) needs
      // no subtraction per score
      f32x16 s, dp;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 Dv = *reinterpret_cast<const f32x4*>(st + (fL + 1) * 64 + 32 * u + 8 * j + 4 * half);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[4 * j + e] = 0.f;
          dp[4 * j + e] = kSeed ? Dv[e] : 0.f;
        }
      }
      if constexpr (kPrioKV & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        s = T::mfma32(lds_b128<T>(qt, dual_off<D>(32 * u + l32, 2 * ks + half)), kf[ks], s);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        dp = T::mfma32(lds_b128<T>(dot, dual_off<D>(32 * u + l32, 2 * ks + half)), vf[ks], dp);
      if constexpr (kPrioKV & 1) __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 Lv = *reinterpret_cast<const f32x4*>(st + fL * 64 + 32 * u + 8 * j + 4 * half);
        f32x4 Dv2 = {0.f, 0.f, 0.f, 0.f};
        if (!kSeed) Dv2 = *reinterpret_cast<const f32x4*>(st + (fL + 1) * 64 + 32 * u + 8 * j + 4 * half);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * j + e;
          float pr;
          if (kML) pr = act ? exp2_fast(fmaf(s[r], p.c, lvl_bias - Lv[e])) : 0.f;
          else pr = exp2_fast(fmaf(s[r], p.c, -Lv[e]));
          s[r] = pr;
          dp[r] = pr * (kSeed ? dp[r] : dp[r] + Dv2[e]);
        }
      }
      // dV^T += dO^T.P and dK^T += Q^T.dS over (16-row half sb, 32-wide d tile dt) steps; the four
      // transposed reads of step j+1 are issued before step j's MFMAs and waited for with
      // lgkmcnt(4), so each wait only covers reads issued one step earlier
      typename T::vec8 pp[2], pd[2];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        pp[sb] = pack8<T>(s, 8 * sb);
        pd[sb] = pack8<T>(dp, 8 * sb);
      }
      constexpr int NST = 2 * DT;
      s16x4 rdo[2][2], rq[2][2];   // [ring][lo/hi]
      auto rd = [&](int j, int slot) __attribute__((always_inline)) {
        const int rr = 32 * u + 16 * (j / DT) + trr;
        const int cc = 32 * (j % DT) + trc;
        rdo[slot][0] = lds_tr4_asm_at(dot, dual_off_col<D>(rr, cc));
        rdo[slot][1] = lds_tr4_asm_at(dot, dual_off_col<D>(rr + 8, cc));
        rq[slot][0] = lds_tr4_asm_at(qt, dual_off_col<D>(rr, cc));
        rq[slot][1] = lds_tr4_asm_at(qt, dual_off_col<D>(rr + 8, cc));
      };
      rd(0, 0);
      if constexpr (kPrioKV & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < NST; ++j) {
        const int sl = j & 1;
        if (j + 1 < NST) {
          rd(j + 1, sl ^ 1);
          asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(rdo[sl][0]), "+v"(rdo[sl][1]), "+v"(rq[sl][0]), "+v"(rq[sl][1]));
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rdo[sl][0]), "+v"(rdo[sl][1]), "+v"(rq[sl][0]), "+v"(rq[sl][1]));
        }
        const int sb = j / DT, dt = j % DT;
        dv[dt] = T::mfma32(join8<T>(rdo[sl][0], rdo[sl][1]), pp[sb], dv[dt]);
        dk[dt] = T::mfma32(join8<T>(rq[sl][0], rq[sl][1]), pd[sb], dk[dt]);
      }
      if constexpr (kPrioKV & 2) __builtin_amdgcn_s_setprio(0);
    }
  };
  for (int t0 = 0; t0 < ntiles; t0 += kBufs) {
    body(t0, std::integral_constant<int, 0>{});
    if (t0 + 1 < ntiles) body(t0 + 1, std::integral_constant<int, 1>{});
    if constexpr (kBufs == 3) {
      if (t0 + 2 < ntiles) body(t0 + 2, std::integral_constant<int, 2>{});
    }
  }

  // ---- epilogue: lane = key, registers = d ---------------------------------------------------------
  if (!kvalid) return;
  const float nanf_ = __builtin_nanf("");
  if (kML && kPooled) {   // pooled pyramid rows: fp32 grads, summed into dk/dv by the level-1 pass
    const int64_t po = (int64_t)bh * (7 * (p.Lpad / 8)) + (ml_row0 - p.Lpad) + key;
    float* dkr = p.dkpyr + po * D;
    float* dvr = p.dvpyr + po * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * half;
        f32x4 a, c;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = dk[dt][4 * g4 + e] * p.scale;
          c[e] = dv[dt][4 * g4 + e];
        }
        *reinterpret_cast<f32x4*>(dkr + d) = a;
        *reinterpret_cast<f32x4*>(dvr + d) = c;
      }
    return;
  }
  if (kML) {   // level-1 key (< L): + the mean-pool adjoints of its level-2/4/8 rows (KML:1494-1563)
    const int64_t rb = (int64_t)bh * (7 * (p.Lpad / 8));
    const float* pk[3];
    const float* pv[3];
#pragma unroll
    for (int e = 1; e < 4; ++e) {
      const int64_t row = rb + (MlGeom(p.Lpad).off[e] - p.Lpad) + (key >> e);
      pk[e - 1] = p.dkpyr + row * D;
      pv[e - 1] = p.dvpyr + row * D;
    }
    const int64_t orow = p.kv_rows ? p.kv_rows[key] : krow0 + key;
    uint8_t* dkr = reinterpret_cast<uint8_t*>(p.dk) + 2 * (b * p.dks[0] + h * p.dks[1] + orow * p.dks[2]);
    uint8_t* dvr = reinterpret_cast<uint8_t*>(p.dv) + 2 * (b * p.dvs[0] + h * p.dvs[1] + orow * p.dvs[2]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * half;
        float a[4], c[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = dk[dt][4 * g4 + e] * p.scale;
          c[e] = dv[dt][4 * g4 + e];
        }
#pragma unroll
        for (int lv = 0; lv < 3; ++lv) {
          const float w = 1.0f / (float)(2 << lv);
          const f32x4 x = *reinterpret_cast<const f32x4*>(pk[lv] + d);
          const f32x4 y = *reinterpret_cast<const f32x4*>(pv[lv] + d);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] = fmaf(x[e], w, a[e]);
            c[e] = fmaf(y[e], w, c[e]);
          }
        }
        u32x2 w2, z;
        w2[0] = pack2<T>(a[0], a[1]); w2[1] = pack2<T>(a[2], a[3]);
        z[0] = pack2<T>(c[0], c[1]); z[1] = pack2<T>(c[2], c[3]);
        *reinterpret_cast<u32x2*>(dkr + d * 2) = w2;
        *reinterpret_cast<u32x2*>(dvr + d * 2) = z;
      }
    return;
  }
  if (kPooled) {
    const int64_t po = ((int64_t)split * BH + bh) * p.Lkp + key;
    float* dkr = p.dkp_part + po * D;
    float* dvr = p.dvp_part + po * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * half;
        f32x4 a, c;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = dk[dt][4 * g4 + e] * p.scale;
          c[e] = dv[dt][4 * g4 + e];
        }
        *reinterpret_cast<f32x4*>(dkr + d) = a;
        *reinterpret_cast<f32x4*>(dvr + d) = c;
      }
    return;
  }
  // full-resolution key: + mean-pool adjoint of the pooled grads (replicate padding folds onto
  // the last token), written at the caller's row
  const float* pk = nullptr;
  const float* pv = nullptr;
  float pw = 0.f;
  if (p.dkp) {
    const int gp = key / p.gap;
    pk = p.dkp + ((int64_t)bh * p.Lkp + gp) * D;
    pv = p.dvp + ((int64_t)bh * p.Lkp + gp) * D;
    const int extra = (key == Lk - 1) ? p.Lkp * p.gap - Lk : 0;
    pw = (float)(1 + extra) / (float)p.gap;
  }
  const int64_t orow = p.kv_rows ? p.kv_rows[key] : krow0 + key;
  uint8_t* dkr = reinterpret_cast<uint8_t*>(p.dk) + 2 * (b * p.dks[0] + h * p.dks[1] + orow * p.dks[2]);
  uint8_t* dvr = reinterpret_cast<uint8_t*>(p.dv) + 2 * (b * p.dvs[0] + h * p.dvs[1] + orow * p.dvs[2]);
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = dt * 32 + 8 * g4 + 4 * half;
      float a[4], c[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = dk[dt][4 * g4 + e] * p.scale;
        c[e] = dv[dt][4 * g4 + e];
      }
      if (pk) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(pk + d);
        const f32x4 y = *reinterpret_cast<const f32x4*>(pv + d);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = fmaf(x[e], pw, a[e]);
          c[e] = fmaf(y[e], pw, c[e]);
        }
      }
      if (nan_head) {
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = c[e] = nanf_;
      }
      u32x2 w, z;
      w[0] = pack2<T>(a[0], a[1]); w[1] = pack2<T>(a[2], a[3]);
      z[0] = pack2<T>(c[0], c[1]); z[1] = pack2<T>(c[2], c[3]);
      *reinterpret_cast<u32x2*>(dkr + d * 2) = w;
      *reinterpret_cast<u32x2*>(dvr + d * 2) = z;
    }
}

// ------------------------------------------------------------------------------------------------
// dQ: one workgroup per (b, h, 128-row q-block); kept full-resolution tiles then pooled tiles
// ------------------------------------------------------------------------------------------------
#ifndef VB_DQ_WAVES_D128
#define VB_DQ_WAVES_D128 2   // D=128: two waves per SIMD with a 2-slot ring (1: one wave, 3-slot ring; Wan backward 1.014-1.018x)
#endif
#ifndef VB_DQ_PRIO64
#define VB_DQ_PRIO64 0     // measured (cog backward): 1 0.990x, 3 0.990x
#endif
#ifndef VB_DQ_PRIO128
#define VB_DQ_PRIO128 1   // measured (Wan backward, two waves per SIMD): 1 1.096x, 3 1.094x
#endif
#ifndef VB_DQ_WAVES_D64
#define VB_DQ_WAVES_D64 2   // waves per SIMD the D=64 dQ kernel is register-budgeted for
#endif
template <int D, class T, bool kPool, bool kML = false>
__global__ void __launch_bounds__(bwd::kThreads, D == 128 ? VB_DQ_WAVES_D128 : VB_DQ_WAVES_D64) bwd_dq_kernel(const BwdParams p) {
  using namespace bwd;
  constexpr int KS = D / 16;
  constexpr int DT = D / 32;
  constexpr int RB = D * 2;
  constexpr int kTileBytes = kT * RB;       // one 64-key K (or V) tile
  constexpr int kInstTile = kTileBytes / 1024;
  constexpr int kRowsPerInst = 1024 / RB;
  constexpr int kCh = RB / 16;
  constexpr int kInst = 2 * kInstTile;
  constexpr int kBufBytes = 2 * kTileBytes;
  // 2-slot K/V ring with a second barrier per tile: D=64, and D=128 at the default two waves per
  // SIMD (VB_DQ_WAVES_D128=2, 68 KiB). Only the one-wave D=128 build (VB_DQ_WAVES_D128=1) takes a
  // 3-slot ring, where tile t is read while t+1 and t+2 are in flight and one barrier per tile both
  // publishes tile t and proves slot (t-1) % 3 free for tile t+2.
  constexpr int kRing = (D == 128 && VB_DQ_WAVES_D128 < 2) ? 3 : 2;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kRing * kBufBytes + kMaxBlocks * 2 + 16];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + kRing * kBufBytes);
  int* list_n = reinterpret_cast<int*>(smem + kRing * kBufBytes + kMaxBlocks * 2);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;

  // heavy-first, then XCD-contiguous head-major (as the forward)
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
  int Lq = p.Lq, Lk = p.Lk;
  int64_t qrow0 = 0, krow0 = 0;
  if (p.cu_q) {
    qrow0 = p.cu_q[b]; Lq = p.cu_q[b + 1] - p.cu_q[b];
    krow0 = p.cu_k[b]; Lk = p.cu_k[b + 1] - p.cu_k[b];
  }
  const int q0 = qblk * kBlk;
  if (q0 >= Lq) return;
  const int nbk = (Lk + kBlk - 1) / kBlk;

  bool nan_head = false;
  const uint8_t* mrow = nullptr;
  const bool use_main = p.k != nullptr;
  if (use_main) {
    const uint8_t* mh = head_mask_base(p.mask, p.ms, p.head_mask_type, p.H, b, h, nan_head, p.hm_mode);
    if (mh) mrow = mh + (int64_t)qblk * p.ms[2];
  }
  if (kML) {
    // per-level key-block lists (levels 1, 2, 4, 8 in that order; as the forward)
    if (threadIdx.x < 64) {
      int cnt[4] = {0, 0, 0, 0};
      for (int j0 = 0; j0 < nbk; j0 += 64) {
        const int j = j0 + lane;
        const int lv = j < nbk ? mrow[j] : 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) cnt[e] += __popcll(__ballot(lv == (1 << e)));
      }
      int pos[4] = {0, cnt[0], cnt[0] + cnt[1], cnt[0] + cnt[1] + cnt[2]};
      for (int j0 = 0; j0 < nbk; j0 += 64) {
        const int j = j0 + lane;
        const int lv = j < nbk ? mrow[j] : 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const unsigned long long bal = __ballot(lv == (1 << e));
          if (lv == (1 << e))
            list[pos[e] + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] = (uint16_t)j;
          pos[e] += __popcll(bal);
        }
      }
      if (lane < 4) list_n[lane] = lane == 0 ? cnt[0] : lane == 1 ? cnt[1] : lane == 2 ? cnt[2] : cnt[3];
    }
  } else if (threadIdx.x < 64) {
    int n = 0;
    if (use_main) {
      for (int j0 = 0; j0 < nbk; j0 += 64) {
        const int j = j0 + lane;
        const bool keep = (j < nbk) && (mrow == nullptr || mrow[j] != 0);
        const unsigned long long bal = __ballot(keep);
        if (keep) {
          const int pos = n + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
          list[pos] = (uint16_t)j;
        }
        n += __popcll(bal);
      }
    }
    if (lane == 0) *list_n = n;
  }

  // this wave's 32 query rows: Q and dO as B operands (lane = query)
  const int g = q0 + wave * 32 + l32;
  const bool qvalid = g < Lq;
  const int gc = qvalid ? g : Lq - 1;
  typename T::vec8 qf[KS], df[KS];
  {
    const uint8_t* qp = reinterpret_cast<const uint8_t*>(p.q) +
                        2 * (b * p.qs[0] + h * p.qs[1] + (qrow0 + gc) * p.qs[2]);
    const uint8_t* dp_ = reinterpret_cast<const uint8_t*>(p.dout) +
                         2 * (b * p.dos[0] + h * p.dos[1] + (qrow0 + gc) * p.dos[2]);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qf[s] = *reinterpret_cast<const typename T::vec8*>(qp + (16 * s + 8 * half) * 2);
      df[s] = *reinterpret_cast<const typename T::vec8*>(dp_ + (16 * s + 8 * half) * 2);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      asm volatile("" : "+v"(qf[s]));
      asm volatile("" : "+v"(df[s]));
    }
  }
  // the clamped row's statistics, as the Q/dO loads (padding rows are never stored)
  const float* st = p.stats + ((int64_t)bh * p.ntile + gc / 64) * 256 + (gc & 63);
  float L1 = st[0], D1 = st[64], L2 = st[128], D2 = st[192];   // D1, D2 = -Delta
  asm volatile("" : "+v"(L1), "+v"(D1), "+v"(L2), "+v"(D2));

  __syncthreads();
  const int nkept = __builtin_amdgcn_readfirstlane(*list_n);
  int ntm = 2 * nkept;
  if (nkept > 0 && list[nkept - 1] == nbk - 1 && (nbk - 1) * kBlk + kT >= Lk && !(kML && p.ref_tail)) ntm -= 1;
  const int ntp = kPool ? (p.Lkp + kT - 1) / kT : 0;
  // multi-level tiles (as the forward): level 1 (2 per block), one per level-2 block, two level-4
  // blocks and four level-8 blocks per tile
  int n2 = 0, n4 = 0, n8 = 0, T12 = 0, T124 = 0;
  if (kML) {
    n2 = __builtin_amdgcn_readfirstlane(list_n[1]);
    n4 = __builtin_amdgcn_readfirstlane(list_n[2]);
    n8 = __builtin_amdgcn_readfirstlane(list_n[3]);
    T12 = ntm + n2;
    T124 = T12 + (n4 + 1) / 2;
  }
  const int ntiles = kML ? T124 + (n8 + 3) / 4 : ntm + ntp;
  // multi-level tile t: pyramid row of 16-row quarter qd, valid keys, level exponent
  const int off4 = p.Lpad + p.Lpad / 2, off8 = off4 + p.Lpad / 4;
  auto ml_quarter = [&](int t, int qd) __attribute__((always_inline)) -> int {
    if (t < ntm) return (int)list[t >> 1] * kBlk + (t & 1) * kT + 16 * qd;
    if (t < T12) return p.Lpad + (int)list[nkept + t - ntm] * 64 + 16 * qd;
    if (t < T124) {
      const int e = min(2 * (t - T12) + (qd >> 1), n4 - 1);
      return off4 + (int)list[nkept + n2 + e] * 32 + 16 * (qd & 1);
    }
    const int e = min(4 * (t - T124) + qd, n8 - 1);
    return off8 + (int)list[nkept + n2 + n4 + e] * 16;
  };
  auto ml_klen = [&](int t) __attribute__((always_inline)) -> int {
    if (t < ntm) return p.ref_tail ? kT : min(kT, Lk - ((int)list[t >> 1] * kBlk + (t & 1) * kT));
    if (t < T12) return kT;
    if (t < T124) return min(kT, (n4 - 2 * (t - T12)) * 32);
    return min(kT, (n8 - 4 * (t - T124)) * 16);
  };
  auto ml_lvl = [&](int t) __attribute__((always_inline)) -> int {
    return t < ntm ? 0 : t < T12 ? 1 : t < T124 ? 2 : 3;
  };

  const uint8_t* kbase = use_main ? reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1] + krow0 * p.ks[2]) : nullptr;
  const uint8_t* vbase = use_main ? reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1] + krow0 * p.vs[2]) : nullptr;
  const uint8_t* kpbase = kPool ? reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1]) : nullptr;
  const uint8_t* vpbase = kPool ? reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1]) : nullptr;

  auto tile_keys = [&](int t, int& kstart, int& klen) __attribute__((always_inline)) {
    if (t < ntm) {
      const int blk = __builtin_amdgcn_readfirstlane(list[t >> 1]);
      kstart = blk * kBlk + (t & 1) * kT;
      klen = min(kT, Lk - kstart);
    } else {
      kstart = (t - ntm) * kT;
      klen = min(kT, p.Lkp - kstart);
    }
  };
  // Tile t -> ring slot by LDS-DMA through buffer descriptors (as the dK/dV kernel): this wave
  // issues instructions i = wave + 4k (K tile first, then V). A lane's part of each instruction
  // (row within the tile, swizzled chunk) is a fixed 32-bit voffset per key source; the tile's first
  // key is the scalar soffset, so no per-lane 64-bit address math runs per tile. The host checks
  // that every (b,h) slice spans < 2 GiB.
  static_assert(kInst % 4 == 0, "every wave issues the same number of DMA instructions");
  constexpr int kPer = kInst / 4;
  const int krowb = 2 * (int)p.ks[2], vrowb = 2 * (int)p.vs[2];
  const int kprowb = kPool ? 2 * (int)p.kps[2] : 0, vprowb = kPool ? 2 * (int)p.vps[2] : 0;
  const int src_rows = kML ? 15 * (p.Lpad / 8) : Lk;
  const srd_t k_srd = make_srd(use_main ? kbase : nullptr, use_main ? (int)((int64_t)(src_rows - 1) * krowb + RB) : 0);
  const srd_t v_srd = make_srd(use_main ? vbase : nullptr, use_main ? (int)((int64_t)(src_rows - 1) * vrowb + RB) : 0);
  const srd_t kp_srd = make_srd(kPool ? kpbase : nullptr, kPool ? (int)((int64_t)(p.Lkp - 1) * kprowb + RB) : 0);
  const srd_t vp_srd = make_srd(kPool ? vpbase : nullptr, kPool ? (int)((int64_t)(p.Lkp - 1) * vprowb + RB) : 0);
  int dr[kPer], dc16[kPer], voff_m[kPer], voff_p[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int i = wave + 4 * k;
    const bool isv = k >= kPer / 2;   // i >= kInstTile exactly when k >= kPer / 2
    const int ii = isv ? i - kInstTile : i;
    dr[k] = ii * kRowsPerInst + lane / kCh;
    dc16[k] = 16 * ((lane % kCh) ^ dual_swz<D>(dr[k]));
    const int rr = kML ? (dr[k] & 15) : dr[k];   // multi-level: row within the 16-row quarter
    voff_m[k] = rr * (isv ? vrowb : krowb) + dc16[k];
    voff_p[k] = dr[k] * (isv ? vprowb : kprowb) + dc16[k];
  }
  auto issue = [&](int t, auto SLOT) __attribute__((always_inline)) {
    constexpr int slot = decltype(SLOT)::value;
    uint8_t* buf = smem + slot * kBufBytes;
    if constexpr (kML) {
      int qsrc[4];
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) qsrc[qd] = __builtin_amdgcn_readfirstlane(ml_quarter(t, qd));
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const bool isv = k >= kPer / 2;
        const int i = wave + 4 * k;
        const int ii = isv ? i - kInstTile : i;
        const int qd = (ii * kRowsPerInst) >> 4;   // wave-uniform: kRowsPerInst divides 16
        const int q = qd == 0 ? qsrc[0] : qd == 1 ? qsrc[1] : qd == 2 ? qsrc[2] : qsrc[3];
        dma16(isv ? v_srd : k_srd, buf + i * 1024, voff_m[k],
              __builtin_amdgcn_readfirstlane(q * (isv ? vrowb : krowb)));
      }
      return;
    }
    int kstart, klen;
    tile_keys(t, kstart, klen);
    const bool pooled = kPool && t >= ntm;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const bool isv = k >= kPer / 2;
      const int i = wave + 4 * k;
      const int rowb = pooled ? (isv ? vprowb : kprowb) : (isv ? vrowb : krowb);
      const srd_t sd = pooled ? (isv ? vp_srd : kp_srd) : (isv ? v_srd : k_srd);
      int voff = pooled ? voff_p[k] : voff_m[k];
      if (klen < kT) voff = min(dr[k], klen - 1) * rowb + dc16[k];   // tail: replicate the last key
      dma16(sd, buf + i * 1024, voff, __builtin_amdgcn_readfirstlane(kstart * rowb));
    }
  };

  f32x16 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[i][r] = 0.f;
  const int trr = tr_row(lane), trc = tr_col(lane);
  constexpr int kHi = (kInst + 3) / 4, kLo = kInst / 4;  // DMA instructions per wave and tile
  const bool many = wave < (kInst & 3);

  constexpr bool kSeedQ = D == 64 || VB_BWD_SEED128;
  // s_setprio 1 around the MFMA chains (bit 0: S and dP, bit 1: the dQ steps) at D=128
  constexpr int kPrioQ = D == 128 ? VB_DQ_PRIO128 : VB_DQ_PRIO64;
  f32x16 cD, zero;
#pragma unroll
  for (int r = 0; r < 16; ++r) cD[r] = zero[r] = 0.f;
  int cur_cls = -1;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  if (ntiles > 0) issue(0, I0{});
  if (kRing == 3 && ntiles > 1) issue(1, I1{});
  // The body is instantiated once per ring slot, so every LDS address is an immediate offset.
  auto body = [&](int t, auto U) __attribute__((always_inline)) {
    constexpr int u_slot = decltype(U)::value;
    if (kRing == 2 && t + 1 < ntiles) issue(t + 1, std::integral_constant<int, (u_slot + 1) % kRing>{});
    // retire this wave's part of tile t (tile t+1's stays in flight), then the barrier
    if (t + 1 < ntiles) {
      if (many) VB_WAIT_VMCNT(kHi);
      else VB_WAIT_VMCNT(kLo);
    } else {
      VB_WAIT_VMCNT(0);
    }
    __builtin_amdgcn_s_barrier();
    if (kRing == 3 && t + 2 < ntiles) issue(t + 2, std::integral_constant<int, (u_slot + 2) % kRing>{});
    int kstart, klen;
    float nL;
    bool pooled;
    int cls;   // tile class (wave-uniform): main/pooled, or the multi-level level
    if (kML) {
      klen = ml_klen(t);
      pooled = false;
      cls = ml_lvl(t);
      nL = (float)cls - L1;   // + log2(level): the +ln p logit bias in the exp2 domain
    } else {
      tile_keys(t, kstart, klen);
      pooled = kPool && t >= ntm;
      cls = pooled;
      nL = -(pooled ? L2 : L1);
    }
    const float Dr = pooled ? D2 : D1;
    if (kSeedQ && cls != cur_cls) {   // only where the key source changes: refresh the persistent seeds
      asm volatile("");
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        cD[r] = kSeedQ ? Dr : 0.f;
      }
      cur_cls = cls;
    }
    const uint8_t* kt_ = smem + u_slot * kBufBytes;
    const uint8_t* vt_ = kt_ + kTileBytes;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {   // 32-key halves: S^T, dP^T -> dS^T -> dQ^T
      // dP^T's chain starts from cD = -Delta of the lane's row (dS = P * (dO.V^T - Delta) with no
      // subtraction per score); the seeds are persistent registers read as the MFMA's C operand
      f32x16 s, dp;
      if constexpr (kPrioQ & 1) __builtin_amdgcn_s_setprio(1);
      s = T::mfma32(lds_b128<T>(kt_, dual_off<D>(kt * 32 + l32, half)), qf[0], zero);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks)
        s = T::mfma32(lds_b128<T>(kt_, dual_off<D>(kt * 32 + l32, 2 * ks + half)), qf[ks], s);
      dp = T::mfma32(lds_b128<T>(vt_, dual_off<D>(kt * 32 + l32, half)), df[0], kSeedQ ? cD : zero);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks)
        dp = T::mfma32(lds_b128<T>(vt_, dual_off<D>(kt * 32 + l32, 2 * ks + half)), df[ks], dp);
      if constexpr (kPrioQ & 1) __builtin_amdgcn_s_setprio(0);
      if (klen < kT) {
        asm volatile("");
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool ok = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half < klen;
          const float pr = ok ? exp2_fast(fmaf(s[r], p.c, nL)) : 0.f;
          dp[r] = pr * (kSeedQ ? dp[r] : dp[r] + Dr);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pr = exp2_fast(fmaf(s[r], p.c, nL));
          dp[r] = pr * (kSeedQ ? dp[r] : dp[r] + Dr);
        }
      }
      // dQ^T += K^T.dS^T over (16-key half sb, d tile dt) steps, reads one step ahead (lgkmcnt(2))
      typename T::vec8 pdv[2];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) pdv[sb] = pack8<T>(dp, 8 * sb);
      constexpr int NST = 2 * DT;
      s16x4 rk[2][2];
      auto rd = [&](int j, int slot) __attribute__((always_inline)) {
        const int rr = kt * 32 + 16 * (j / DT) + trr;
        const int cc = 32 * (j % DT) + trc;
        rk[slot][0] = lds_tr4_asm_at(kt_, dual_off_col<D>(rr, cc));
        rk[slot][1] = lds_tr4_asm_at(kt_, dual_off_col<D>(rr + 8, cc));
      };
      rd(0, 0);
      if constexpr (kPrioQ & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < NST; ++j) {
        const int sl = j & 1;
        if (j + 1 < NST) {
          rd(j + 1, sl ^ 1);
          asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(rk[sl][0]), "+v"(rk[sl][1]));
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rk[sl][0]), "+v"(rk[sl][1]));
        }
        dq[j % DT] = T::mfma32(join8<T>(rk[sl][0], rk[sl][1]), pdv[j / DT], dq[j % DT]);
      }
      if constexpr (kPrioQ & 2) __builtin_amdgcn_s_setprio(0);
    }
    if (kRing == 2) __builtin_amdgcn_s_barrier();   // slot t % 2 is refilled by the next issue
  };
  for (int t0 = 0; t0 < ntiles; t0 += kRing) {
    body(t0, I0{});
    if (t0 + 1 < ntiles) body(t0 + 1, I1{});
    if constexpr (kRing > 2)
      if (t0 + 2 < ntiles) body(t0 + 2, std::integral_constant<int, 2>{});
  }

  if (!qvalid) return;
  const float mul = nan_head ? __builtin_nanf("") : p.scale;
  const int64_t orow = p.q_rows ? p.q_rows[g] : qrow0 + g;
  uint8_t* ob = reinterpret_cast<uint8_t*>(p.dq) + 2 * (b * p.dqs[0] + h * p.dqs[1] + orow * p.dqs[2]);
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = dt * 32 + 8 * g4 + 4 * half;
      u32x2 w;
      w[0] = pack2<T>(dq[dt][4 * g4 + 0] * mul, dq[dt][4 * g4 + 1] * mul);
      w[1] = pack2<T>(dq[dt][4 * g4 + 2] * mul, dq[dt][4 * g4 + 3] * mul);
      *reinterpret_cast<u32x2*>(ob + d * 2) = w;
    }
}

// sum of the pooled-key gradient partials: dkp = sum_s part[s] (fixed order: deterministic)
__global__ void __launch_bounds__(256) pool_grad_reduce_kernel(const float* pk, const float* pv, int64_t n4, int nsplit,
                                                               float* dk, float* dv) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  f32x4 a = reinterpret_cast<const f32x4*>(pk)[i];
  f32x4 c = reinterpret_cast<const f32x4*>(pv)[i];
  for (int s = 1; s < nsplit; ++s) {
    a += reinterpret_cast<const f32x4*>(pk)[s * n4 + i];
    c += reinterpret_cast<const f32x4*>(pv)[s * n4 + i];
  }
  reinterpret_cast<f32x4*>(dk)[i] = a;
  reinterpret_cast<f32x4*>(dv)[i] = c;
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
#ifndef VB_BWD_FORK
#define VB_BWD_FORK 1   // D=128: dQ on a side stream beside the dK/dV chain (they share only the prep's output)
#endif
// dQ depends only on the prep kernel's row statistics; the dK/dV chain (pooled keys, their reduce,
// main keys) never reads dQ. So dQ is launched on a per-device side stream that waits for the
// caller's stream at the fork and is joined back (an event) before the call returns: the two
// launches fill each other's last rounds and the chain's small launches. Work and results are
// unchanged (no atomics, disjoint outputs). Graph capture: the side stream joins the caller's
// capture through the event wait. The mutex keeps one call's record/wait pairs together.
// Measured (tools/ab.py, profiles/r06_bwd_fork_ab.log): Wan backward 1.016-1.019x, CogVideoX
// 0.998-1.000x, the multi-level backward 0.987-0.990x, so only the D=128 main backward forks.
struct BwdFork {
  hipStream_t side = nullptr;
  hipEvent_t forked = nullptr, joined = nullptr;
};
class ForkScope {
 public:
  ForkScope(hipStream_t s, bool enable) : s_(s), lock_(mu(), std::defer_lock) {
    if (!VB_BWD_FORK || !enable) return;
    lock_.lock();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    BwdFork& f = forks()[dev];
    if (!f.side) {
      if (hipStreamCreateWithFlags(&f.side, hipStreamNonBlocking) != hipSuccess ||
          hipEventCreateWithFlags(&f.forked, hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&f.joined, hipEventDisableTiming) != hipSuccess) {
        f = BwdFork{};
        return;   // no side stream: everything stays on the caller's stream
      }
    }
    if (hipEventRecord(f.forked, s) != hipSuccess || hipStreamWaitEvent(f.side, f.forked, 0) != hipSuccess) return;
    f_ = &f;
  }
  ~ForkScope() {
    if (f_ && hipEventRecord(f_->joined, f_->side) == hipSuccess) (void)hipStreamWaitEvent(s_, f_->joined, 0);
  }
  hipStream_t dq_stream() const { return f_ ? f_->side : s_; }
  bool forked() const { return f_ != nullptr; }

 private:
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static std::map<int, BwdFork>& forks() {
    static std::map<int, BwdFork> m;
    return m;
  }
  hipStream_t s_;
  std::unique_lock<std::mutex> lock_;   // held from the fork to the join (the destructor's event wait)
  BwdFork* f_ = nullptr;
};

template <class T>
static int launch_prep(const PrepParams& pp, hipStream_t s) {
  const int64_t threads = (int64_t)pp.B * pp.H * pp.ntile * 64 * (pp.D / 8);
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipLaunchKernelGGL(bwd_prep_kernel<T>, grid, dim3(256), 0, s, pp);
  return check_launch("bwd_prep_kernel");
}

// kernel choice: vb_attn_bwd_args.kernel_select (VB_BWD_SEL_* bits); `ran` collects VB_BWD_RAN_* bits
template <int D, class T>
static int launch_dq(const BwdParams& p, bool pool, hipStream_t s, int sel, int& ran) {
  constexpr bool kF16 = std::is_same<T, F16>::value;
  if (!(sel & VB_BWD_SEL_DQ_ROUND3)) return launch_dq_pipe(p, D, pool, kF16, s, sel, ran);
  ran |= VB_BWD_RAN_DQ_ROUND3;
  const int BH = p.B * p.H;
  if (pool)
    hipLaunchKernelGGL((bwd_dq_kernel<D, T, true>), dim3(p.nbq * BH), dim3(bwd::kThreads), 0, s, p);
  else
    hipLaunchKernelGGL((bwd_dq_kernel<D, T, false>), dim3(p.nbq * BH), dim3(bwd::kThreads), 0, s, p);
  return check_launch("bwd_dq_kernel");
}

template <int D, class T>
static int launch_grads(const BwdParams& p, bool pool, hipStream_t s, int sel, int& ran) {
  const int BH = p.B * p.H;
  const bool pipe = !(sel & VB_BWD_SEL_DKDV_ROUND3);
  if ((pool && p.dkp) || p.k) ran |= pipe ? VB_BWD_RAN_DKDV_PIPE : VB_BWD_RAN_DKDV_ROUND3;
  constexpr bool kF16 = std::is_same<T, F16>::value;
  ForkScope fork(s, D == 128);
  if (fork.forked())   // dQ first, on the side stream
    if (int rc = launch_dq<D, T>(p, pool, fork.dq_stream(), sel, ran)) return rc;
  if (pool && p.dkp) {
    if (pipe) {
      if (int rc = launch_dkdv_pipe(p, D, true, kF16, s)) return rc;
    } else {
      hipLaunchKernelGGL((bwd_dkdv_kernel<D, T, true>), dim3(p.nbkp * BH * p.psplit), dim3(bwd::kThreads), 0, s, p);
      if (int rc = check_launch("bwd_dkdv_kernel<pooled>")) return rc;
    }
    if (p.psplit > 1) {
      const int64_t n4 = (int64_t)BH * p.Lkp * D / 4;
      hipLaunchKernelGGL(pool_grad_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, p.dkp_part,
                         p.dvp_part, n4, p.psplit, p.dkp, p.dvp);
      if (int rc = check_launch("pool_grad_reduce_kernel")) return rc;
    }
  }
  if (p.k) {
    if (pipe) {
      if (int rc = launch_dkdv_pipe(p, D, false, kF16, s)) return rc;
    } else {
      hipLaunchKernelGGL((bwd_dkdv_kernel<D, T, false>), dim3(p.nbk * BH), dim3(bwd::kThreads), 0, s, p);
      if (int rc = check_launch("bwd_dkdv_kernel")) return rc;
    }
  }
  return fork.forked() ? 0 : launch_dq<D, T>(p, pool, s, sel, ran);
}

static int dispatch_bwd(const PrepParams& pp, const BwdParams& p, int D, int dtype, bool pool, hipStream_t s,
                        int sel = 0, int32_t* ran_out = nullptr) {
  int ran = 0, rc;
  if (dtype == VB_DTYPE_BF16) {
    rc = launch_prep<BF16>(pp, s);
    if (!rc) rc = D == 64 ? launch_grads<64, BF16>(p, pool, s, sel, ran) : launch_grads<128, BF16>(p, pool, s, sel, ran);
  } else {
    rc = launch_prep<F16>(pp, s);
    if (!rc) rc = D == 64 ? launch_grads<64, F16>(p, pool, s, sel, ran) : launch_grads<128, F16>(p, pool, s, sel, ran);
  }
  if (ran_out) *ran_out = ran;
  return rc;
}

struct WsLayout {
  uint64_t stats, q_r, do_r, dkp, dvp, dkp_part, dvp_part, total;
  int psplit;
};
// pooled-key q-range split: aim at ~3k workgroups per sample for the pooled dK/dV pass. The split
// sets the order of the partial sums, so it does not depend on B: a sample's gradients are the
// same bits in any batch (the B=5 training-batch test).
static int pool_split(int B, int H, int Lq, int Lkp) {
  (void)B;
  if (Lkp <= 0) return 1;
  const int nbkp = (Lkp + 127) / 128, nbq = (Lq + 127) / 128;
  const int wg = nbkp * H;
  int s = (3072 + wg / 2) / wg;
  return s < 1 ? 1 : (s > nbq ? nbq : s);
}
static WsLayout ws_layout(int B, int H, int Lq, int D, bool copies, int Lkp) {
  auto up = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  WsLayout w{};
  const uint64_t ntile = (uint64_t)((Lq + 63) / 64);
  uint64_t off = 0;
  w.stats = off; off = up(off + (uint64_t)B * H * ntile * 256 * 4);
  w.q_r = w.do_r = 0;
  if (copies) {
    w.q_r = off; off = up(off + (uint64_t)B * H * Lq * D * 2);
    w.do_r = off; off = up(off + (uint64_t)B * H * Lq * D * 2);
  }
  w.dkp = w.dvp = w.dkp_part = w.dvp_part = 0;
  w.psplit = pool_split(B, H, Lq, Lkp);
  if (Lkp > 0) {
    w.dkp = off; off = up(off + (uint64_t)B * H * Lkp * D * 4);
    w.dvp = off; off = up(off + (uint64_t)B * H * Lkp * D * 4);
    w.dkp_part = w.dkp; w.dvp_part = w.dvp;
    if (w.psplit > 1) {
      w.dkp_part = off; off = up(off + (uint64_t)w.psplit * B * H * Lkp * D * 4);
      w.dvp_part = off; off = up(off + (uint64_t)w.psplit * B * H * Lkp * D * 4);
    }
  }
  w.total = off;
  return w;
}

static bool mul8(const int64_t* s) { return ((s[0] | s[1] | s[2]) & 7) == 0; }
// one (b,h) slice of L rows at `row_stride` elements must be addressable by a 32-bit buffer offset
static bool slice_ok(int L, int64_t row_stride, int D) {
  return (int64_t)(L - 1) * 2 * row_stride + 2 * D < (int64_t(1) << 31);
}
static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace vb

extern "C" uint64_t vb_attn_bwd_workspace_size(const vb_attn_bwd_args* a) {
  if (!a) return 0;
  return vb::ws_layout(a->B, a->H, a->Lq, a->D, a->q_rows != nullptr, a->kp ? a->Lkp : 0).total;
}

extern "C" int vb_attn_bwd(const vb_attn_bwd_args* a, void* stream) {
  using namespace vb;
  if (!a) return fail(VB_ERR_INVALID, "vb_attn_bwd: null args");
  if (a->B <= 0 || a->H <= 0 || a->Lq <= 0 || a->Lk <= 0 || a->D <= 0)
    return fail(VB_ERR_INVALID, "vb_attn_bwd: B, H, Lq, Lk, D must be positive");
  if (a->D != 64 && a->D != 128)
    return fail(VB_ERR_UNSUPPORTED, "vb_attn_bwd: head_dim must be 64 or 128, got " + std::to_string(a->D));
  if (a->dtype != VB_DTYPE_BF16 && a->dtype != VB_DTYPE_F16) return fail(VB_ERR_INVALID, "vb_attn_bwd: unknown dtype");
  if (!a->q || !a->k || !a->v || !a->out || !a->lse || !a->dout || !a->dq || !a->dk || !a->dv)
    return fail(VB_ERR_INVALID, "vb_attn_bwd: missing tensor");
  if (a->kernel_select & ~(VB_BWD_SEL_DKDV_ROUND3 | VB_BWD_SEL_DQ_ROUND3 | VB_BWD_SEL_DQ_RING4))
    return fail(VB_ERR_INVALID, "vb_attn_bwd: unknown kernel_select bits");
  const bool pool = a->kp != nullptr;
  if (pool && (!a->vp || a->Lkp <= 0 || !a->out2 || !a->lse2 || a->pool_gap <= 0))
    return fail(VB_ERR_INVALID, "vb_attn_bwd: pooled branch needs vp, Lkp, out2, lse2 and pool_gap");
  if (pool && (int64_t)a->Lkp * a->pool_gap < a->Lk)
    return fail(VB_ERR_INVALID, "vb_attn_bwd: Lkp * pool_gap must cover Lk");
  const int nbk = (a->Lk + 127) / 128;
  const int nbq = (a->Lq + 127) / 128;
  if (nbk > bwd::kMaxBlocks || nbq > bwd::kMaxBlocks) return fail(VB_ERR_UNSUPPORTED, "vb_attn_bwd: sequence too long");
  const int64_t* strides[] = {a->q_stride, a->k_stride, a->v_stride, a->out_stride, a->dout_stride,
                              a->dq_stride, a->dk_stride, a->dv_stride};
  for (const int64_t* s : strides)
    if (!mul8(s)) return fail(VB_ERR_INVALID, "vb_attn_bwd: strides must be multiples of 8 elements");
  if (pool && (!mul8(a->kp_stride) || !mul8(a->vp_stride) || !mul8(a->out2_stride)))
    return fail(VB_ERR_INVALID, "vb_attn_bwd: strides must be multiples of 8 elements");
  const void* ptrs[] = {a->q, a->k, a->v, a->out, a->dout, a->dq, a->dk, a->dv};
  for (const void* q : ptrs)
    if (!al16(q)) return fail(VB_ERR_INVALID, "vb_attn_bwd: tensors must be 16-byte aligned");
  if (pool && (!al16(a->kp) || !al16(a->vp) || !al16(a->out2)))
    return fail(VB_ERR_INVALID, "vb_attn_bwd: tensors must be 16-byte aligned");
  const WsLayout w = ws_layout(a->B, a->H, a->Lq, a->D, a->q_rows != nullptr, pool ? a->Lkp : 0);
  if (!a->workspace || a->workspace_bytes < w.total || !al16(a->workspace))
    return fail(VB_ERR_INVALID, "vb_attn_bwd: workspace missing or smaller than vb_attn_bwd_workspace_size()");
  if (!a->q_rows && (!slice_ok(a->Lq, a->q_stride[2], a->D) || !slice_ok(a->Lq, a->dout_stride[2], a->D)))
    return fail(VB_ERR_UNSUPPORTED, "vb_attn_bwd: a q/dout (b,h) slice spans >= 2 GiB");
  if (!slice_ok(a->Lk, a->k_stride[2], a->D) || !slice_ok(a->Lk, a->v_stride[2], a->D) ||
      (pool && (!slice_ok(a->Lkp, a->kp_stride[2], a->D) || !slice_ok(a->Lkp, a->vp_stride[2], a->D))))
    return fail(VB_ERR_UNSUPPORTED, "vb_attn_bwd: a k/v/kp/vp (b,h) slice spans >= 2 GiB");
  uint8_t* ws = reinterpret_cast<uint8_t*>(a->workspace);

  PrepParams pp{};
  pp.q = a->q; pp.dout = a->dout; pp.out = a->out; pp.out2 = pool ? a->out2 : nullptr;
  for (int i = 0; i < 3; ++i) {
    pp.qs[i] = a->q_stride[i]; pp.dos[i] = a->dout_stride[i]; pp.os[i] = a->out_stride[i];
    pp.o2s[i] = pool ? a->out2_stride[i] : 0;
  }
  pp.lse = a->lse; pp.lse2 = pool ? a->lse2 : nullptr; pp.alpha = a->alpha;
  pp.q_rows = a->q_rows;
  pp.stats = reinterpret_cast<float*>(ws + w.stats);
  if (a->q_rows) { pp.q_r = ws + w.q_r; pp.do_r = ws + w.do_r; }
  pp.B = a->B; pp.H = a->H; pp.Lq = a->Lq; pp.D = a->D; pp.ntile = (a->Lq + 63) / 64;

  BwdParams p{};
  if (a->q_rows) {
    p.q = ws + w.q_r; p.dout = ws + w.do_r;
    p.qs[0] = p.dos[0] = (int64_t)a->H * a->Lq * a->D;
    p.qs[1] = p.dos[1] = (int64_t)a->Lq * a->D;
    p.qs[2] = p.dos[2] = a->D;
  } else {
    p.q = a->q; p.dout = a->dout;
    for (int i = 0; i < 3; ++i) { p.qs[i] = a->q_stride[i]; p.dos[i] = a->dout_stride[i]; }
  }
  p.k = a->k; p.v = a->v;
  for (int i = 0; i < 3; ++i) {
    p.ks[i] = a->k_stride[i]; p.vs[i] = a->v_stride[i];
    p.ms[i] = a->mask_stride[i];
    p.dqs[i] = a->dq_stride[i]; p.dks[i] = a->dk_stride[i]; p.dvs[i] = a->dv_stride[i];
    if (pool) { p.kps[i] = a->kp_stride[i]; p.vps[i] = a->vp_stride[i]; }
  }
  p.kp = pool ? a->kp : nullptr; p.vp = pool ? a->vp : nullptr; p.Lkp = pool ? a->Lkp : 0;
  p.mask = a->block_mask;
  p.stats = pp.stats; p.ntile = pp.ntile;
  p.dq = a->dq; p.q_rows = a->q_rows;
  p.dk = a->dk; p.dv = a->dv; p.kv_rows = a->kv_rows;
  p.psplit = 1;
  if (pool) {
    p.dkp = reinterpret_cast<float*>(ws + w.dkp); p.dvp = reinterpret_cast<float*>(ws + w.dvp);
    p.psplit = w.psplit;
    p.dkp_part = reinterpret_cast<float*>(ws + w.dkp_part); p.dvp_part = reinterpret_cast<float*>(ws + w.dvp_part);
  }
  p.gap = pool ? a->pool_gap : 1;
  p.B = a->B; p.H = a->H; p.Lq = a->Lq; p.Lk = a->Lk; p.nbq = nbq; p.nbk = nbk;
  p.nbkp = pool ? (a->Lkp + 127) / 128 : 0;
  p.scale = a->scale > 0.f ? a->scale : (float)(1.0 / sqrt((double)a->D));
  p.c = p.scale * kLog2e;
  p.heavy_rows = a->heavy_rows;
  return dispatch_bwd(pp, p, a->D, a->dtype, pool, reinterpret_cast<hipStream_t>(stream), a->kernel_select,
                      a->kernels_ran);
}

extern "C" uint64_t vb_block_sparse_attn_bwd_workspace_size(int batch, int num_heads, int max_seqlen_q) {
  if (batch <= 0 || num_heads <= 0 || max_seqlen_q <= 0) return 0;
  return vb::ws_layout(batch, num_heads, max_seqlen_q, 64, false, 0).total;
}

extern "C" int vb_block_sparse_attn_bwd(const void* dout, const void* q_unpad, const void* k_unpad,
                                        const void* v_unpad, const void* out_unpad, const float* softmax_lse,
                                        const int32_t* cu_seqlens_q, const int32_t* cu_seqlens_k,
                                        const int32_t* head_mask_type, const int32_t* streaming_info,
                                        const uint8_t* base_blockmask, int batch, int num_heads, int head_dim,
                                        int max_seqlen_q, int max_seqlen_k, float p_dropout, float softmax_scale,
                                        int is_causal, int exact_streaming, int deterministic, int dtype,
                                        void* dq, void* dk, void* dv, void* workspace, uint64_t workspace_bytes,
                                        int mask_head_mode, void* stream) {
  using namespace vb;
  (void)streaming_info;
  (void)deterministic;  // always deterministic (no atomics)
  if (p_dropout != 0.f) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_bwd: p_dropout must be 0");
  if (is_causal || exact_streaming) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_bwd: causal/streaming not supported");
  if (mask_head_mode != VB_MASK_HEAD_PER_HEAD && mask_head_mode != VB_MASK_HEAD_SHARED0)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_bwd: unknown mask_head_mode");
  if (!dout || !q_unpad || !k_unpad || !v_unpad || !out_unpad || !softmax_lse || !cu_seqlens_q || !cu_seqlens_k ||
      !dq || !dk || !dv)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_bwd: null tensor");
  if (batch <= 0 || num_heads <= 0 || max_seqlen_q <= 0 || max_seqlen_k <= 0)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_bwd: bad sizes");
  if (head_dim != 64 && head_dim != 128)
    return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_bwd: head_dim must be 64 or 128");
  if (dtype != VB_DTYPE_BF16 && dtype != VB_DTYPE_F16) return fail(VB_ERR_INVALID, "vb_block_sparse_attn_bwd: unknown dtype");
  const int nbq = (max_seqlen_q + 127) / 128;
  const int nbk = (max_seqlen_k + 127) / 128;
  if (nbk > bwd::kMaxBlocks || nbq > bwd::kMaxBlocks) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_bwd: sequence too long");
  const WsLayout w = ws_layout(batch, num_heads, max_seqlen_q, head_dim, false, 0);
  if (!workspace || workspace_bytes < w.total || !al16(workspace))
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_bwd: workspace missing or too small");
  if (!slice_ok(max_seqlen_q, (int64_t)num_heads * head_dim, head_dim))
    return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_bwd: a sequence's q/dout span >= 2 GiB");
  if (!slice_ok(max_seqlen_k, (int64_t)num_heads * head_dim, head_dim))
    return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_bwd: a sequence's k/v span >= 2 GiB");
  const void* ptrs[] = {dout, q_unpad, k_unpad, v_unpad, out_unpad, dq, dk, dv};
  for (const void* q : ptrs)
    if (!al16(q)) return fail(VB_ERR_INVALID, "vb_block_sparse_attn_bwd: tensors must be 16-byte aligned");
  const int64_t row = (int64_t)num_heads * head_dim;
  int64_t s3[3] = {0, head_dim, row};

  PrepParams pp{};
  pp.q = q_unpad; pp.dout = dout; pp.out = out_unpad;
  for (int i = 0; i < 3; ++i) pp.qs[i] = pp.dos[i] = pp.os[i] = s3[i];
  pp.lse = softmax_lse;
  pp.cu_q = cu_seqlens_q;
  pp.stats = reinterpret_cast<float*>(reinterpret_cast<uint8_t*>(workspace) + w.stats);
  pp.B = batch; pp.H = num_heads; pp.Lq = max_seqlen_q; pp.D = head_dim; pp.ntile = (max_seqlen_q + 63) / 64;

  BwdParams p{};
  p.q = q_unpad; p.dout = dout; p.k = k_unpad; p.v = v_unpad;
  for (int i = 0; i < 3; ++i) p.qs[i] = p.dos[i] = p.ks[i] = p.vs[i] = p.dqs[i] = p.dks[i] = p.dvs[i] = s3[i];
  p.cu_q = cu_seqlens_q; p.cu_k = cu_seqlens_k; p.head_mask_type = head_mask_type;
  p.hm_mode = mask_head_mode;
  p.mask = base_blockmask;
  p.ms[0] = head_mask_type ? -1 : (int64_t)num_heads * nbq * nbk;
  p.ms[1] = (int64_t)nbq * nbk; p.ms[2] = nbk;
  p.stats = pp.stats; p.ntile = pp.ntile;
  p.dq = dq; p.dk = dk; p.dv = dv;
  p.gap = 1;
  p.psplit = 1;
  p.B = batch; p.H = num_heads; p.Lq = max_seqlen_q; p.Lk = max_seqlen_k; p.nbq = nbq; p.nbk = nbk;
  p.scale = softmax_scale > 0.f ? softmax_scale : (float)(1.0 / sqrt((double)head_dim));
  p.c = p.scale * kLog2e;
  return dispatch_bwd(pp, p, head_dim, dtype, false, reinterpret_cast<hipStream_t>(stream));
}

// ------------------------------------------------------------------------------------------------
// multi-level backward (kernels/block_sparse_attn_kernel_with_backward_9_10.py _backward :1375-1576)
// ------------------------------------------------------------------------------------------------
namespace vb {
struct MlWs {
  uint64_t stats, q_r, do_r, dkpyr, dvpyr, total;
};
static MlWs ml_ws_layout(int B, int H, int L, int D, bool copies) {
  auto up = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
  MlWs w{};
  const uint64_t ntile = (uint64_t)((L + 63) / 64);
  const uint64_t lpad = (uint64_t)(L + 127) / 128 * 128;
  uint64_t off = 0;
  w.stats = off; off = up(off + (uint64_t)B * H * ntile * 256 * 4);
  if (copies) {
    w.q_r = off; off = up(off + (uint64_t)B * H * L * D * 2);
    w.do_r = off; off = up(off + (uint64_t)B * H * L * D * 2);
  }
  w.dkpyr = off; off = up(off + (uint64_t)B * H * (7 * lpad / 8) * D * 4);
  w.dvpyr = off; off = up(off + (uint64_t)B * H * (7 * lpad / 8) * D * 4);
  w.total = off;
  return w;
}

template <int D, class T>
static int launch_ml_grads(const PrepParams& pp, const BwdParams& p, hipStream_t s, int sel, int& ran) {
  if (int rc = launch_prep<T>(pp, s)) return rc;
  ran |= VB_BWD_RAN_ML_PYRAMID;
  const int BH = p.B * p.H;
  // dQ stays last on the caller's stream: forked beside the pyramid and level-1 passes it measured
  // 0.987-0.990x (ForkScope)
  {
    constexpr int kW = D == 64 ? VB_ML_PYR_WAVES : 4, kRows = 32 * kW;   // items of kRows pyramid rows
    int items = 0;
    for (int e = 1; e < 4; ++e) items += ((p.Lpad >> e) + kRows - 1) / kRows;
    hipLaunchKernelGGL((bwd_dkdv_kernel<D, T, true, true, kW>), dim3(items * BH), dim3(kW * 64), 0, s, p);
  }
  if (int rc = check_launch("bwd_dkdv_kernel<multi-level pooled>")) return rc;
  if (!(sel & VB_BWD_SEL_DKDV_ROUND3)) {
    ran |= VB_BWD_RAN_DKDV_PIPE;
    if (int rc = launch_ml_dkdv_pipe(p, D, std::is_same<T, F16>::value, s)) return rc;
  } else {
    ran |= VB_BWD_RAN_DKDV_ROUND3;
    hipLaunchKernelGGL((bwd_dkdv_kernel<D, T, false, true>), dim3(p.nbk * BH), dim3(bwd::kThreads), 0, s, p);
    if (int rc = check_launch("bwd_dkdv_kernel<multi-level>")) return rc;
  }
  if (!(sel & VB_BWD_SEL_DQ_ROUND3)) {
    ran |= VB_BWD_RAN_DQ_PIPE_RING2;
    return launch_ml_dq_pipe(p, D, std::is_same<T, F16>::value, s);
  }
  ran |= VB_BWD_RAN_DQ_ROUND3;
  hipLaunchKernelGGL((bwd_dq_kernel<D, T, false, true>), dim3(p.nbq * BH), dim3(bwd::kThreads), 0, s, p);
  return check_launch("bwd_dq_kernel<multi-level>");
}
}  // namespace vb

extern "C" uint64_t vb_ml_attn_bwd_workspace_size(const vb_ml_attn_bwd_args* a) {
  if (!a || a->B <= 0 || a->H <= 0 || a->L <= 0 || a->D <= 0) return 0;
  return vb::ml_ws_layout(a->B, a->H, a->L, a->D, a->rows != nullptr).total;
}

extern "C" int vb_ml_attn_bwd(const vb_ml_attn_bwd_args* a, void* stream) {
  using namespace vb;
  if (!a) return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: null args");
  if (a->B <= 0 || a->H <= 0 || a->L <= 0) return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: B, H, L must be positive");
  if (a->D != 64 && a->D != 128)
    return fail(VB_ERR_UNSUPPORTED, "vb_ml_attn_bwd: head_dim must be 64 or 128, got " + std::to_string(a->D));
  if (a->dtype != VB_DTYPE_BF16 && a->dtype != VB_DTYPE_F16) return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: unknown dtype");
  if (!a->q || !a->kpyr || !a->vpyr || !a->level_mask || !a->out || !a->lse || !a->dout || !a->dq || !a->dk || !a->dv)
    return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: missing tensor");
  if (a->kernel_select & ~(VB_BWD_SEL_DKDV_ROUND3 | VB_BWD_SEL_DQ_ROUND3))
    return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: unsupported kernel_select bits (the multi-level dQ has one ring)");
  const int nb = (a->L + 127) / 128;
  if (nb > bwd::kMaxBlocks) return fail(VB_ERR_UNSUPPORTED, "vb_ml_attn_bwd: sequence too long");
  const int64_t* strides[] = {a->q_stride, a->out_stride, a->dout_stride, a->dq_stride, a->dk_stride, a->dv_stride};
  for (const int64_t* st : strides)
    if (!mul8(st)) return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: strides must be multiples of 8 elements");
  const void* ptrs[] = {a->q, a->kpyr, a->vpyr, a->out, a->dout, a->dq, a->dk, a->dv};
  for (const void* q : ptrs)
    if (!al16(q)) return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: tensors must be 16-byte aligned");
  const MlWs w = ml_ws_layout(a->B, a->H, a->L, a->D, a->rows != nullptr);
  if (!a->workspace || a->workspace_bytes < w.total || !al16(a->workspace))
    return fail(VB_ERR_INVALID, "vb_ml_attn_bwd: workspace missing or smaller than vb_ml_attn_bwd_workspace_size()");
  if (!a->rows && (!slice_ok(a->L, a->q_stride[2], a->D) || !slice_ok(a->L, a->dout_stride[2], a->D)))
    return fail(VB_ERR_UNSUPPORTED, "vb_ml_attn_bwd: a q/dout (b,h) slice spans >= 2 GiB");
  if ((int64_t)vb_kv_pyramid_rows(a->L) * 2 * a->D >= (int64_t(1) << 31))
    return fail(VB_ERR_UNSUPPORTED, "vb_ml_attn_bwd: a pyramid (b,h) slice spans >= 2 GiB");
  uint8_t* ws = reinterpret_cast<uint8_t*>(a->workspace);
  const int Lpad = nb * 128;
  const int R = 15 * (Lpad / 8);

  PrepParams pp{};
  pp.q = a->q; pp.dout = a->dout; pp.out = a->out;
  for (int i = 0; i < 3; ++i) { pp.qs[i] = a->q_stride[i]; pp.dos[i] = a->dout_stride[i]; pp.os[i] = a->out_stride[i]; }
  pp.lse = a->lse;
  pp.q_rows = a->rows;
  pp.stats = reinterpret_cast<float*>(ws + w.stats);
  if (a->rows) { pp.q_r = ws + w.q_r; pp.do_r = ws + w.do_r; }
  pp.B = a->B; pp.H = a->H; pp.Lq = a->L; pp.D = a->D; pp.ntile = (a->L + 63) / 64;

  BwdParams p{};
  if (a->rows) {
    p.q = ws + w.q_r; p.dout = ws + w.do_r;
    p.qs[0] = p.dos[0] = (int64_t)a->H * a->L * a->D;
    p.qs[1] = p.dos[1] = (int64_t)a->L * a->D;
    p.qs[2] = p.dos[2] = a->D;
  } else {
    p.q = a->q; p.dout = a->dout;
    for (int i = 0; i < 3; ++i) { p.qs[i] = a->q_stride[i]; p.dos[i] = a->dout_stride[i]; }
  }
  p.k = a->kpyr; p.v = a->vpyr;
  p.ks[0] = p.vs[0] = (int64_t)a->H * R * a->D;
  p.ks[1] = p.vs[1] = (int64_t)R * a->D;
  p.ks[2] = p.vs[2] = a->D;
  for (int i = 0; i < 3; ++i) {
    p.ms[i] = a->mask_stride[i];
    p.dqs[i] = a->dq_stride[i]; p.dks[i] = a->dk_stride[i]; p.dvs[i] = a->dv_stride[i];
  }
  p.mask = a->level_mask;
  p.stats = pp.stats; p.ntile = pp.ntile;
  p.dq = a->dq; p.q_rows = a->rows;
  p.dk = a->dk; p.dv = a->dv; p.kv_rows = a->rows;
  p.psplit = 1;
  p.gap = 1;
  p.B = a->B; p.H = a->H; p.Lq = a->L; p.Lk = a->L; p.nbq = nb; p.nbk = nb;
  p.nbkp = (nb + 1) / 2 + (nb + 3) / 4 + (nb + 7) / 8;
  p.Lpad = Lpad;
  p.ref_tail = a->ref_tail ? 1 : 0;
  p.dkpyr = reinterpret_cast<float*>(ws + w.dkpyr);
  p.dvpyr = reinterpret_cast<float*>(ws + w.dvpyr);
  p.scale = a->scale > 0.f ? a->scale : (float)(1.0 / sqrt((double)a->D));
  p.c = p.scale * kLog2e;
  p.heavy_rows = a->heavy_rows;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int sel = a->kernel_select;
  int ran = 0, rc;
  if (a->dtype == VB_DTYPE_BF16)
    rc = a->D == 64 ? launch_ml_grads<64, BF16>(pp, p, st, sel, ran) : launch_ml_grads<128, BF16>(pp, p, st, sel, ran);
  else
    rc = a->D == 64 ? launch_ml_grads<64, F16>(pp, p, st, sel, ran) : launch_ml_grads<128, F16>(pp, p, st, sel, ran);
  if (a->kernels_ran) *a->kernels_ran = ran;
  return rc;
}

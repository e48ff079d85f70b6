// dK / dV of the block-sparse FMHA backward at head_dim 128, hand-scheduled for gfx950 (MI355X).
//
// Same work items, operand maps, math and outputs as bwd_dkdv_kernel<128> (vb_attn_bwd.hip; the
// reference's backward semantics are described there): one workgroup per (b, h, 128-key block),
// wave = 32 keys, the 64-row Q / dO / stats tiles of the q-blocks that keep the key block streamed
// through LDS by LDS-DMA. What differs is the schedule. bwd_dkdv_kernel<128> runs one wave per SIMD
// (its registers allow no more) and leaves each step's latency exposed: S/dP MFMAs, then the
// exp/dS VALU with the MFMA pipe idle, then the dV/dK MFMAs, every LDS read waited for right
// before its MFMA (profiles/r04_pmc_bwd_wan.txt: MFMA busy 0.30).
//
// Here every wave runs one fixed stream of 64 MFMAs per tile t, in four sections of 16:
//   A = X(t,0)   S = Q.K^T and dP = dO.V^T of rows 0-31 (two interleaved chains)
//   B = Y(t-1,1) dV += dO^T.P, dK += Q^T.dS of the previous tile's rows 32-63
//   C = X(t,1)   rows 32-63
//   D = Y(t,0)   rows 0-31
// and places all other work in the gaps between the MFMAs (one gap per MFMA, pinned with
// sched_barrier): the exp / dS / pack arithmetic of X(t,0) spread over gaps 18-47 and of X(t,1)
// over gaps 50-63 and 0-15 of the next tile (64 VALU each, about two per gap); every MFMA's LDS
// operand read issued kLA gaps ahead (asm reads, waited with exact lgkmcnt counts derived from
// the schedule below); the tile's row statistics; the barrier (gap 52) and the nine LDS-DMA
// pieces of tile t+3 (gaps 52-60) into a 4-slot ring. K and V (the B operands of X) and the dK/dV
// accumulators live in AGPRs; all MFMAs are asm (v_mfma_f32_32x32x16); the VALU-write -> MFMA-read
// wait states the compiler cannot see for them are checked on the ISA (tools/diag/mfma_hazard_check.py).
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "vb_attn_bwd.hpp"

#ifndef VB_KV64_WAVES
#define VB_KV64_WAVES 1    // waves per SIMD the D=64 kernel is register-budgeted for (2 spills)
#endif
#ifndef VB_BWD_DQ128_RING
// ring slots of the D=128 dQ pipeline: 2 (two workgroups per CU; Wan backward 1.073x over the
// round-3 dQ, 1.057x over the 4-slot form, profiles/archive/r05_bwd_dq2_ab.log) or 4 (one per CU)
#define VB_BWD_DQ128_RING 2
#endif
#ifndef VB_DQ2_LA
#define VB_DQ2_LA 2        // operand lookahead of the 2-slot dQ pipeline
#endif
#ifndef VB_BWD_DQ64_RING
// ring slots of the D=64 dQ pipeline: 2 (CogVideoX backward 1.011x over 4, bit-for-bit the same
// math as the D=128 form; profiles/archive/r05_bwd_dq64_ring_ab.log) or 4
#define VB_BWD_DQ64_RING 2
#endif
#ifndef VB_DQ64_R2_WGS
#define VB_DQ64_R2_WGS 2     // workgroups per CU the D=64 2-slot form is register-budgeted for (3: 1.005x)
#endif
#ifndef VB_KV128_LA
#define VB_KV128_LA 4      // operand lookahead in MFMAs
#endif
#ifndef VB_KV128_NODMA
#define VB_KV128_NODMA 0   // diagnostic (wrong results): no DMA after the prologue
#endif
#ifndef VB_KV_ABL
#define VB_KV_ABL 0        // diagnostic ablations of the dK/dV kernel (wrong results): bit 0 no score
                           // VALU, bit 1 no operand LDS reads in the loop, bit 2 no tile barrier,
                           // bit 4 no DMA after the prologue
#endif
// s_nop 1 ahead of the asm MFMAs that read VALU-written registers (the packed P / dS, the -Delta
// seeds): off by default — the schedule places every such write >= 2 instructions before its MFMA,
// which tools/diag/mfma_hazard_check.py verifies on the ISA in tests/test_codegen.py (measured
// 2.2 % on the Wan backward)
#ifndef VB_KV_YNOP
#define VB_KV_YNOP 0
#endif
#if VB_KV_YNOP
#define KV_YNOP "s_nop 1\n\t"
#else
#define KV_YNOP ""
#endif
#ifndef VB_KV128_XNOP
#define VB_KV128_XNOP 0    // 1: s_nop 1 ahead of the S/dP MFMAs too (measured 2 % slower on the Wan backward)
#endif
#if VB_KV128_XNOP
#define KV_XNOP "s_nop 1\n\t"
#else
#define KV_XNOP ""
#endif

namespace vb {
namespace kvp {

constexpr int kLA = VB_KV128_LA;
static_assert(kLA >= 2 && kLA <= 4, "lookahead out of range (the next tile's operands are read in 4 gaps)");

// The per-tile schedule of head dim D: kSec MFMAs per section, N = 4 kSec per tile (gaps 0..N-1).
// LDS map (bytes): Q ring 4 x kTileBytes, dO ring 4 x kTileBytes, stats ring 4 x 1 KiB, the 1 KiB
// sink of the waves' padding DMA piece, the q-block list.
template <int D>
struct Sched {
  static constexpr int KS = D / 16, DT = D / 32, RB = 2 * D;
  static constexpr int kTileBytes = bwd::kT * RB;
  static constexpr int kSec = 2 * KS;        // 16 at D=128, 8 at D=64
  static constexpr int N = 4 * kSec;
  static constexpr int kQOff = 0;
  static constexpr int kDOOff = 4 * kTileBytes;
  static constexpr int kStOff = 8 * kTileBytes;
  static constexpr int kSinkOff = kStOff + 4096;
  static constexpr int kListOff = kSinkOff + 1024;
  static constexpr int kLdsBytes = kListOff + 2 * bwd::kMaxBlocks + 16 + 4 * (bwd::kMaxBlocks / 64);
  static constexpr int kPQ = kTileBytes / 1024 / 4;   // LDS-DMA pieces per wave and matrix
  static constexpr int kPieces = 2 * kPQ + 1;          // + stats (wave 0) or sink
  static constexpr int kRpp = 1024 / RB;               // rows per piece
  // V(t,0) in gaps kV0 .. kV0 + kV0n - 1 (after X(t,0), before Y(t,0)); V(t,1) in gaps kV1 .. N-1
  // and 0 .. kSec-1 of the next tile (before Y(t,1))
  static constexpr int kV0 = kSec + 2, kV0n = 2 * kSec - 2;
  static constexpr int kV1 = 3 * kSec + 2, kV1n = 2 * kSec - 2;
  // (a barrier right after section B, the last reads of slot t-1, with tile t+3's pieces spread
  // over the rest of the tile measured 1.00x / 0.99x, profiles/archive/r05_bwd_dma_spread_ab.log)
  static constexpr int kGb = N - 12;                   // the tile barrier
  static constexpr int kDma0 = kGb > kV1 ? kGb : kV1;  // DMA pieces of tile t+3 from here (needs the list entry)
  static constexpr int kLq0 = kV0 - 10;                // L' of rows 0-31 (two gaps)
  static constexpr int kDq1 = 2 * kSec - 8;            // -Delta seeds of rows 32-63 (two gaps)
  static constexpr int kLq1 = 3 * kSec - 8;            // L' of rows 32-63 (two gaps)
  static constexpr int kList = 3 * kSec - 6;           // the q-block of tile t+3
  static constexpr int kNx = kGb + 1;                  // tile t+1: -Delta seeds (2 gaps) and first operands
  static_assert(kDma0 + kPieces <= N, "DMA pieces past the tile");
  static_assert(kNx + 3 <= N - 1 - kLA, "next tile's operands must be covered by the last MFMA's wait");

  // ---- the LDS read schedule (drives both the issue and the lgkmcnt of every wait) ------------
  // gap h issues, in order: the operand reads of MFMA h + kLA (X: one ds_read_b128; Y: two
  // ds_read_b64_tr_b16), unless h + kLA >= N; then the extra reads of extra_reads(h)
  static constexpr int op_reads(int g) { return ((g / kSec) & 1) ? 2 : 1; }
  static constexpr int extra_reads(int h) {
    return (h == kLq0 || h == kLq0 + 1 || h == kDq1 || h == kDq1 + 1 || h == kLq1 || h == kLq1 + 1) ? 2
           : (h == kNx || h == kNx + 1) ? 2 + (h - kNx < kLA)
           : (h == kNx + 2 || h == kNx + 3) ? (h - kNx < kLA)
           : h == kList ? 1 : 0;
  }
  static constexpr int gap_reads(int h) { return (h + kLA < N ? op_reads(h + kLA) : 0) + extra_reads(h); }
  // lgkmcnt before MFMA g: the reads issued after g's operand (LDS returns in order); MFMAs
  // 0..kLA-1 read operands completed before the tile started
  static constexpr int wait_n(int g) {
    if (g < kLA) return 15;
    int n = extra_reads(g - kLA);
    for (int h = g - kLA + 1; h < g; ++h) n += gap_reads(h);
    return n > 15 ? 15 : n;
  }
  static_assert(extra_reads(kGb) == 0 && extra_reads(kGb - 1) == 0, "no read beside the barrier");
};

template <class F, int... Gs>
__device__ __forceinline__ void for_gaps(F&& f, std::integer_sequence<int, Gs...>) {
  (f(std::integral_constant<int, Gs>{}), ...);
}

// ---- asm building blocks (device pass only: the host pass has no VGPR/AGPR constraints) ----------
template <class T>
__device__ __forceinline__ void mf_zero(f32x16& d, const typename T::vec8& a, const typename T::vec8& b) {
#if __HIP_DEVICE_COMPILE__
  if constexpr (std::is_same<T, BF16>::value)
    asm volatile(KV_XNOP "v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "a"(b));
  else
    asm volatile(KV_XNOP "v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(d) : "v"(a), "a"(b));
#endif
}
// kSeed: the first MFMA of a dP chain, whose C operand (the -Delta seeds) may have been assembled by
// VALU moves: always padded
template <class T, bool kSeed = false>
__device__ __forceinline__ void mf_vacc(f32x16& d, const typename T::vec8& a, const typename T::vec8& b) {
#if __HIP_DEVICE_COMPILE__
  if constexpr (kSeed && !VB_KV128_XNOP) {
    if constexpr (std::is_same<T, BF16>::value)
      asm volatile(KV_YNOP "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
    else
      asm volatile(KV_YNOP "v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
  } else if constexpr (std::is_same<T, BF16>::value) {
    asm volatile(KV_XNOP "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
  } else {
    asm volatile(KV_XNOP "v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
  }
#endif
}
template <class T>
__device__ __forceinline__ void mf_aacc(f32x16& d, const typename T::vec8& a, const typename T::vec8& b) {
#if __HIP_DEVICE_COMPILE__
  if constexpr (std::is_same<T, BF16>::value)
    asm volatile(KV_YNOP "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b));
  else
    asm volatile(KV_YNOP "v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(d) : "v"(a), "v"(b));
#endif
}
template <int kImm, class V>
__device__ __forceinline__ void rd128(V& r, uint32_t addr) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(kImm));
#endif
}
template <int kImm>
__device__ __forceinline__ void rdtr(s16x4& r, uint32_t addr) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(kImm));
#endif
}
__device__ __forceinline__ void rd64(u32x2& r, uint32_t addr) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(addr));
#endif
}
__device__ __forceinline__ void rdu16(uint32_t& r, uint32_t addr) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("ds_read_u16 %0, %1" : "=v"(r) : "v"(addr));
#endif
}
template <int N, class V>
__device__ __forceinline__ void wait1(V& a) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N));
#endif
}
template <int N>
__device__ __forceinline__ void wait2(s16x4& a, s16x4& b) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N));
#endif
}
// makes a value produced by an asm read usable only after the wait that preceded this statement
template <class V>
__device__ __forceinline__ void launder(V& a) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(a));
#endif
}
// a value the optimizer cannot see through (see tile_dma in bwd_dq_pipe_kernel)
template <class V>
__device__ __forceinline__ V opaque(V a) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(a));
#endif
  return a;
}
__device__ __forceinline__ int uniform(int a) { return __builtin_amdgcn_readfirstlane(a); }
__device__ __forceinline__ const uint8_t* uniform_ptr(const uint8_t* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
}
template <class V>
__device__ __forceinline__ void to_agpr(V& a) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("" : "+a"(a));
#endif
}

// op k (0..63) of the score arithmetic of one 32-row half, in four stages of 16 so every op's
// input was produced >= 7 gaps earlier:
//   P = exp2(S c - L')   (fma, then exp, in place in s)
//   dS = P * dP          (dp holds dO.V^T - Delta: seeded with -Delta)
//   pp / pd = bf16 pairs of P / dS (the B operands of dV / dK)
template <class T, int k>
__device__ __forceinline__ void vop(f32x16& s, f32x16& dp, const f32x4 (&lq)[4], u32x4 (&pp)[2], u32x4 (&pd)[2],
                                    float c) {
  constexpr int st = k >> 4, r = k & 15;
  if constexpr (st == 0) s[r] = fmaf(s[r], c, -lq[r >> 2][r & 3]);
  else if constexpr (st == 1) s[r] = exp2_fast(s[r]);
  else if constexpr (st == 2) dp[r] = dp[r] * s[r];
  else if constexpr (r < 8) pp[r >> 2][r & 3] = pack2<T>(s[2 * r], s[2 * r + 1]);
  else pd[(r - 8) >> 2][(r - 8) & 3] = pack2<T>(dp[2 * (r - 8)], dp[2 * (r - 8) + 1]);
}
template <class T, int lo, int... Ks>
__device__ __forceinline__ void vops_at(f32x16& s, f32x16& dp, const f32x4 (&lq)[4], u32x4 (&pp)[2],
                                        u32x4 (&pd)[2], float c, std::integer_sequence<int, Ks...>) {
  (vop<T, lo + Ks>(s, dp, lq, pp, pd, c), ...);
}
// the ops of gap i (0..n-1) of a half's arithmetic spread over n gaps
template <class T, int i, int n>
__device__ __forceinline__ void vgap(f32x16& s, f32x16& dp, const f32x4 (&lq)[4], u32x4 (&pp)[2], u32x4 (&pd)[2],
                                     float c) {
  constexpr int lo = i * 64 / n, hi = (i + 1) * 64 / n;
  vops_at<T, lo>(s, dp, lq, pp, pd, c, std::make_integer_sequence<int, hi - lo>{});
}

// ---- the dQ kernel's schedule (bwd_dq_pipe_kernel): per 64-key tile t, sections
//   A = X(t,0) S^T = K.Q^T, dP^T = V.dO^T of keys 0-31 (kX MFMAs)   B = Y(t-1,1) dQ^T of keys 32-63 (kY)
//   C = X(t,1) keys 32-63                                          D = Y(t,0)   keys 0-31
// R = 4: a 4-slot K/V ring, one barrier per tile (kGb), the DMA of tile t+3 after it.
// R = 2: a 2-slot ring (64 KiB at D=128, so two workgroups per CU) filled half a tile at a time,
// with two barriers per tile. Half h of a tile is read by X(t,h) and, for K, by Y(t,h) one section
// (h = 0) or two (h = 1) later; each barrier first drains the wave's LDS reads, so the halves whose
// last reads precede it are free:
//   G1 = kC - L (before C's first operand reads): K half 1 of t-1 and V half 0 of t are free, and
//       half 1 of t must have landed; then the DMA of half 1 of tile t+1 (into t-1's slot);
//   G2 = N - L (before tile t+1's first reads): K half 0 and V half 1 of t are free, half 0 of t+1
//       must have landed; the DMA of half 0 of tile t+2 (into t's slot) follows in gaps 0.. of t+1.
// Every barrier waits for all but the last half-tile batch (vmcnt = kPieces / 2); each batch is
// issued a whole tile (N - L gaps or more) before its barrier.
template <int D, int R = 4, int L = kLA>
struct QSched {
  static_assert(R == 2 || R == 4, "ring slots");
  static_assert(L >= 2 && L <= 4, "lookahead");
  static constexpr int KS = D / 16, DT = D / 32, RB = 2 * D;
  static constexpr int kTileBytes = bwd::kT * RB;
  static constexpr int LA = L;
  static constexpr int kX = 2 * KS, kY = 2 * DT;
  static constexpr int N = 2 * kX + 2 * kY;
  static constexpr int kB = kX, kC = kX + kY, kD = 2 * kX + kY;
  static constexpr int kKOff = 0;
  static constexpr int kVOff = R * kTileBytes;
  static constexpr int kListOff = 2 * R * kTileBytes;
  static constexpr int kLdsBytes = kListOff + 2 * bwd::kMaxBlocks + 16 + 4 * (bwd::kMaxBlocks / 64);
  static constexpr int kPQ = kTileBytes / 1024 / 4;
  static constexpr int kPieces = 2 * kPQ;
  static constexpr int kRpp = 1024 / RB;
  static constexpr int kV0 = kB + 2, kV0n = kD - kV0;          // V(t,0): [kB+2, kD)
  static constexpr int kV1 = kD + 2, kV1n = N - kV1 + kB;      // V(t,1): [kD+2, N) and [0, kB) of t+1
  // R = 4
  static constexpr int kGb = R == 4 ? N - 12 : -1;             // the tile barrier (after section B)
  static constexpr int kDma0 = kGb + 1;
  // R = 2
  static constexpr int kG1 = R == 2 ? kC - L : -1, kG2 = R == 2 ? N - L : -1;
  static constexpr int kHalf = kPieces / 2;                    // pieces per half-tile batch
  static constexpr int kP0 = 0, kP1 = kG1 + 1;                 // first gaps of the two batches (back to
                                                               // back; spread 3 or 5 gaps apart: 1.00x)
  static constexpr int kList = R == 4 ? kGb - 6 : kG2 - 4;     // the key block of tile t+3 (R=4) / t+2
  static constexpr int kNx = R == 4 ? kGb + 1 : kG2;           // tile t+1's first operands
  static_assert(R == 2 || kGb >= kC, "the barrier must follow the reads of the previous tile");
  static_assert(R == 2 || kDma0 + kPieces <= N, "DMA pieces past the tile");
  static_assert(R == 4 || (kP1 + kHalf <= kG2 && kHalf <= kG1), "DMA batches overlap a barrier");
  static_assert(kNx + L - 1 <= N - 1 || R == 2, "next tile's operands must be covered by the last MFMA's wait");
  static_assert(R == 4 || kNx + L == N, "next tile's operands are read after G2");
  static constexpr int sec(int g) { return g < kB ? 0 : g < kC ? 1 : g < kD ? 2 : 3; }
  static constexpr int sec0(int c) { return c == 0 ? 0 : c == 1 ? kB : c == 2 ? kC : kD; }
  static constexpr int op_reads(int g) { return (sec(g) & 1) ? 2 : 1; }
  static constexpr int extra_reads(int h) { return (h == kList || (h >= kNx && h < kNx + L)) ? 1 : 0; }
  static constexpr int gap_reads(int h) { return (h + L < N ? op_reads(h + L) : 0) + extra_reads(h); }
  // lgkmcnt before MFMA g (reads issued after g's operand; a barrier's drain only lowers the count).
  // MFMAs g < L take the operands read at the end of the previous tile (nx): R = 4 reads them early
  // enough that the last MFMAs' waits cover them; R = 2 reads them after G2 and waits here.
  static constexpr int wait_n(int g) {
    if (g < L && R == 4) return 15;
    if (g < L) {
      int n = N - 1 - (kNx + g);
      for (int h = 0; h < g; ++h) n += gap_reads(h);
      return n > 15 ? 15 : n;
    }
    int n = extra_reads(g - L);
    for (int h = g - L + 1; h < g; ++h) n += gap_reads(h);
    return n > 15 ? 15 : n;
  }
  static_assert(R == 2 || extra_reads(kGb) == 0, "no read beside the barrier");
  static_assert(R == 4 || kList < kG2, "the list entry is read before G2's drain");
};

// d = a . b(AGPR) + c (c a separate VGPR tile: the dP^T chain's -Delta seeds, which hipcc
// assembles with v_movs right before this MFMA: always padded)
template <class T>
__device__ __forceinline__ void mf_cacc(f32x16& d, const typename T::vec8& a, const typename T::vec8& b,
                                        const f32x16& c) {
#if __HIP_DEVICE_COMPILE__
  if constexpr (std::is_same<T, BF16>::value)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "a"(b), "v"(c));
  else
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "a"(b), "v"(c));
#endif
}
// op k (0..55) of one 32-key half of the dQ pass: P = exp2(S c + nL), dS = P * dP (dP seeded with
// -Delta), pd = bf16 pairs of dS (the B operand of dQ^T += K^T.dS^T)
// kSeeded = false (the R = 2 kernel, whose registers do not hold a -Delta seed tile): dP starts
// from zero and dS = P * (dP + nd), nd = -Delta of the lane's row
template <class T, bool kSeeded, int k>
__device__ __forceinline__ void qop(f32x16& s, f32x16& dp, u32x4 (&pd)[2], float c, float nl, float nd) {
  constexpr int st = k >> 4, r = k & 15;
  if constexpr (st == 0) s[r] = fmaf(s[r], c, nl);
  else if constexpr (st == 1) s[r] = exp2_fast(s[r]);
  else if constexpr (st == 2) dp[r] = kSeeded ? dp[r] * s[r] : (dp[r] + nd) * s[r];
  else pd[r >> 2][r & 3] = pack2<T>(dp[2 * r], dp[2 * r + 1]);
}
template <class T, bool kSeeded, int lo, int... Ks>
__device__ __forceinline__ void qops_at(f32x16& s, f32x16& dp, u32x4 (&pd)[2], float c, float nl, float nd,
                                        std::integer_sequence<int, Ks...>) {
  (qop<T, kSeeded, lo + Ks>(s, dp, pd, c, nl, nd), ...);
}
template <class T, bool kSeeded, int i, int n>
__device__ __forceinline__ void qgap(f32x16& s, f32x16& dp, u32x4 (&pd)[2], float c, float nl, float nd) {
  constexpr int lo = i * 56 / n, hi = (i + 1) * 56 / n;
  qops_at<T, kSeeded, lo>(s, dp, pd, c, nl, nd, std::make_integer_sequence<int, hi - lo>{});
}

}  // namespace kvp

// D=128: one workgroup per CU (one wave per SIMD); D=64: VB_KV64_WAVES.
// kML: the multi-level backward's level-1 dK/dV (vb_ml_attn_bwd; bwd_dkdv_kernel<kPooled = false,
// kML>): K/V are the pyramids' level-1 rows, a key block takes the q-blocks whose level for it is 1,
// and each key adds the mean-pool adjoints of its level-2/4/8 pyramid rows (the reference kernel's
// _bwd_kv epilogue, block_sparse_attn_kernel_with_backward_9_10.py:1494-1563).
template <int D, class T, bool kPooled, bool kML = false>
__global__ void __launch_bounds__(bwd::kThreads, D == 128 ? 1 : VB_KV64_WAVES) bwd_dkdv_pipe_kernel(const BwdParams p) {
  using namespace bwd;
  using namespace kvp;
  static_assert(!(kML && kPooled), "the multi-level pooled levels run bwd_dkdv_kernel's union walk");
  using S = Sched<D>;
  using V8 = typename T::vec8;
  constexpr int KS = S::KS, DT = S::DT, RB = S::RB, N = S::N, kSec = S::kSec, TB = S::kTileBytes;
  constexpr int kPieces = S::kPieces, kPQ = S::kPQ;
  constexpr int fL = kPooled ? 2 : 0;   // stats fields of this branch: L' at fL, -Delta at fL + 1
  __shared__ __attribute__((aligned(16))) uint8_t smem[S::kLdsBytes];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + S::kListOff);
  int* list_n = reinterpret_cast<int*>(smem + S::kListOff + 2 * kMaxBlocks);
  int* chunk_n = list_n + 4;   // per-64-block chunk counts of the list build

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;

  // ---- work item: bwd_dkdv_kernel's mapping (heavy text columns first, then XCD-contiguous) ----
  const int BH = p.B * p.H;
  const int nkb = kPooled ? p.nbkp : p.nbk;
  const int split = kPooled ? (int)blockIdx.x % p.psplit : 0;
  int bh, kblk;
  if (kPooled) {
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
  const int Lkey = kPooled ? p.Lkp : Lk;
  const int k0 = kblk * kBlk;
  if (k0 >= Lkey || Lq <= 0) return;
  const int nbq = (Lq + kBlk - 1) / kBlk;

  bool nan_head = false;
  const uint8_t* mcol = nullptr;
  if (!kPooled) {
    const uint8_t* mh = head_mask_base(p.mask, p.ms, p.head_mask_type, p.H, b, h, nan_head, p.hm_mode);
    if (mh) mcol = mh + kblk;
  }
  const int qlo = kPooled ? split * nbq / p.psplit : 0;
  const int qhi = kPooled ? (split + 1) * nbq / p.psplit : nbq;
  // this wave's 32 keys as B operands (lane = key, d = 16 ks + 8 half + 0..7), held in AGPRs; loaded
  // first, so their latency overlaps the list build's mask loads
  const int key = k0 + wave * 32 + l32;
  const bool kvalid = key < Lkey;
  const int keyc = kvalid ? key : Lkey - 1;
  const uint8_t* kb = kPooled
      ? reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1] + (int64_t)keyc * p.kps[2])
      : reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1] + (krow0 + keyc) * p.ks[2]);
  const uint8_t* vb_ = kPooled
      ? reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1] + (int64_t)keyc * p.vps[2])
      : reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1] + (krow0 + keyc) * p.vs[2]);
  V8 kf[KS], vf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    kf[s] = *reinterpret_cast<const V8*>(kb + (16 * s + 8 * half) * 2);
    vf[s] = *reinterpret_cast<const V8*>(vb_ + (16 * s + 8 * half) * 2);
  }
  {   // the q-blocks that keep this key block, ascending: the four waves ballot 64-block chunks
      // wave, wave + 4, .. in one round of mask loads, then place their entries after the counts of
      // the chunks before them (a single wave's serial loop waited for one load round per chunk)
    constexpr int kCPW = kMaxBlocks / 64 / 4;   // chunks per wave
    unsigned long long bal[kCPW];
#pragma unroll
    for (int r = 0; r < kCPW; ++r) {
      const int i = qlo + 64 * (wave + 4 * r) + lane;
      const bool keep = (i < qhi) && (mcol == nullptr || (kML ? mcol[(int64_t)i * p.ms[2]] == 1 : mcol[(int64_t)i * p.ms[2]] != 0));
      bal[r] = __ballot(keep);
      if (lane == 0) chunk_n[wave + 4 * r] = __popcll(bal[r]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kCPW; ++r) {
      const int c = wave + 4 * r;
      int base = 0;
      for (int c2 = 0; c2 < c; ++c2) base += chunk_n[c2];
      if ((bal[r] >> lane) & 1)
        list[base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal[r] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal[r], 0u))] =
            (uint16_t)(qlo + 64 * c + lane);
    }
    if (threadIdx.x == 0) {
      int n = 0;
      for (int c = 0; c < 4 * kCPW; ++c) n += chunk_n[c];
      *list_n = n;
    }
  }

#pragma unroll
  for (int s = 0; s < KS; ++s) {
    to_agpr(kf[s]);
    to_agpr(vf[s]);
  }
  __syncthreads();
  const int nlist = __builtin_amdgcn_readfirstlane(*list_n);
  int ntiles = 2 * nlist;
  if (nlist > 0 && list[nlist - 1] == nbq - 1 && (nbq - 1) * kBlk + kT >= Lq) ntiles -= 1;

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[i][r] = dv[i][r] = 0.f;
#pragma unroll
  for (int i = 0; i < DT; ++i) {
    to_agpr(dk[i]);
    to_agpr(dv[i]);
  }
  static_assert(DT == 2 || DT == 4, "head dim 64 or 128");

  if (ntiles > 0) {
    const uint8_t* qsrc = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + qrow0 * p.qs[2]);
    const uint8_t* dosrc = reinterpret_cast<const uint8_t*>(p.dout) + 2 * (b * p.dos[0] + h * p.dos[1] + qrow0 * p.dos[2]);
    const int qrowb = 2 * (int)p.qs[2], dorowb = 2 * (int)p.dos[2];   // host: every slice < 2 GiB
    const float* stsrc = p.stats + (int64_t)bh * p.ntile * 256;
    const int qbytes = (int)((int64_t)(Lq - 1) * qrowb + RB);
    const int dobytes = (int)((int64_t)(Lq - 1) * dorowb + RB);
    const int stbytes = p.ntile * 1024;

    // Tile tt -> ring slot tt % 4: piece k of this wave is Q rows kRpp (wave + 4k).. (k < kPQ), dO
    // rows kRpp (wave + 4(k-kPQ)).. (k < 2 kPQ), and the stats KiB (wave 0) or a zero-extent piece
    // into the sink (waves 1-3), so every wave issues kPieces per tile and every vmcnt is a
    // constant. Tiles past the last one are zero-extent too (they land in slots nobody reads).
    int voff[kPieces];
#pragma unroll
    for (int k = 0; k < kPieces; ++k) {
      voff[k] = lane * 16;
      if (k < 2 * kPQ) {
        const int r = (wave + 4 * (k % kPQ)) * S::kRpp + lane / (RB / 16);
        const int c = (lane % (RB / 16)) ^ dual_swz<D>(r);
        voff[k] = r * (k < kPQ ? qrowb : dorowb) + c * 16;
      }
    }
    struct TileDma {
      srd_t q, dout, st;
      int soff_q, soff_do, soff_st;
    };
    auto tile_dma = [&](int tt, int qb) __attribute__((always_inline)) -> TileDma {
      const bool live = tt < ntiles && !(VB_KV128_NODMA && tt >= 3);
      const int row0 = qb * kBlk + (tt & 1) * kT;
      TileDma d;
      d.q = srd_t{qsrc, live ? qbytes : 0};
      d.dout = srd_t{dosrc, live ? dobytes : 0};
      d.st = srd_t{stsrc, (live && wave == 0) ? stbytes : 0};
      d.soff_q = row0 * qrowb;
      d.soff_do = row0 * dorowb;
      d.soff_st = (row0 / 64) * 1024;
      return d;
    };
    auto piece = [&](const TileDma& d, int slot, int k) __attribute__((always_inline)) {
      if (k < kPQ) dma16(d.q, smem + S::kQOff + slot * TB + (wave + 4 * k) * 1024, voff[k], d.soff_q);
      else if (k < 2 * kPQ)
        dma16(d.dout, smem + S::kDOOff + slot * TB + (wave + 4 * (k - kPQ)) * 1024, voff[k], d.soff_do);
      else dma16(d.st, smem + (wave == 0 ? S::kStOff + slot * 1024 : S::kSinkOff), voff[k], d.soff_st);
    };
    auto list_at = [&](int tt) __attribute__((always_inline)) -> int {
      return __builtin_amdgcn_readfirstlane((int)list[min(tt >> 1, nlist - 1)]);
    };

    // lane addresses of the asm reads (slot, row-half and k-step offsets are immediates)
    const uint32_t sbase = static_cast<uint32_t>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)smem));
    // When every dO offset fits the 16-bit immediate beside the Q ring (D=64), the dO reads use the
    // Q reads' address registers with +kDOOff in the immediate (NA = 1 address set, else 2).
    constexpr bool kShare = S::kDOOff + 3 * TB + 48 * RB < 65536;
    constexpr int NA = kShare ? 1 : 2;
    constexpr int kDOImm = kShare ? S::kDOOff : 0;
    uint32_t xa[NA][KS];       // [Q, dO][ks]: row l32, chunk 2 ks + half
    uint32_t ya[NA][DT][2];    // [Q, dO][dt][+0, +8 rows]: transposed reads
    const int trr = tr_row(lane), trc = tr_col(lane);
#pragma unroll
    for (int m = 0; m < NA; ++m) {
      const uint32_t rb = sbase + (m ? S::kDOOff : S::kQOff);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xa[m][ks] = rb + l32 * RB + 16 * ((2 * ks + half) ^ dual_swz<D>(l32));
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int p8 = 0; p8 < 2; ++p8) {
          const int r = trr + 8 * p8;
          ya[m][dt][p8] = rb + r * RB + 16 * ((4 * dt + (trc >> 3)) ^ dual_swz<D>(r)) + 2 * (trc & 7);
        }
    }
    const uint32_t sta = sbase + S::kStOff + 16 * half;
    const uint32_t lista = sbase + S::kListOff;
    const float c = p.c;

    f32x16 s0, dp0, s1, dp1;     // scores / dP of rows 0-31 and 32-63
    f32x4 dq0[4], dq1[4];        // -Delta seeds of dp0 / dp1 (asm reads)
    f32x4 lq0[4], lq1[4];        // L' of rows 0-31 / 32-63 (asm reads)
    u32x4 pp0[2], pd0[2], pp1[2], pd1[2];
    V8 nx[kLA];                  // operands of the next tile's first kLA MFMAs (read from gap kNx)
    uint32_t qb_raw = 0;         // the q-block of tile t+3 (asm read)
    TileDma dn{};                // the DMA of tile t+3

    // ---- prologue: tiles 0-2 in flight, tile 0 landed, its seeds and first operands read -------
    dn = tile_dma(0, list_at(0));
#pragma unroll
    for (int k = 0; k < kPieces; ++k) piece(dn, 0, k);
    dn = tile_dma(1, list_at(1));
#pragma unroll
    for (int k = 0; k < kPieces; ++k) piece(dn, 1, k);
    dn = tile_dma(2, list_at(2));
#pragma unroll
    for (int k = 0; k < kPieces; ++k) piece(dn, 2, k);
    VB_WAIT_VMCNT(2 * kPieces);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd128<(fL + 1) * 256 + 0 * 32>(dq0[0], sta);
    rd128<(fL + 1) * 256 + 1 * 32>(dq0[1], sta);
    rd128<(fL + 1) * 256 + 2 * 32>(dq0[2], sta);
    rd128<(fL + 1) * 256 + 3 * 32>(dq0[3], sta);
    rd128<0>(nx[0], xa[0][0]);
    rd128<kDOImm>(nx[1], xa[NA - 1][0]);
    if constexpr (kLA > 2) rd128<0>(nx[2], xa[0][1]);
    if constexpr (kLA > 3) rd128<kDOImm>(nx[3], xa[NA - 1][1]);
#if __HIP_DEVICE_COMPILE__
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
#pragma unroll
    for (int j = 0; j < 4; ++j) launder(dq0[j]);
#pragma unroll
    for (int q = 0; q < kLA; ++q) launder(nx[q]);

    // ---- one tile: U = slot of tile t, M = 0 steady, 1 first tile (no B section), 2 drain (only
    // the B section of the last tile, gaps 0-31) ------------------------------------------------
    auto iter = [&](int t, auto U, auto M) __attribute__((always_inline)) {
      constexpr int u = decltype(U)::value;
      constexpr int up = (u + 3) & 3, un = (u + 1) & 3;
      constexpr int mode = decltype(M)::value;
      V8 xop[N];
      s16x4 ylo[N], yhi[N];
      auto gap = [&](auto G) __attribute__((always_inline)) {
        constexpr int g = decltype(G)::value;
        constexpr int sc = g / kSec, i = g % kSec;
        // ---- MFMA g ----
        if constexpr (sc == 0 || sc == 2) {
          V8& a = g < kLA ? nx[g % kLA] : xop[g];
          if constexpr (g >= kLA) wait1<S::wait_n(g)>(a);
          if constexpr (g == 1 || g == 2 * kSec + 1) {
            f32x4 (&dq)[4] = g == 1 ? dq0 : dq1;
            f32x16& dp = g == 1 ? dp0 : dp1;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              launder(dq[j]);
#pragma unroll
              for (int e = 0; e < 4; ++e) dp[4 * j + e] = dq[j][e];
            }
          }
          if constexpr (mode != 2) {
            f32x16& s = sc == 0 ? s0 : s1;
            f32x16& dp = sc == 0 ? dp0 : dp1;
            constexpr int ks = i >> 1;
            if constexpr (i & 1) mf_vacc<T, i == 1>(dp, a, vf[ks]);
            else if constexpr (ks == 0) mf_zero<T>(s, a, kf[0]);
            else mf_vacc<T>(s, a, kf[ks]);
          }
        } else {
          wait2<S::wait_n(g)>(ylo[g], yhi[g]);
          constexpr bool run = sc == 1 ? mode != 1 : mode != 2;
          if constexpr (run) {
            constexpr int j = i >> 1, sb = j / DT, dt = j % DT;
            const V8 a = join8<T>(ylo[g], yhi[g]);
            if constexpr (i & 1) mf_aacc<T>(dk[dt], a, __builtin_bit_cast(V8, sc == 1 ? pd1[sb] : pd0[sb]));
            else mf_aacc<T>(dv[dt], a, __builtin_bit_cast(V8, sc == 1 ? pp1[sb] : pp0[sb]));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- fillers of gap g ----
        constexpr int m = g + kLA;   // operand reads of MFMA m
        if constexpr (m < N && !(VB_KV_ABL & 2)) {
          constexpr int ms = m / kSec, mi = m % kSec;
          if constexpr (ms == 0 || ms == 2) {
            rd128<u * TB + (ms >> 1) * 32 * RB + ((mi & 1) ? kDOImm : 0)>(xop[m], xa[(mi & 1) && !kShare][mi >> 1]);
          } else {
            constexpr int slot = ms == 1 ? up : u;
            constexpr int half_u = ms == 1 ? 1 : 0;
            constexpr int j = mi >> 1, sb = j / DT, dt = j % DT;
            constexpr int mat = (mi & 1) ? 0 : 1;   // dK reads Q, dV reads dO
            constexpr int imm = slot * TB + (32 * half_u + 16 * sb) * RB;
            constexpr int imm2 = imm + (mat ? kDOImm : 0);
            rdtr<imm2>(ylo[m], ya[mat && !kShare][dt][0]);
            rdtr<imm2>(yhi[m], ya[mat && !kShare][dt][1]);
          }
        }
        if constexpr (g == S::kLq0 || g == S::kLq0 + 1) {
          constexpr int j = 2 * (g - S::kLq0);
          rd128<u * 1024 + fL * 256 + (0 + 8 * j) * 4>(lq0[j], sta);
          rd128<u * 1024 + fL * 256 + (0 + 8 * (j + 1)) * 4>(lq0[j + 1], sta);
        }
        if constexpr (g == S::kDq1 || g == S::kDq1 + 1) {
          constexpr int j = 2 * (g - S::kDq1);
          rd128<u * 1024 + (fL + 1) * 256 + (32 + 8 * j) * 4>(dq1[j], sta);
          rd128<u * 1024 + (fL + 1) * 256 + (32 + 8 * (j + 1)) * 4>(dq1[j + 1], sta);
        }
        if constexpr (g == S::kLq1 || g == S::kLq1 + 1) {
          constexpr int j = 2 * (g - S::kLq1);
          rd128<u * 1024 + fL * 256 + (32 + 8 * j) * 4>(lq1[j], sta);
          rd128<u * 1024 + fL * 256 + (32 + 8 * (j + 1)) * 4>(lq1[j + 1], sta);
        }
        if constexpr (g == S::kList) rdu16(qb_raw, lista + 2 * min((t + 3) >> 1, nlist - 1));
        if constexpr (g == S::kNx || g == S::kNx + 1) {
          constexpr int j = 2 * (g - S::kNx);
          rd128<un * 1024 + (fL + 1) * 256 + (8 * j) * 4>(dq0[j], sta);
          rd128<un * 1024 + (fL + 1) * 256 + (8 * (j + 1)) * 4>(dq0[j + 1], sta);
        }
        if constexpr (g >= S::kNx && g < S::kNx + kLA) {
          constexpr int q = g - S::kNx;
          rd128<un * TB + ((q & 1) ? kDOImm : 0)>(nx[q], xa[(q & 1) && !kShare][q >> 1]);
        }
        // ---- score arithmetic ----
        if constexpr (!(VB_KV_ABL & 1) && mode != 2 && g >= S::kV0 && g < S::kV0 + S::kV0n) {
          if constexpr (g == S::kV0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) launder(lq0[j]);
          }
          vgap<T, g - S::kV0, S::kV0n>(s0, dp0, lq0, pp0, pd0, c);
        }
        if constexpr (!(VB_KV_ABL & 1) && mode != 2 && g >= S::kV1) {
          if constexpr (g == S::kV1) {
#pragma unroll
            for (int j = 0; j < 4; ++j) launder(lq1[j]);
          }
          vgap<T, g - S::kV1, S::kV1n>(s1, dp1, lq1, pp1, pd1, c);
        }
        if constexpr (!(VB_KV_ABL & 1) && mode != 1 && g < S::kV1 + S::kV1n - N) vgap<T, g + N - S::kV1, S::kV1n>(s1, dp1, lq1, pp1, pd1, c);
        // ---- barrier and the DMA of tile t+3 into the slot tile t-1 left ----
        if constexpr (mode != 2 && g == S::kV1) {
          launder(qb_raw);
          dn = tile_dma(t + 3, __builtin_amdgcn_readfirstlane((int)qb_raw));
        }
        if constexpr (mode != 2 && g == S::kGb) {
          VB_WAIT_VMCNT(kPieces);   // tile t+1 landed (tile t+2 may be in flight)
          if constexpr (!(VB_KV_ABL & 4)) __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
        if constexpr (!(VB_KV_ABL & 16) && mode != 2 && g >= S::kDma0 && g < S::kDma0 + kPieces) piece(dn, up, g - S::kDma0);
        if constexpr (g == N - 1) {
#pragma unroll
          for (int q = 0; q < kLA; ++q) launder(nx[q]);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      if constexpr (mode == 2) {
        for_gaps(gap, std::make_integer_sequence<int, 2 * kSec>{});
        // The drain stops after the B section with reads in flight whose consumers it never
        // reaches (the L' of rows 0-31, the seeds of rows 32-63, the operands of the C section's
        // first kLA MFMAs). Keep their
        // registers live past a full wait: hipcc must not hand a register to another value while
        // an LDS read is still due to write it.
#if __HIP_DEVICE_COMPILE__
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          launder(lq0[j]);
          launder(dq1[j]);
        }
#pragma unroll
        for (int q = 2 * kSec; q < 2 * kSec + kLA; ++q) launder(xop[q]);
      } else {
        for_gaps(gap, std::make_integer_sequence<int, N>{});
      }
    };

    // Tiles 1.. in groups of four (slots 1, 2, 3, 0: every LDS offset an immediate), so the loop
    // body is one straight block; the up-to-three tiles past ntiles are zero tiles (zero-extent
    // DMA: Q = dO = 0 and L' = -Delta = 0, hence P = 1, dP = 0, dS = 0: they add exact zeros).
    iter(0, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    int t = 1;
    for (; t < ntiles; t += 4) {
      iter(t, std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
      iter(t + 1, std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{});
      iter(t + 2, std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{});
      iter(t + 3, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    }
    iter(t, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});   // B section of tile t-1
#if __HIP_DEVICE_COMPILE__
    // drain: the zero-extent DMA of tiles past the end must land before the LDS is released, and
    // the dK/dV accumulators (asm MFMA results) need their wait states before the VALU reads them
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+a"(dk[0]), "+a"(dk[1]), "+a"(dv[0]), "+a"(dv[1])::"memory");
    if constexpr (DT == 4) asm volatile("s_nop 0" : "+a"(dk[2]), "+a"(dk[3]), "+a"(dv[2]), "+a"(dv[3])::"memory");
#endif
  }

  // ---- epilogue: lane = key, registers = d (bwd_dkdv_kernel's) ---------------------------------
  if (!kvalid) return;
  const float nanf_ = __builtin_nanf("");
  if (kPooled) {
    const int64_t po = ((int64_t)split * BH + bh) * p.Lkp + key;
    float* dkr = p.dkp_part + po * D;
    float* dvr = p.dvp_part + po * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * half;
        f32x4 a, cc;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = dk[dt][4 * g4 + e] * p.scale;
          cc[e] = dv[dt][4 * g4 + e];
        }
        *reinterpret_cast<f32x4*>(dkr + d) = a;
        *reinterpret_cast<f32x4*>(dvr + d) = cc;
      }
    return;
  }
  if constexpr (kML) {   // level-1 key: + the mean-pool adjoints of its level-2/4/8 pyramid rows
    const int64_t rb = (int64_t)bh * (7 * (p.Lpad / 8));
    const float* qk[3];
    const float* qv[3];
#pragma unroll
    for (int e = 1; e < 4; ++e) {
      const int64_t row = rb + (MlGeom(p.Lpad).off[e] - p.Lpad) + (key >> e);
      qk[e - 1] = p.dkpyr + row * D;
      qv[e - 1] = p.dvpyr + row * D;
    }
    const int64_t orow = p.kv_rows ? p.kv_rows[key] : krow0 + key;
    uint8_t* dkr = reinterpret_cast<uint8_t*>(p.dk) + 2 * (b * p.dks[0] + h * p.dks[1] + orow * p.dks[2]);
    uint8_t* dvr = reinterpret_cast<uint8_t*>(p.dv) + 2 * (b * p.dvs[0] + h * p.dvs[1] + orow * p.dvs[2]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * half;
        float a[4], cc[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = dk[dt][4 * g4 + e] * p.scale;
          cc[e] = dv[dt][4 * g4 + e];
        }
#pragma unroll
        for (int lv = 0; lv < 3; ++lv) {
          const float w = 1.0f / (float)(2 << lv);
          const f32x4 x = *reinterpret_cast<const f32x4*>(qk[lv] + d);
          const f32x4 y = *reinterpret_cast<const f32x4*>(qv[lv] + d);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[e] = fmaf(x[e], w, a[e]);
            cc[e] = fmaf(y[e], w, cc[e]);
          }
        }
        u32x2 w2, z;
        w2[0] = pack2<T>(a[0], a[1]); w2[1] = pack2<T>(a[2], a[3]);
        z[0] = pack2<T>(cc[0], cc[1]); z[1] = pack2<T>(cc[2], cc[3]);
        *reinterpret_cast<u32x2*>(dkr + d * 2) = w2;
        *reinterpret_cast<u32x2*>(dvr + d * 2) = z;
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
      float a[4], cc[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = dk[dt][4 * g4 + e] * p.scale;
        cc[e] = dv[dt][4 * g4 + e];
      }
      if (pk) {
        const f32x4 x = *reinterpret_cast<const f32x4*>(pk + d);
        const f32x4 y = *reinterpret_cast<const f32x4*>(pv + d);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = fmaf(x[e], pw, a[e]);
          cc[e] = fmaf(y[e], pw, cc[e]);
        }
      }
      if (nan_head) {
#pragma unroll
        for (int e = 0; e < 4; ++e) a[e] = cc[e] = nanf_;
      }
      u32x2 w, z;
      w[0] = pack2<T>(a[0], a[1]); w[1] = pack2<T>(a[2], a[3]);
      z[0] = pack2<T>(cc[0], cc[1]); z[1] = pack2<T>(cc[2], cc[3]);
      *reinterpret_cast<u32x2*>(dkr + d * 2) = w;
      *reinterpret_cast<u32x2*>(dvr + d * 2) = z;
    }
}


// ------------------------------------------------------------------------------------------------
// dQ: one workgroup per (b, h, 128-row q-block), wave = 32 query rows (bwd_dq_kernel's geometry and
// math), kept full-resolution K/V tiles then the pooled ones, on the same hand-placed stream as the
// dK/dV kernel above (QSched). Keys past a tile's end read as zero rows (buffer extent), which add
// nothing to dQ (dQ^T += K^T.dS^T with K = 0).
// ------------------------------------------------------------------------------------------------
// R = 4: the 4-slot ring (one workgroup per CU at D=128); R = 2: the 2-slot ring with half-tile DMA
// batches, two workgroups per CU (QSched).
// kML: the multi-level backward's dQ (vb_ml_attn_bwd; the reference kernel's _bwd_dq pass,
// block_sparse_attn_kernel_with_backward_9_10.py:1420-1505): K/V are the pyramids, and the tiles are
// bwd_dq_kernel<kML>'s: level 1 (two per kept block), one per level-2 block, two level-4 blocks and
// four level-8 blocks per tile, each tile carrying its level's +log2(p) logit bias. A tile's four
// 16-row quarters come from a per-tile table built in the prologue; a quarter past its level's list
// and level-1 keys past L (without ref_tail) read as zero rows.
template <int D, class T, bool kPool, int R, bool kML = false>
__global__ void __launch_bounds__(bwd::kThreads, R == 2 ? (D == 128 ? (kML ? 1 : 2) : VB_DQ64_R2_WGS) : (D == 128 ? 1 : VB_KV64_WAVES))
    bwd_dq_pipe_kernel(const BwdParams p) {
  using namespace bwd;
  using namespace kvp;
  using S = QSched<D, R, R == 2 ? VB_DQ2_LA : kLA>;
  using V8 = typename T::vec8;
  static_assert(!kML || (R == 2 && !kPool), "the multi-level dQ runs on the 2-slot ring, no pooled branch");
  constexpr int KS = S::KS, DT = S::DT, RB = S::RB, N = S::N, TB = S::kTileBytes;
  constexpr int kPieces = S::kPieces, kPQ = S::kPQ;
  constexpr int kLA = S::LA;              // shadows kvp::kLA
  constexpr bool kSeeded = R == 4;        // R = 2 holds no -Delta seed tile (qop)
  // multi-level: per tile, its four quarters' pyramid rows / 16 (u16; 0xFFFF = a zero quarter)
  constexpr int kMlTiles = 2 * kMaxBlocks + kMaxBlocks + kMaxBlocks / 2 + kMaxBlocks / 4 + 8;
  constexpr int kTabOff = (S::kLdsBytes + 7) / 8 * 8;
  __shared__ __attribute__((aligned(16))) uint8_t smem[kML ? kTabOff + 8 * kMlTiles : S::kLdsBytes];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + S::kListOff);
  int* list_n = reinterpret_cast<int*>(smem + S::kListOff + 2 * kMaxBlocks);   // [4] + chunk counts

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int half = lane >> 5;
  const int l32 = lane & 31;

  // heavy-first, then XCD-contiguous head-major (bwd_dq_kernel's mapping)
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

  // this wave's 32 query rows: Q and dO as B operands (lane = query), held in AGPRs
  const int g = q0 + wave * 32 + l32;
  const bool qvalid = g < Lq;
  const int gc = qvalid ? g : Lq - 1;
  V8 qf[KS], df[KS];
  // row statistics of the clamped row, as the Q/dO loads (padding waves of a short last q-block
  // would otherwise read past the stats region; their rows are never stored)
  const float* st = p.stats + ((int64_t)bh * p.ntile + gc / 64) * 256 + (gc & 63);
  const float L1 = st[0], D1 = st[64], L2 = st[128], D2 = st[192];   // D1, D2 = -Delta
  {   // (these loads first: their latency overlaps the list build's mask loads)
    const uint8_t* qp = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + (qrow0 + gc) * p.qs[2]);
    const uint8_t* dp_ = reinterpret_cast<const uint8_t*>(p.dout) + 2 * (b * p.dos[0] + h * p.dos[1] + (qrow0 + gc) * p.dos[2]);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      qf[s] = *reinterpret_cast<const V8*>(qp + (16 * s + 8 * half) * 2);
      df[s] = *reinterpret_cast<const V8*>(dp_ + (16 * s + 8 * half) * 2);
    }
    if constexpr (kML) {   // per-level key-block lists, levels 1, 2, 4, 8 in that order (wave 0)
      if (wave == 0) {
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
              list[pos[e] + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u))] =
                  (uint16_t)j;
            pos[e] += __popcll(bal);
          }
#if __HIP_DEVICE_COMPILE__
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // a bounded LDS-counter state per iteration (lgkm_check)
#endif
        }
        if (lane < 4) list_n[lane] = lane == 0 ? cnt[0] : lane == 1 ? cnt[1] : lane == 2 ? cnt[2] : cnt[3];
      }
    } else {   // the kept key blocks, ascending: the four waves ballot 64-block chunks wave, wave + 4, .. in
               // one round of mask loads, then place their entries after the counts of the chunks before them
      constexpr int kCPW = kMaxBlocks / 64 / 4;
      int* chunk_n = list_n + 4;
      unsigned long long bal[kCPW];
#pragma unroll
      for (int r = 0; r < kCPW; ++r) {
        const int j = 64 * (wave + 4 * r) + lane;
        const bool keep = use_main && (j < nbk) && (mrow == nullptr || mrow[j] != 0);
        bal[r] = __ballot(keep);
        if (lane == 0) chunk_n[wave + 4 * r] = __popcll(bal[r]);
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < kCPW; ++r) {
        const int c = wave + 4 * r;
        int base = 0;
        for (int c2 = 0; c2 < c; ++c2) base += chunk_n[c2];
        if ((bal[r] >> lane) & 1)
          list[base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal[r] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal[r], 0u))] =
              (uint16_t)(64 * c + lane);
      }
      if (threadIdx.x == 0) {
        int n = 0;
        for (int c = 0; c < 4 * kCPW; ++c) n += chunk_n[c];
        *list_n = n;
      }
    }

#pragma unroll
    for (int s = 0; s < KS; ++s) {
      to_agpr(qf[s]);
      to_agpr(df[s]);
    }
  }
  __syncthreads();
  const int nkept = __builtin_amdgcn_readfirstlane(*list_n);
  int ntm = 2 * nkept;
  if (nkept > 0 && list[nkept - 1] == nbk - 1 && (nbk - 1) * kBlk + kT >= Lk && !(kML && p.ref_tail)) ntm -= 1;
  const int ntp = kPool ? (p.Lkp + kT - 1) / kT : 0;
  // multi-level tile ranges: [0, ntm) level 1, [ntm, T12) level 2, [T12, T124) level 4, then level 8
  int T12 = ntm, T124 = ntm, ntiles = ntm + ntp;
  if constexpr (kML) {
    const int n2 = __builtin_amdgcn_readfirstlane(list_n[1]);
    const int n4 = __builtin_amdgcn_readfirstlane(list_n[2]);
    const int n8 = __builtin_amdgcn_readfirstlane(list_n[3]);
    T12 = ntm + n2;
    T124 = T12 + (n4 + 1) / 2;
    ntiles = T124 + (n8 + 3) / 4;
    // the quarter table (bwd_dq_kernel<kML>'s ml_quarter, rows / 16; zero quarters past a list)
    const int r2 = p.Lpad / 16, r4 = r2 + p.Lpad / 32, r8 = r4 + p.Lpad / 64;
    uint32_t* tab = reinterpret_cast<uint32_t*>(smem + kTabOff);
    // branch-free per entry (selects): one list read per quarter
    for (int tt = threadIdx.x; tt < ntiles; tt += kThreads) {
      const int lv = (tt >= ntm) + (tt >= T12) + (tt >= T124);
      uint32_t w[2] = {0u, 0u};
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        const int e = lv == 2 ? 2 * (tt - T12) + (qd >> 1) : 4 * (tt - T124) + qd;   // levels 4, 8
        const int li = lv == 0 ? tt >> 1 : lv == 1 ? nkept + tt - ntm : lv == 2 ? nkept + n2 + e : nkept + n2 + n4 + e;
        const bool ok = lv < 2 || e < (lv == 2 ? n4 : n8);
        const int blk = (int)list[max(min(li, kMaxBlocks - 1), 0)];
        const int r16 = lv == 0 ? blk * 8 + (tt & 1) * 4 + qd
                      : lv == 1 ? r2 + blk * 4 + qd
                      : lv == 2 ? r4 + blk * 2 + (qd & 1)
                                : r8 + blk;
        w[qd >> 1] |= (uint32_t)(ok ? r16 : 0xFFFF) << (16 * (qd & 1));
      }
      tab[2 * tt] = w[0];
      tab[2 * tt + 1] = w[1];
#if __HIP_DEVICE_COMPILE__
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // a bounded LDS-counter state per iteration (lgkm_check)
#endif
    }
    __syncthreads();
  }

  f32x16 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[i][r] = 0.f;
#pragma unroll
  for (int i = 0; i < DT; ++i) to_agpr(dq[i]);

  if (ntiles > 0) {
    const uint8_t* kbase = use_main ? reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1] + krow0 * p.ks[2]) : nullptr;
    const uint8_t* vbase = use_main ? reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1] + krow0 * p.vs[2]) : nullptr;
    const uint8_t* kpbase = kPool ? reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1]) : nullptr;
    const uint8_t* vpbase = kPool ? reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1]) : nullptr;
    const int krowb = 2 * (int)p.ks[2], vrowb = 2 * (int)p.vs[2];
    const int kprowb = kPool ? 2 * (int)p.kps[2] : 0, vprowb = kPool ? 2 * (int)p.vps[2] : 0;
    const int kbytes = use_main ? (int)((int64_t)(Lk - 1) * krowb + RB) : 0;
    const int vbytes = use_main ? (int)((int64_t)(Lk - 1) * vrowb + RB) : 0;
    const int kpbytes = kPool ? (int)((int64_t)(p.Lkp - 1) * kprowb + RB) : 0;
    const int vpbytes = kPool ? (int)((int64_t)(p.Lkp - 1) * vprowb + RB) : 0;
    // piece k of this wave: K rows kRpp (wave + 4k).. (k < kPQ), V rows kRpp (wave + 4(k-kPQ))..;
    // the lane's voffset per key source (main / pooled row strides). R = 2 keeps piece 0's only:
    // the swizzle depends on row bits the piece index does not touch (rows differ by 4 kRpp k), so
    // piece k adds 4 kRpp k rows as a scalar offset (TileDma::krb / vrb)
    // Multi-level: a piece's rows lie in one 16-row quarter (pieces start at multiples of kRpp),
    // so its voffset is the row within the quarter and the quarter's pyramid row the soffset.
    constexpr int kVo = R == 2 ? 2 : kPieces;
    int voff_m[kVo], voff_p[kVo];
#pragma unroll
    for (int k = 0; k < kVo; ++k) {
      const bool isv = R == 2 ? k == 1 : k >= kPQ;
      const int r = (wave + 4 * (R == 2 ? 0 : k % kPQ)) * S::kRpp + lane / (RB / 16);
      const int c16 = 16 * ((lane % (RB / 16)) ^ dual_swz<D>(r));
      voff_m[k] = (kML ? (r & 15) : r) * (isv ? vrowb : krowb) + c16;
      voff_p[k] = r * (isv ? vprowb : kprowb) + c16;
    }
    struct TileDma {
      srd_t k, v;
      int soff_k, soff_v;
      int krb, vrb;   // row strides (R = 2)
      bool pooled;
      int qk[4], qv[4];   // multi-level: the quarters' byte offsets (K, V)
    };
    // tile tt's source: kept block list[tt/2] half tt%2, then pooled tiles; past the end zero-extent
    // Every select below takes opaque operands (readfirstlane / an empty asm): hipcc otherwise turns
    // a select between two loads of captured locals into a load through a selected address, which
    // moves those locals to scratch.
    // The pooled variant blends the main and pooled sources with a uniform mask (x ^ ((x ^ y) & pm))
    // of values made uniform once, here: a select between them compiles to a branch per field.
    struct Src {
      uint32_t klo, khi, vlo, vhi;
      int kbytes, vbytes, krowb, vrowb;
    };
    auto src_of = [](const uint8_t* kb, const uint8_t* vb, int kby, int vby, int krb, int vrb) -> Src {
      const uint64_t k = reinterpret_cast<uint64_t>(kb), v = reinterpret_cast<uint64_t>(vb);
      return Src{(uint32_t)uniform((int)(uint32_t)k), (uint32_t)uniform((int)(uint32_t)(k >> 32)),
                 (uint32_t)uniform((int)(uint32_t)v), (uint32_t)uniform((int)(uint32_t)(v >> 32)),
                 uniform(kby), uniform(vby), uniform(krb), uniform(vrb)};
    };
    const Src sm = src_of(kbase, vbase, kbytes, vbytes, krowb, vrowb);
    Src sx{};   // main ^ pooled
    if constexpr (kPool) {
      const Src sp = src_of(kpbase, vpbase, kpbytes, vpbytes, kprowb, vprowb);
      sx = Src{sm.klo ^ sp.klo, sm.khi ^ sp.khi, sm.vlo ^ sp.vlo, sm.vhi ^ sp.vhi,
               sm.kbytes ^ sp.kbytes, sm.vbytes ^ sp.vbytes, sm.krowb ^ sp.krowb, sm.vrowb ^ sp.vrowb};
    }
    auto tile_dma = [&](int tt, int blk) __attribute__((always_inline)) -> TileDma {
      TileDma d;
      d.pooled = kPool && tt >= ntm;
      const int pm = kPool ? -(int)(tt >= ntm) : 0;
      const int lm = -(int)(tt < ntiles);
      const int kstart = d.pooled ? (tt - ntm) * kT : blk * kBlk + (tt & 1) * kT;
      const uint32_t klo = sm.klo ^ (sx.klo & (uint32_t)pm), khi = sm.khi ^ (sx.khi & (uint32_t)pm);
      const uint32_t vlo = sm.vlo ^ (sx.vlo & (uint32_t)pm), vhi = sm.vhi ^ (sx.vhi & (uint32_t)pm);
      d.k = srd_t{reinterpret_cast<const void*>(((uint64_t)khi << 32) | klo), (sm.kbytes ^ (sx.kbytes & pm)) & lm};
      d.v = srd_t{reinterpret_cast<const void*>(((uint64_t)vhi << 32) | vlo), (sm.vbytes ^ (sx.vbytes & pm)) & lm};
      d.krb = sm.krowb ^ (sx.krowb & pm);
      d.vrb = sm.vrowb ^ (sx.vrowb & pm);
      d.soff_k = kstart * d.krb;
      d.soff_v = kstart * d.vrb;
      return d;
    };
    // multi-level tile tt from its table entry (w0 = quarters 0-1, w1 = 2-3, rows / 16): level-1
    // tiles end at L unless ref_tail (zero rows past it), the other levels at the pyramid's end
    const int ml_kall = kML ? (int)((int64_t)(15 * (p.Lpad / 8) - 1) * krowb + RB) : 0;
    const int ml_vall = kML ? (int)((int64_t)(15 * (p.Lpad / 8) - 1) * vrowb + RB) : 0;
    auto tile_dma_ml = [&](int tt, uint32_t w0, uint32_t w1) __attribute__((always_inline)) -> TileDma {
      TileDma d{};
      const int lm = -(int)(tt < ntiles);
      const bool l1 = tt < ntm && !p.ref_tail;
      d.k = srd_t{reinterpret_cast<const void*>(((uint64_t)sm.khi << 32) | sm.klo), (l1 ? sm.kbytes : uniform(ml_kall)) & lm};
      d.v = srd_t{reinterpret_cast<const void*>(((uint64_t)sm.vhi << 32) | sm.vlo), (l1 ? sm.vbytes : uniform(ml_vall)) & lm};
      d.krb = krowb;
      d.vrb = vrowb;
      const int q16[4] = {(int)(w0 & 0xFFFF), (int)(w0 >> 16), (int)(w1 & 0xFFFF), (int)(w1 >> 16)};
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        d.qk[qd] = q16[qd] * 16 * krowb;
        d.qv[qd] = q16[qd] * 16 * vrowb;
      }
      return d;
    };
    auto piece = [&](const TileDma& d, int slot, int k) __attribute__((always_inline)) {
      const int kv = R == 2 ? (k >= kPQ) : k;
      if constexpr (kML) {
        // the piece's quarter: (kRpp (wave + 4 kk)) / 16 = q0 + (kRpp wave) / 16 with q0 known here
        // and the wave part 0 (D=128) or wave / 2 (D=64), blended with a uniform mask (a select
        // between the two fields would become an indexed load from scratch)
        const int kk = k < kPQ ? k : k - kPQ;
        const int q0 = (S::kRpp * 4 * kk) >> 4;
        int sk = d.qk[q0], sv = d.qv[q0];
        if constexpr (S::kRpp * 3 >= 16) {
          int wm = uniform(-(((S::kRpp * wave) >> 4) & 1));
#if __HIP_DEVICE_COMPILE__
          asm volatile("" : "+s"(wm));
#endif
          sk = (sk & ~wm) | (d.qk[(q0 + 1) & 3] & wm);
          sv = (sv & ~wm) | (d.qv[(q0 + 1) & 3] & wm);
        }
        if (k < kPQ) dma16(d.k, smem + S::kKOff + slot * TB + (wave + 4 * k) * 1024, voff_m[kv], sk);
        else dma16(d.v, smem + S::kVOff + slot * TB + (wave + 4 * kk) * 1024, voff_m[kv], sv);
        return;
      }
      int vo = voff_m[kv];
      if constexpr (kPool) {   // one v_bfi on a uniform mask; a select here becomes a branch per piece
        int pm = uniform(d.pooled ? -1 : 0);
#if __HIP_DEVICE_COMPILE__
        asm volatile("" : "+s"(pm));
#endif
        vo = (pm & voff_p[kv]) | (~pm & vo);
      }
      const int kk = k < kPQ ? k : k - kPQ;
      const int radd = R == 2 ? 4 * S::kRpp * kk : 0;   // rows past piece 0 (scalar)
      if (k < kPQ) dma16(d.k, smem + S::kKOff + slot * TB + (wave + 4 * k) * 1024, vo, d.soff_k + radd * d.krb);
      else dma16(d.v, smem + S::kVOff + slot * TB + (wave + 4 * kk) * 1024, vo, d.soff_v + radd * d.vrb);
    };
    // piece j (0..kHalf-1) of half h's batch: K pieces h kPQ/2.., then V pieces kPQ + h kPQ/2..
    auto half_piece = [&](const TileDma& d, int slot, int h, int j) __attribute__((always_inline)) {
      constexpr int kq = kPQ / 2;
      piece(d, slot, j < kq ? h * kq + j : kPQ + h * kq + (j - kq));
    };
    auto list_at = [&](int tt) __attribute__((always_inline)) -> int {
      return __builtin_amdgcn_readfirstlane((int)list[max(min(tt >> 1, nkept - 1), 0)]);
    };
    const uint32_t* tab32 = reinterpret_cast<const uint32_t*>(smem + kTabOff);
    auto tile_at = [&](int tt) __attribute__((always_inline)) -> TileDma {
      if constexpr (kML) {
        const int i = min(tt, kMlTiles - 1);
        return tile_dma_ml(tt, (uint32_t)uniform((int)tab32[2 * i]), (uint32_t)uniform((int)tab32[2 * i + 1]));
      } else {
        return tile_dma(tt, list_at(tt));
      }
    };

    const uint32_t sbase = static_cast<uint32_t>(
        reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)smem));
    constexpr bool kShare = S::kVOff + (R - 1) * TB + 48 * RB < 65536;
    constexpr int NA = kShare ? 1 : 2;
    constexpr int kVImm = kShare ? S::kVOff : 0;
    uint32_t xa[NA][KS];       // [K, V][ks]: key row l32, chunk 2 ks + half
    uint32_t ya[DT][2];        // K^T transposed reads [dt][+0, +8 rows]
    const int trr = tr_row(lane), trc = tr_col(lane);
#pragma unroll
    for (int m = 0; m < NA; ++m) {
      const uint32_t rb = sbase + (m ? S::kVOff : S::kKOff);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xa[m][ks] = rb + l32 * RB + 16 * ((2 * ks + half) ^ dual_swz<D>(l32));
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int p8 = 0; p8 < 2; ++p8) {
        const int r = trr + 8 * p8;
        ya[dt][p8] = sbase + S::kKOff + r * RB + 16 * ((4 * dt + (trc >> 3)) ^ dual_swz<D>(r)) + 2 * (trc & 7);
      }
    const uint32_t lista = sbase + S::kListOff;
    const float c = p.c;

    f32x16 s0, dp0, s1, dp1;   // S^T / dP^T of keys 0-31 and 32-63 (lane = query)
    f32x16 cdt;                // -Delta seeds of the current tile's key source (kSeeded)
    float nl0 = 0.f, nl1 = 0.f;   // -L' of the tile whose V(t,0) / V(t,1) runs
    float nd0 = 0.f, nd1 = 0.f;   // -Delta of the same (!kSeeded)
    u32x4 pd0[2], pd1[2];
    V8 nx[kLA];
    uint32_t blk_raw = 0;
    u32x2 tab_raw = {0u, 0u};
    const uint32_t taba = sbase + kTabOff;
    TileDma dn{};
    // multi-level: the tile's level exponent e (0..3) is its logit bias +log2(2^e) = e
    auto ml_level = [&](int tt) __attribute__((always_inline)) -> int {
      return tt < ntm ? 0 : tt < T12 ? 1 : tt < T124 ? 2 : 3;
    };
    auto set_level = [&](int e) __attribute__((always_inline)) {
      nd0 = opaque(D1);
      nl0 = (float)e - opaque(L1);
    };
    auto ml_level_s = [&](int tt) __attribute__((always_inline)) -> int {   // scalar selects, no branches
      return (int)(tt >= ntm) + (int)(tt >= T12) + (int)(tt >= T124);
    };
    auto set_class = [&](bool pooled) __attribute__((always_inline)) {
      const float dr = pooled ? opaque(D2) : opaque(D1);
      if constexpr (kSeeded) {
#pragma unroll
        for (int r = 0; r < 16; ++r) cdt[r] = dr;
        launder(cdt);   // kept in 16 registers: hipcc would rebuild the broadcast with 16 v_movs per tile
      } else {
        nd0 = dr;
      }
      nl0 = pooled ? -opaque(L2) : -opaque(L1);
    };

    if constexpr (R == 4) {
      // ---- prologue: tiles 0-2 in flight, tile 0 landed, its first operands read -------------
      dn = tile_dma(0, list_at(0));
#pragma unroll
      for (int k = 0; k < kPieces; ++k) piece(dn, 0, k);
      dn = tile_dma(1, list_at(1));
#pragma unroll
      for (int k = 0; k < kPieces; ++k) piece(dn, 1, k);
      dn = tile_dma(2, list_at(2));
#pragma unroll
      for (int k = 0; k < kPieces; ++k) piece(dn, 2, k);
      VB_WAIT_VMCNT(2 * kPieces);
    } else {
      // ---- prologue: both halves of tile 0 in flight, half 0 landed; dn = tile 1 (its halves
      // are issued in tile 0, at gaps kP0.. and after G1) ---------------------------------------
      dn = tile_at(0);
#pragma unroll
      for (int j = 0; j < S::kHalf; ++j) half_piece(dn, 0, 0, j);
#pragma unroll
      for (int j = 0; j < S::kHalf; ++j) half_piece(dn, 0, 1, j);
      dn = tile_at(1);
      VB_WAIT_VMCNT(S::kHalf);
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd128<0>(nx[0], xa[0][0]);
    rd128<kVImm>(nx[1], xa[NA - 1][0]);
    if constexpr (kLA > 2) rd128<0>(nx[2], xa[0][1]);
    if constexpr (kLA > 3) rd128<kVImm>(nx[3], xa[NA - 1][1]);
#if __HIP_DEVICE_COMPILE__
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
#pragma unroll
    for (int q = 0; q < kLA; ++q) launder(nx[q]);
    if constexpr (kML) set_level(ml_level(0));
    else set_class(kPool && 0 >= ntm);

    auto iter = [&](int t, auto U, auto M) __attribute__((always_inline)) {
      constexpr int u = decltype(U)::value % R;   // tile t's ring slot (t mod R)
      constexpr int up = (u + R - 1) % R, un = (u + 1) % R;
      constexpr int mode = decltype(M)::value;
      V8 xop[N];
      s16x4 ylo[N], yhi[N];
      auto gap = [&](auto G) __attribute__((always_inline)) {
        constexpr int g = decltype(G)::value;
        constexpr int sc = S::sec(g), i = g - S::sec0(S::sec(g));
        // R = 2: the half-tile barriers come before the gap's reads (QSched)
        auto half_barrier = [&]() __attribute__((always_inline)) {
#if __HIP_DEVICE_COMPILE__
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
          VB_WAIT_VMCNT(S::kHalf);
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        };
        // ---- MFMA g ----
        if constexpr (sc == 0 || sc == 2) {
          V8& a = g < kLA ? nx[g % kLA] : xop[g];
          if constexpr (g >= kLA || R == 2) wait1<S::wait_n(g)>(a);
          if constexpr (mode != 2) {
            f32x16& s_ = sc == 0 ? s0 : s1;
            f32x16& dp = sc == 0 ? dp0 : dp1;
            constexpr int ks = i >> 1;
            if constexpr (i & 1) {
              if constexpr (ks == 0 && kSeeded) mf_cacc<T>(dp, a, df[0], cdt);
              else if constexpr (ks == 0) mf_zero<T>(dp, a, df[0]);
              else mf_vacc<T>(dp, a, df[ks]);
            } else {
              if constexpr (ks == 0) mf_zero<T>(s_, a, qf[0]);
              else mf_vacc<T>(s_, a, qf[ks]);
            }
          }
        } else {
          wait2<S::wait_n(g)>(ylo[g], yhi[g]);
          constexpr bool run = sc == 1 ? mode != 1 : mode != 2;
          if constexpr (run) {
            constexpr int sb = i / DT, dt = i % DT;
            const V8 a = join8<T>(ylo[g], yhi[g]);
            mf_aacc<T>(dq[dt], a, __builtin_bit_cast(V8, sc == 1 ? pd1[sb] : pd0[sb]));
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (R == 2 && mode != 2 && g == S::kG1) half_barrier();
        if constexpr (R == 2 && mode != 2 && g == S::kG2) {
          half_barrier();
          if constexpr (kML) {
            launder(tab_raw);
            dn = tile_dma_ml(t + 2, (uint32_t)uniform((int)tab_raw[0]), (uint32_t)uniform((int)tab_raw[1]));
          } else {
            launder(blk_raw);
            dn = tile_dma(t + 2, __builtin_amdgcn_readfirstlane((int)blk_raw));   // for tile t+1's batches
          }
        }
        // ---- fillers of gap g ----
        constexpr int m = g + kLA;
        if constexpr (m < N) {
          constexpr int ms = S::sec(m), mi = m - S::sec0(ms);
          if constexpr (ms == 0 || ms == 2) {
            constexpr int kt = ms >> 1;
            rd128<u * TB + kt * 32 * RB + ((mi & 1) ? kVImm : 0)>(xop[m], xa[(mi & 1) && !kShare][mi >> 1]);
          } else {
            constexpr int slot = ms == 1 ? up : u;
            constexpr int kt = ms == 1 ? 1 : 0;
            constexpr int sb = mi / DT, dt = mi % DT;
            constexpr int imm = slot * TB + (32 * kt + 16 * sb) * RB;
            rdtr<imm>(ylo[m], ya[dt][0]);
            rdtr<imm>(yhi[m], ya[dt][1]);
          }
        }
        if constexpr (g == S::kList) {
          if constexpr (kML) rd64(tab_raw, taba + 8 * min(t + 2, kMlTiles - 1));
          else rdu16(blk_raw, lista + 2 * max(min((t + (R == 4 ? 3 : 2)) >> 1, nkept - 1), 0));
        }
        if constexpr (g >= S::kNx && g < S::kNx + kLA) {
          constexpr int q = g - S::kNx;
          rd128<un * TB + ((q & 1) ? kVImm : 0)>(nx[q], xa[(q & 1) && !kShare][q >> 1]);
        }
        // ---- score arithmetic ----
        if constexpr (mode != 2 && g >= S::kV0 && g < S::kV0 + S::kV0n)
          qgap<T, kSeeded, g - S::kV0, S::kV0n>(s0, dp0, pd0, c, nl0, nd0);
        if constexpr (mode != 2 && g >= S::kV1) {
          if constexpr (g == S::kV1) {
            nl1 = nl0;
            nd1 = nd0;
          }
          qgap<T, kSeeded, g - S::kV1, S::kV1n>(s1, dp1, pd1, c, nl1, nd1);
        }
        if constexpr (mode != 1 && g < S::kV1 + S::kV1n - N)
          qgap<T, kSeeded, g + N - S::kV1, S::kV1n>(s1, dp1, pd1, c, nl1, nd1);
        // ---- R = 2: the two half-tile batches of tile t+1 into the slot tile t-1 left ----
        if constexpr (R == 2 && mode != 2 && g >= S::kP0 && g < S::kP0 + S::kHalf) half_piece(dn, up, 0, g - S::kP0);
        if constexpr (R == 2 && mode != 2 && g >= S::kP1 && g < S::kP1 + S::kHalf) half_piece(dn, up, 1, g - S::kP1);
        // ---- R = 4: barrier and the DMA of tile t+3 into the slot tile t-1 left ----
        if constexpr (R == 4 && mode != 2 && g == S::kGb) {
          VB_WAIT_VMCNT(kPieces);   // tile t+1 landed (tile t+2 may be in flight)
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
          launder(blk_raw);
          dn = tile_dma(t + 3, __builtin_amdgcn_readfirstlane((int)blk_raw));
        }
        if constexpr (R == 4 && mode != 2 && g >= S::kDma0 && g < S::kDma0 + kPieces) piece(dn, up, g - S::kDma0);
        if constexpr (g == N - 1) {
#pragma unroll
          for (int q = 0; q < kLA; ++q) launder(nx[q]);
          // tile t+1's seeds and -L': they change once, at the first pooled tile (multi-level: at
          // each level's first tile)
          if constexpr (mode != 2 && kPool) {
            if (t + 1 == ntm) set_class(true);
          }
          if constexpr (mode != 2 && kML) set_level(ml_level_s(t + 1));   // every tile: two VALU
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      if constexpr (mode == 2) {
        for_gaps(gap, std::make_integer_sequence<int, S::kC>{});
#if __HIP_DEVICE_COMPILE__
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
#pragma unroll
        for (int q = S::kC; q < S::kC + kLA; ++q) launder(xop[q]);
        if constexpr (S::kList < S::kC) launder(blk_raw);   // D=64: the list read falls inside the drain
      } else {
        for_gaps(gap, std::make_integer_sequence<int, N>{});
      }
    };

    iter(0, std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    int t = 1;
    for (; t < ntiles; t += 4) {
      iter(t, std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
      iter(t + 1, std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{});
      iter(t + 2, std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{});
      iter(t + 3, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    }
    iter(t, std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{});   // B section of tile t-1
#if __HIP_DEVICE_COMPILE__
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+a"(dq[0]), "+a"(dq[1])::"memory");
    if constexpr (DT == 4) asm volatile("s_nop 0" : "+a"(dq[2]), "+a"(dq[3])::"memory");
#endif
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

template <int D>
static int launch_pipe(const BwdParams& p, bool pooled, bool f16, hipStream_t s) {
  const int BH = p.B * p.H;
  if (pooled) {
    const dim3 grid(p.nbkp * BH * p.psplit);
    if (f16) hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<D, F16, true>), grid, dim3(bwd::kThreads), 0, s, p);
    else hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<D, BF16, true>), grid, dim3(bwd::kThreads), 0, s, p);
    return check_launch("bwd_dkdv_pipe_kernel<pooled>");
  }
  const dim3 grid(p.nbk * BH);
  if (f16) hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<D, F16, false>), grid, dim3(bwd::kThreads), 0, s, p);
  else hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<D, BF16, false>), grid, dim3(bwd::kThreads), 0, s, p);
  return check_launch("bwd_dkdv_pipe_kernel");
}

template <int D, int R>
static int launch_dq(const BwdParams& p, bool pool, bool f16, hipStream_t s) {
  const dim3 grid(p.nbq * p.B * p.H);
  if (pool) {
    if (f16) hipLaunchKernelGGL((bwd_dq_pipe_kernel<D, F16, true, R>), grid, dim3(bwd::kThreads), 0, s, p);
    else hipLaunchKernelGGL((bwd_dq_pipe_kernel<D, BF16, true, R>), grid, dim3(bwd::kThreads), 0, s, p);
  } else {
    if (f16) hipLaunchKernelGGL((bwd_dq_pipe_kernel<D, F16, false, R>), grid, dim3(bwd::kThreads), 0, s, p);
    else hipLaunchKernelGGL((bwd_dq_pipe_kernel<D, BF16, false, R>), grid, dim3(bwd::kThreads), 0, s, p);
  }
  return check_launch("bwd_dq_pipe_kernel");
}

// ring slots: VB_BWD_DQ{64,128}_RING by default, 4 with VB_BWD_SEL_DQ_RING4
int launch_dq_pipe(const BwdParams& p, int D, bool pool, bool f16, hipStream_t s, int sel, int& ran) {
  const bool ring4 = (sel & VB_BWD_SEL_DQ_RING4) || (D == 64 ? VB_BWD_DQ64_RING : VB_BWD_DQ128_RING) != 2;
  ran |= ring4 ? VB_BWD_RAN_DQ_PIPE_RING4 : VB_BWD_RAN_DQ_PIPE_RING2;
  if (D == 64) return ring4 ? launch_dq<64, 4>(p, pool, f16, s) : launch_dq<64, 2>(p, pool, f16, s);
  return ring4 ? launch_dq<128, 4>(p, pool, f16, s) : launch_dq<128, 2>(p, pool, f16, s);
}

int launch_ml_dkdv_pipe(const BwdParams& p, int D, bool f16, hipStream_t s) {
  const dim3 grid(p.nbk * p.B * p.H);
  if (D == 128) {
    if (f16) hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<128, F16, false, true>), grid, dim3(bwd::kThreads), 0, s, p);
    else hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<128, BF16, false, true>), grid, dim3(bwd::kThreads), 0, s, p);
  } else {
    if (f16) hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<64, F16, false, true>), grid, dim3(bwd::kThreads), 0, s, p);
    else hipLaunchKernelGGL((bwd_dkdv_pipe_kernel<64, BF16, false, true>), grid, dim3(bwd::kThreads), 0, s, p);
  }
  return check_launch("bwd_dkdv_pipe_kernel<multi-level>");
}

template <int D>
static int launch_ml_dq(const BwdParams& p, bool f16, hipStream_t s) {
  const dim3 grid(p.nbq * p.B * p.H);
  if (f16) hipLaunchKernelGGL((bwd_dq_pipe_kernel<D, F16, false, 2, true>), grid, dim3(bwd::kThreads), 0, s, p);
  else hipLaunchKernelGGL((bwd_dq_pipe_kernel<D, BF16, false, 2, true>), grid, dim3(bwd::kThreads), 0, s, p);
  return check_launch("bwd_dq_pipe_kernel<multi-level>");
}

int launch_ml_dq_pipe(const BwdParams& p, int D, bool f16, hipStream_t s) {
  return D == 128 ? launch_ml_dq<128>(p, f16, s) : launch_ml_dq<64>(p, f16, s);
}

int launch_dkdv_pipe(const BwdParams& p, int D, bool pooled, bool f16, hipStream_t s) {
  return D == 128 ? launch_pipe<128>(p, pooled, f16, s) : launch_pipe<64>(p, pooled, f16, s);
}

}  // namespace vb

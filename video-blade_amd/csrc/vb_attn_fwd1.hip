// Block-sparse FMHA forward, inference form, one compute wave per SIMD (gfx950 / MI355X).
//
// Same semantics as attn_fwd_kernel's lazy (inference) launches (vb_attn_fwd.hip: the reference's
// block_sparse_attn_func forward as called at cogvideo_blocksparseattn.py:316-320 fused with the
// pooled-KV branch and LSE combine of :367-393), built on a different machine model:
//
//  * a workgroup = one 128-row q-block, 4 compute waves of 32 rows, ONE workgroup per CU, so each
//    compute wave is alone on its SIMD. The D=64 loop is bound by the SIMD's vector-issue port (two
//    v_exp_f32, two adds and one bf16 pack per MFMA), and MFMA and VALU work of two waves sharing
//    a SIMD barely overlap (profiles/r02_mfma_valu_overlap.json: 0.955 of the sum); inside ONE wave
//    the VALU issues in the shadow of the wave's own MFMAs (0.71 of the sum, and a gap holds
//    ~5 single-issue fillers for free, MI355X_MICROARCH.md 'Per-instruction cycle constants').
//  * a three-stage software pipeline per 64-key tile t, so that every MFMA has independent VALU
//    work beside it:
//        region A: P(t-1)[keys 32..63] . V(t-1)   and  S(t+1)[keys 0..31] = K(t+1) . Q^T
//                  beside exp2/sum/pack of S(t)[keys 0..31]
//        region B: S(t+1)[keys 32..63]             and  P(t)[keys 0..31] . V(t)
//                  beside exp2/sum/pack of S(t)[keys 32..63]
//    Every MFMA opens a gap whose fillers are placed by hand (sched_barrier around each gap).
//  * K and V stream through separate R-slot LDS rings by LDS-DMA with R-1 tiles of lead (K(t+R)
//    and V(t+R-1) are issued in iteration t), one barrier per tile. Issues past the last tile use a
//    zero-extent buffer descriptor (no memory access), so every vmcnt is a constant. With kProd the
//    DMA is issued by 4 producer waves (one beside each compute wave; a VMEM-only wave takes no
//    VALU issue slots from its SIMD partner), otherwise by the compute waves in their gaps.
//
// The lazy running max, the overflow check per half-tile and the exp2-domain seeding of the S
// accumulator are attn_fwd_kernel's (see there). A failing check rescales everything still at
// the old max exactly once: O, l, the C seed, S(t) and the part of S(t+1) already computed.
#include <type_traits>
#include <utility>

#include "vb_attn_fwd.hpp"

namespace vb {

#ifndef VB_FWD1_OCC64
#define VB_FWD1_OCC64 1   // workgroups per CU the D=64 kernel is register-budgeted for
#endif
#ifndef VB_FWD1_PROD64
#define VB_FWD1_PROD64 0  // D=64: 4 producer waves issue the LDS-DMA (8-wave workgroups)
#endif
#ifndef VB_FWD1_NODMA
#define VB_FWD1_NODMA 0   // diagnostic builds only: no LDS-DMA after the prologue (stale tiles, wrong results)
#endif
#ifndef VB_FWD1_ABL
#define VB_FWD1_ABL 0     // diagnostic ablations (wrong results): bit 0 no LDS reads in the loop, bit 1 no
                          // v_exp (the adds/packs stay), bit 2 no filler VALU at all
#endif
#ifndef VB_FWD1_RING64
#define VB_FWD1_RING64 6   // K and V ring slots at D=64 (one workgroup per CU; 4 at two)
#endif
#ifndef VB_FWD1_RING128
#define VB_FWD1_RING128 4
#endif

#ifndef VB_DIAG
#define VB_DIAG 0
#endif
#if VB_DIAG
// diagnostic builds only: per-segment s_memtime sums over the compute waves ([0] wait+barrier, [1]
// region A, [2] region B, [3] end of iteration, [4] prologue, [5] epilogue, [8] tiles, [9] WGs)
__device__ unsigned long long g_fwd1_stamp[16];
__device__ __forceinline__ unsigned long long fwd1_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define F1_STAMP(v) const unsigned long long v = fwd1_stamp()
#define F1_ACC(i, d) st_acc[i] += (d)
#else
#define F1_STAMP(v)
#define F1_ACC(i, d)
#endif

namespace fwd1 {

// s_waitcnt lgkmcnt(0) for the asm transposed reads, then every fragment laundered through an
// empty asm so no MFMA that reads one can be scheduled above the wait
template <int N>
__device__ __forceinline__ void lgkm_wait(s16x4 (&lo)[2][N], s16x4 (&hi)[2][N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int d = 0; d < N; ++d) asm volatile("" : "+v"(lo[i][d]), "+v"(hi[i][d]));
}
// MFMAs with operands pinned to register files (D=128: O accumulates in AGPRs and Q is read from
// AGPRs, so the ~330 live registers split over the two files without copies). hipcc's hazard
// recognizer cannot see into these statements: a VALU that reads their results (or writes their
// inputs) right after them needs the s_nop padding of hazard_pad() (only the rare paths do).
// (The AGPR constraints exist only for the device pass: on the host pass "a" names x86's eax,
// which these operands cannot bind, and clang then silently drops the kernels' host stubs.)
template <class T>
__device__ __forceinline__ void mfma_acc_a(f32x16& acc, const typename T::vec8& a, const typename T::vec8& b) {
#if __HIP_DEVICE_COMPILE__
  // s_nop 1: the two wait states a VALU write of a or b (join8's moves) needs before the MFMA
  if constexpr (std::is_same<T, BF16>::value)
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
#endif
}
// d = a . b(AGPR) + c, all VGPR tuples except b
template <class T>
__device__ __forceinline__ f32x16 mfma_bq(const typename T::vec8& a, const typename T::vec8& b, const f32x16& c) {
  f32x16 d = c;
#if __HIP_DEVICE_COMPILE__
  if constexpr (std::is_same<T, BF16>::value)
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "a"(b), "v"(c));
  else
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "a"(b), "v"(c));
#endif
  return d;
}
template <class T>
__device__ __forceinline__ void mfma_bq_acc(f32x16& d, const typename T::vec8& a, const typename T::vec8& b) {
#if __HIP_DEVICE_COMPILE__
  if constexpr (std::is_same<T, BF16>::value)
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
  else
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "a"(b));
#endif
}
// Wait states between an asm MFMA and a VALU touching its registers (16-pass XDL). The registers
// involved are operands of the padding statement, so no access to them can move across it.
__device__ __forceinline__ void hazard_pad(f32x16 (&o)[4], f32x16& x, f32x16& y, f32x16& z) {
#if __HIP_DEVICE_COMPILE__
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4"
               : "+a"(o[0]), "+a"(o[1]), "+a"(o[2]), "+a"(o[3]), "+v"(x), "+v"(y), "+v"(z)::"memory");
#endif
}
// f(integral_constant<int, U>) for U = 0 .. N-1, in order
template <class F, int... Us>
__device__ __forceinline__ void for_phases(F&& f, std::integer_sequence<int, Us...>) {
  (f(std::integral_constant<int, Us>{}), ...);
}
}  // namespace fwd1

template <int D, class T, bool kPool, int kOcc, bool kProd>
__global__ void __launch_bounds__(kProd ? 2 * kThreads : kThreads, kOcc) attn_fwd1_kernel(const FwdParams p) {
  using namespace fwd1;
  using V8 = typename T::vec8;
  constexpr int KS = D / 16;                   // k-steps of S = K.Q^T
  constexpr int DT = D / 32;                   // 32-wide d tiles of O
  constexpr float kLazyBound = std::is_same<T, BF16>::value ? kLazyBoundBF16 : kLazyBoundF16;
  constexpr int kRowB = D * 2;
  constexpr int kMatBytes = kKT * kRowB;       // one 64-key K (or V) tile
  // slots per ring: K(t+1) .. K(t+R-1) and V(t) .. V(t+R-2) are in flight or landed during tile t
  constexpr int kRing = D == 64 ? (kOcc == 1 ? VB_FWD1_RING64 : 4) : VB_FWD1_RING128;
  constexpr int kPeriod = kRing % 2 ? 2 * kRing : kRing;   // slot phase x S-buffer parity
  constexpr int kVBase = kRing * kMatBytes;    // V ring after the K ring
  constexpr int kChunks = kRowB / 16;
  constexpr int kRowsPerInst = 1024 / kRowB;
  constexpr int kPieces = kMatBytes / 1024 / 2;   // LDS-DMA pieces per DMA wave and tile (2 per matrix)
  constexpr int nA = 2 * DT + KS;                 // MFMAs per region (both regions)
  constexpr bool kRegSplit = D == 128;            // O in AGPRs, Q read from AGPRs (asm MFMAs)
  constexpr int epg = 16 / nA;                    // exps per gap: 2 at D=64, 1 at D=128
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * kRing * kMatBytes + kMaxBlocks * 2 + 16];
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + 2 * kRing * kMatBytes);
  int* list_n = reinterpret_cast<int*>(smem + 2 * kRing * kMatBytes + kMaxBlocks * 2);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool producer = kProd && wave >= 4;   // wave-uniform
  const int cw = wave & 3;                    // compute rows / DMA role of this wave
  const int half = lane >> 5;
  const int l32 = lane & 31;

  // ---- work order: attn_fwd_kernel's (heavy text rows first, then XCD-contiguous head ranges) ----
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
  if (q0 >= Lq) return;
  const int nbk = (Lk + kQBlk - 1) / kQBlk;

  // ---- kept key blocks (diagonal first; see attn_fwd_kernel); a producer wave builds the list ----
  if (wave == (kProd ? 4 : 0)) {
    const uint8_t* mrow = (p.use_main && p.mask) ? p.mask + b * p.ms[0] + (int64_t)h * p.ms[1] + (int64_t)qblk * p.ms[2]
                                                 : nullptr;
    int n = 0;
    int dpos = -1;
    if (p.use_main) {
      for (int j0 = 0; j0 < nbk; j0 += 64) {
        const int j = j0 + lane;
        const bool keep = (j < nbk) && (mrow == nullptr || mrow[j] != 0);
        const unsigned long long bal = __ballot(keep);
        if (keep) {
          const int pos = n + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
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
    }
    if (lane == 0) *list_n = n;
  }

  // ---- Q fragment, pre-scaled by scale*log2(e) (B operand of S^T = K.Q^T) -------------------------
  const int qg = q0 + cw * 32 + l32;
  const bool qvalid = qg < Lq;
  int qrow = qvalid ? qg : Lq - 1;
  V8 qf[KS];
  if (!producer) {
    if (p.q_rows) qrow = p.q_rows[qrow];
    const uint8_t* qp = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1]) +
                        (int64_t)qrow * 2 * p.qs[2];
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const V8*>(qp + (16 * s + 8 * half) * 2);
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[s][e] = T::from_f32(T::to_f32(qf[s][e]) * p.c);
    // Q's home: AGPRs at D=128 (read there by the asm MFMAs), VGPRs otherwise
    if constexpr (D == 128) {
#if __HIP_DEVICE_COMPILE__
#pragma unroll
      for (int s = 0; s < KS; ++s) asm volatile("" : "+a"(qf[s]));
#endif
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(qf[s]));
    }
  }
  __syncthreads();
  const int nkept = __builtin_amdgcn_readfirstlane(*list_n);
  int ntm = 2 * nkept;
  if (nkept > 0 && list[nkept - 1] == nbk - 1 && (nbk - 1) * kQBlk + kKT >= Lk) ntm -= 1;
  const int ntp = kPool ? (p.Lkp + kKT - 1) / kKT : 0;
  const int ntiles = ntm + ntp;

  auto blk_of = [&](int tt) __attribute__((always_inline)) -> int {
    return (int)list[min(max(tt, 0) >> 1, kMaxBlocks - 1)];
  };

  // ---- LDS-DMA sources: DMA roles 0-1 fill K tiles, 2-3 V tiles (kPieces 1-KiB pieces each) ------
  const int my_mat = cw >> 1;
  const int sub = cw & 1;
  const uint8_t* kbase = reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1]);
  const uint8_t* vbase = reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1]);
  // Row strides: main and pooled keys share one (the host launches this kernel only then), so a
  // lane's DMA offsets are loop-invariant and a tile's start moves into the descriptor's base.
  const int my_rowb = (int)(2 * (my_mat == 0 ? p.ks[2] : p.vs[2]));
  const int main_bytes = p.use_main ? (int)((int64_t)(Lk - 1) * my_rowb + kRowB) : 0;
  const uint8_t* const my_mbase = my_mat == 0 ? kbase : vbase;
  const uint8_t* my_pbase = my_mbase;
  int pool_bytes = 0;
  if constexpr (kPool) {
    const uint8_t* kpb = reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1]);
    const uint8_t* vpb = reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1]);
    my_pbase = my_mat == 0 ? kpb : vpb;
    pool_bytes = (int)((int64_t)(p.Lkp - 1) * my_rowb + kRowB);
  }
  // the byte offset of every piece's 16-byte chunk within a tile (the K/V images' XOR swizzles
  // applied on the source side, as attn_fwd_kernel does)
  const int row0 = sub * kPieces * kRowsPerInst + lane / kChunks;
  int vo[kPieces];
#pragma unroll
  for (int i = 0; i < kPieces; ++i) {
    const int r = row0 + i * kRowsPerInst;
    const int sl = lane % kChunks;
    int ch;
    if (my_mat == 0) {
      ch = sl ^ ((D == 64) ? ((r >> 1) & 7) : (r & 15));
    } else {
      const int vsw = (D == 64) ? ((r >> 1) & 1) : (r & 3);
      ch = (((sl >> 2) ^ vsw) << 2) | (sl & 3);
    }
    vo[i] = r * my_rowb + 16 * ch;
  }
  // Descriptor of tile tt of this wave's matrix: it starts at the tile's first key and ends at the
  // slice's end, so the rows past a short last tile read as zeros (their scores are masked; zero V
  // rows add nothing); tt >= ntiles gives a zero-extent descriptor (no access, same vmcnt count).
  auto tile_srd = [&](int tt, int blk_raw) __attribute__((always_inline)) -> srd_t {
    const int blk = __builtin_amdgcn_readfirstlane(blk_raw);
    int kstart = blk * kQBlk + (tt & 1) * kKT;
    const uint8_t* base = my_mbase;
    int bytes = main_bytes;
    if (tt >= ntm) {
      kstart = (tt - ntm) * kKT;
      base = my_pbase;
      bytes = pool_bytes;
    }
    const int soff = kstart * my_rowb;
    return srd_t{base + soff, tt >= ntiles ? 0 : bytes - soff};
  };
  auto issue = [&](int tt, int blk_raw, int slot_off) __attribute__((always_inline)) {
    const srd_t sd = tile_srd(tt, blk_raw);
    uint8_t* dst = smem + slot_off + sub * kPieces * 1024;
#pragma unroll
    for (int i = 0; i < kPieces; ++i) dma16(sd, dst + i * 1024, vo[i], 0);
  };
  // the slots DMA-filled in iteration t: K(t+R) into K(t)'s, V(t+R-1) into V(t-1)'s
  auto dma_slot_off = [&](int t) __attribute__((always_inline)) -> int {
    return my_mat == 0 ? (t % kRing) * kMatBytes : kVBase + ((t + kRing - 1) % kRing) * kMatBytes;
  };
  const bool dma_wave = kProd ? producer : true;
  // LDS address of this wave's pieces within a slot of its matrix's ring
  const uint32_t dma_wave_base = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)smem)) +
      (my_mat == 0 ? 0 : kVBase) + sub * kPieces * 1024);

  // ---- prologue DMA: K(0..R-1), V(0..R-2) ---------------------------------------------------------
  if (dma_wave) {
    if (my_mat == 0) {
#pragma unroll
      for (int i = 0; i < kRing; ++i) issue(i, blk_of(i), i * kMatBytes);
      VB_WAIT_VMCNT((kRing - 1) * kPieces);   // K(0) landed
    } else {
#pragma unroll
      for (int i = 0; i < kRing - 1; ++i) issue(i, blk_of(i), kVBase + i * kMatBytes);
    }
  }

  if constexpr (kProd) {
    if (producer) {
      // The producer's whole program: one barrier per tile, matching the compute waves', then the
      // next tile's pieces into the slot that barrier freed.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      int blk_next = blk_of(kRing - my_mat);
      for (int t = 0; t < ntiles; ++t) {
        VB_WAIT_VMCNT((kRing - 2) * kPieces);   // K(t+1) / V(t) landed
        const int blk = blk_next;
        blk_next = blk_of(t + kRing + 1 - my_mat);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (!VB_FWD1_NODMA) issue(t + kRing - my_mat, blk, dma_slot_off(t));
      }
      VB_WAIT_VMCNT(0);
      return;
    }
  }

  // ======================================== compute waves ==========================================
  // valid keys of tile tt (64 unless it is the short last tile of the main or pooled keys)
  auto klen_of = [&](int tt, int blk_raw) __attribute__((always_inline)) -> int {
    const int blk = __builtin_amdgcn_readfirstlane(blk_raw);
    return tt >= ntm ? min(kKT, p.Lkp - (tt - ntm) * kKT) : min(kKT, Lk - (blk * kQBlk + (tt & 1) * kKT));
  };
  const uint32_t smem_u32 = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)smem));
  int k_lane[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) k_lane[ks] = k_off<D>(l32, 2 * ks + half);
  const int vrow = 4 * half + (lane & 15) / 4;
  const int vcol = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
  uint32_t v_lane[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) v_lane[dt] = smem_u32 + kVBase + v_off_bytes<D>(vrow, dt * 32 + vcol);

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = 0.f;                  // running max (exp2 domain) of this lane's query row
  float l = 0.f;                  // running partial row sum (this lane's keys)
  f32x16 cb;                      // C seed of the S MFMAs: bias(tile) - m
  f32x16 s[2][2];                 // S of two tiles [buffer][key half], ping-pong by tile parity
  V8 pp[2];                       // P(t-1) of keys 32..63: the B operands of its last two k-steps
  s16x4 vlo23[2][DT], vhi23[2][DT];   // V(t-1)^T fragments of k-steps 2, 3
  V8 pf01[2];                     // P(t) of keys 0..31
  s16x4 vlo01[2][DT], vhi01[2][DT];   // V(t)^T fragments of k-steps 0, 1
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int e = 0; e < 8; ++e) pp[i][e] = T::from_f32(0.f);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int e = 0; e < 4; ++e) vlo23[i][dt][e] = vhi23[i][dt][e] = 0;
  }

  // O += a . b; S = k . q + c; S += k . q (the register-split forms at D=128)
  auto o_mma = [&](f32x16& acc, const V8& a, const V8& bb) __attribute__((always_inline)) {
    if constexpr (kRegSplit) mfma_acc_a<T>(acc, a, bb);
    else acc = T::mfma32(a, bb, acc);
  };
  auto s_mma0 = [&](const V8& a, const V8& bq, const f32x16& c) __attribute__((always_inline)) -> f32x16 {
    if constexpr (kRegSplit) return mfma_bq<T>(a, bq, c);
    else return T::mfma32(a, bq, c);
  };
  auto s_mma = [&](f32x16& acc, const V8& a, const V8& bq) __attribute__((always_inline)) {
    if constexpr (kRegSplit) mfma_bq_acc<T>(acc, a, bq);
    else acc = T::mfma32(a, bq, acc);
  };
  // P = exp2(S) of one 32-key half packed to the storage type; returns the lane's fp32 sum (the
  // slow path's recomputation; the placed loop below spreads the same arithmetic over the gaps)
  auto exp_pack = [&](const f32x16& x, V8& p0, V8& p1) __attribute__((always_inline)) -> float {
    float e[16];
    float h4[4];
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
    p0 = __builtin_bit_cast(V8, u0);
    p1 = __builtin_bit_cast(V8, u1);
    return (h4[0] + h4[1]) + (h4[2] + h4[3]);
  };
  auto half_max = [&](const f32x16& x) __attribute__((always_inline)) -> float {
    const float a = max3f(max3f(max3f(x[0], x[1], x[2]), x[3], x[4]), x[5], x[6]);
    const float c = max3f(max3f(max3f(x[8], x[9], x[10]), x[11], x[12]), x[13], x[14]);
    return max3f(a, c, fmaxf(x[7], x[15]));
  };
  auto mask_tail = [&](f32x16& x, int kt, int klen) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= klen) x[r] = -INFINITY;
  };
  // raise m by delta (> 0 somewhere): rescale O, l, the seed and the three S registers still at
  // the old max
  auto raise_m = [&](float mt_half, f32x16& r0, f32x16& r1, f32x16& r2) __attribute__((always_inline)) {
    const float delta = fmaxf(max_xor32(mt_half), 0.f);
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
      r0[r] -= delta;
      r1[r] -= delta;
      r2[r] -= delta;
    }
  };

#if VB_DIAG
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  F1_STAMP(p0);
  // ---- prologue: S(0) and the first tile's exact max ---------------------------------------------
  {
    const int b0 = blk_of(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const float bias0 = (kPool && ntm == 0) ? p.pool_bias_l2 : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) cb[r] = bias0;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      V8 kf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[ks] = lds_b128<T>(smem + kt * 32 * kRowB, k_lane[ks]);
      s[0][kt] = s_mma0(kf[0], qf[0], cb);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) s_mma(s[0][kt], kf[ks], qf[ks]);
    }
    if constexpr (kRegSplit) hazard_pad(o, s[0][0], s[0][1], cb);
    const int kl0 = klen_of(0, b0);
    if (kl0 < kKT) {
      asm volatile("");
      mask_tail(s[0][0], 0, kl0);
      mask_tail(s[0][1], 1, kl0);
    }
    const float mt = max_xor32(fmaxf(half_max(s[0][0]), half_max(s[0][1])));
    m = mt;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[0][0][r] -= mt;
      s[0][1][r] -= mt;
      cb[r] -= mt;
    }
    if (kPool && ntm == 1) {   // tile 1 is the first pooled tile: the seed of S(1) carries the bias
#pragma unroll
      for (int r = 0; r < 16; ++r) cb[r] += p.pool_bias_l2;
    }
  }
  F1_STAMP(p1);
  F1_ACC(4, p1 - p0);
  // carried list entries: the block of tile t+1 (its klen) and of this wave's next DMA tile
  int blk_s1 = blk_of(1);
  int blk_dma = kProd ? 0 : blk_of(kRing - my_mat);

  // ---- iteration t, compile-time phase U = t % kPeriod ---------------------------------------------
  // Each MFMA gets a fixed set of fillers, pinned by sched_barrier: the exps of S(t) spread evenly
  // (16 per region), each exp's row-sum add and the bf16 pack of each finished pair one gap later
  // (off the exp's latency), the LDS reads of the operands two or more gaps before their MFMA, and
  // the LDS-DMA pieces in the gaps after the region's reads (the DMA writes LDS; it goes last).
  auto body = [&](int t, auto U) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    constexpr int cur = u & 1, nxt = cur ^ 1;
    constexpr int kSlotK1 = ((u + 1) % kRing) * kMatBytes;
    constexpr int kSlotV = (u % kRing) * kMatBytes;
    F1_STAMP(b0);
    if constexpr (!kProd) VB_WAIT_VMCNT((kRing - 2) * kPieces);   // K(t+1) / V(t) landed
    lgkm_wait(vlo23, vhi23);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    F1_STAMP(b1);
    F1_ACC(0, b1 - b0);
    srd_t sd{nullptr, 0};
    uint32_t dma_dst = 0;
    if constexpr (!kProd) {   // this iteration's DMA descriptor (scalar work, before the MFMA stream)
      sd = tile_srd(t + kRing - my_mat, blk_dma);
      // LDS address of this wave's first piece: an opaque scalar, so each piece's M0 is one s_add
      // of an immediate (hipcc would otherwise keep every slot x piece address in an SGPR)
      dma_dst = dma_wave_base + (my_mat == 0 ? (u % kRing) * kMatBytes : ((u + kRing - 1) % kRing) * kMatBytes);
#if __HIP_DEVICE_COMPILE__   // "s" (an SGPR) is no constraint on the host target
      asm volatile("" : "+s"(dma_dst));
#endif
    }
    // piece i of this iteration's DMA (half of them in each region, one every `step` gaps)
    auto dma_piece = [&](int i) __attribute__((always_inline)) {
#if __HIP_DEVICE_COMPILE__   // an integer-to-LDS-pointer cast has no host meaning (the host pass would drop the stub)
      if (!VB_FWD1_NODMA)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(sd.base), (short)0, sd.bytes, 0x00020000),
            (__attribute__((address_space(3))) void*)(uintptr_t)(dma_dst + i * 1024), 16, vo[i], 0, 0, 0);
#endif
    };
    constexpr int step = 2 * nA / kPieces;
    __builtin_amdgcn_sched_barrier(0);

    V8 kf0[KS], kf1[KS];
    float e[16], h4[4];
    u32x4 pk[2];
    // fillers of gap g for the 16 exps of x: exps of gap g, adds + packs of gap g-1
    auto fill = [&](const f32x16& x, int g) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < epg; ++j) {
        const int r = g * epg + j;
        if (r < 16) e[r] = (VB_FWD1_ABL & 2) ? x[r] : exp2_fast(x[r]);
      }
#pragma unroll
      for (int j = 0; j < epg; ++j) {
        const int r = (g - 1) * epg + j;
        if (r >= 0 && r < 16 && !(VB_FWD1_ABL & 4)) {
          if (r < 4) h4[r] = e[r];
          else h4[r & 3] += e[r];
          if (r & 1) {
            // the pack stays in this gap: hipcc would otherwise sink it past the overflow
            // check (the check's slow path recomputes the packs)
            pk[r >> 3][(r & 7) >> 1] = pack2<T>(e[r - 1], e[r]);
            asm volatile("" : "+v"(pk[r >> 3][(r & 7) >> 1]));
          }
        }
      }
    };
    // the tail of the filler stream after the last gap: adds and packs of the last gap's exps
    auto finish = [&](V8& p0, V8& p1) __attribute__((always_inline)) -> float {
#pragma unroll
      for (int j = 0; j < epg; ++j) {
        const int r = (nA - 1) * epg + j;
        if (VB_FWD1_ABL & 4) {
          if (r < 4) h4[r] = e[r];
          continue;
        }
        if (r >= 4 && r < 16) h4[r & 3] += e[r];
        if (r < 16 && (r & 1)) {
          pk[r >> 3][(r & 7) >> 1] = pack2<T>(e[r - 1], e[r]);
          asm volatile("" : "+v"(pk[r >> 3][(r & 7) >> 1]));
        }
      }
      p0 = __builtin_bit_cast(V8, pk[0]);
      p1 = __builtin_bit_cast(V8, pk[1]);
      return (h4[0] + h4[1]) + (h4[2] + h4[3]);
    };

    // ======== region A: P(t-1).V(t-1) k-steps 2,3 | S(t+1) keys 0..31 ; exps of S(t) keys 0..31 ====
#pragma unroll
    for (int g = 0; g < nA; ++g) {
      if (g < 2 * DT) {
        const int kk = g / DT, dt = g % DT;
        o_mma(o[dt], join8<T>(vlo23[kk][dt], vhi23[kk][dt]), pp[kk]);
      } else {
        const int ks = g - 2 * DT;
        if (ks == 0) s[nxt][0] = s_mma0(kf0[ks], qf[ks], cb);
        else s_mma(s[nxt][0], kf0[ks], qf[ks]);
      }
      __builtin_amdgcn_sched_barrier(0);   // the MFMA opens its gap
      fill(s[cur][0], g);
      // LDS reads, two per gap: K(t+1) keys 0..31, K(t+1) keys 32..63, then V(t) k-steps 0, 1
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int d = 2 * g + j;
        if (VB_FWD1_ABL & 1) {
          if (d < KS) kf0[d] = qf[d];
          else if (d < 2 * KS) kf1[d - KS] = qf[d - KS];
          continue;
        }
        if (d < KS) kf0[d] = lds_b128<T>(smem + kSlotK1, k_lane[d]);
        else if (d < 2 * KS) kf1[d - KS] = lds_b128<T>(smem + kSlotK1 + 32 * kRowB, k_lane[d - KS]);
        else if (d < 2 * KS + 4 * DT) {
          const int v = d - 2 * KS;               // kk = v / (2 DT), dt = (v / 2) % DT, lo/hi = v & 1
          const int kk = v / (2 * DT), dt = (v / 2) % DT;
          const int r0 = (kk >> 1) * 32 + 16 * (kk & 1) + 8 * (v & 1);
          s16x4 x = lds_tr4_asm(v_lane[dt], kSlotV + r0 * kRowB);
          if (v & 1) vhi01[kk][dt] = x;
          else vlo01[kk][dt] = x;
        }
      }
      if constexpr (!kProd)
        if (g % step == 1) dma_piece(g / step);
      __builtin_amdgcn_sched_barrier(0);
    }
    float hs0 = finish(pf01[0], pf01[1]);
    if (!__all(hs0 <= kLazyBound)) {
      asm volatile("");
      if constexpr (kRegSplit) hazard_pad(o, s[nxt][0], s[cur][0], cb);
      raise_m(half_max(s[cur][0]), s[cur][0], s[cur][1], s[nxt][0]);
      hs0 = exp_pack(s[cur][0], pf01[0], pf01[1]);
      if constexpr (kRegSplit) hazard_pad(o, s[nxt][0], s[cur][1], cb);
    }
    l += hs0;
    F1_STAMP(b2);
    F1_ACC(1, b2 - b1);

    // ======== region B: S(t+1) keys 32..63 | P(t).V(t) k-steps 0,1 ; exps of S(t) keys 32..63 ====
    int blk_s2 = 0, blk_dma_next = 0;
#pragma unroll
    for (int g = 0; g < nA; ++g) {
      if (g < KS) {
        if (g == 0) s[nxt][1] = s_mma0(kf1[g], qf[g], cb);
        else s_mma(s[nxt][1], kf1[g], qf[g]);
      } else {
        if (g == KS) lgkm_wait(vlo01, vhi01);   // region A's V reads (no region-B read is older)
        const int kk = (g - KS) / DT, dt = (g - KS) % DT;
        o_mma(o[dt], join8<T>(vlo01[kk][dt], vhi01[kk][dt]), pf01[kk]);
      }
      __builtin_amdgcn_sched_barrier(0);
      fill(s[cur][1], g);
      if constexpr (!kProd)
        if (g % step == 1) dma_piece(kPieces / 2 + g / step);
      if (g == 0) blk_s2 = blk_of(t + 2);
      if (!kProd && g == 1) blk_dma_next = blk_of(t + kRing + 1 - my_mat);
      // V(t) k-steps 2, 3 for the next iteration, after the P.V MFMAs started (two per gap)
      if (g >= KS && !(VB_FWD1_ABL & 1)) {
#pragma unroll
        for (int j = 0; j < 4 * DT / (nA - KS); ++j) {
          const int v = (g - KS) * (4 * DT / (nA - KS)) + j;
          const int kk = v / (2 * DT), dt = (v / 2) % DT;
          const int r0 = ((kk + 2) >> 1) * 32 + 16 * ((kk + 2) & 1) + 8 * (v & 1);
          s16x4 x = lds_tr4_asm(v_lane[dt], kSlotV + r0 * kRowB);
          if (v & 1) vhi23[kk][dt] = x;
          else vlo23[kk][dt] = x;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    float hs1 = finish(pp[0], pp[1]);
    if (!__all(hs1 <= kLazyBound)) {
      asm volatile("");
      if constexpr (kRegSplit) hazard_pad(o, s[nxt][0], s[nxt][1], cb);
      raise_m(half_max(s[cur][1]), s[cur][1], s[nxt][0], s[nxt][1]);
      hs1 = exp_pack(s[cur][1], pp[0], pp[1]);
      if constexpr (kRegSplit) hazard_pad(o, s[nxt][0], s[nxt][1], cb);
    }
    l += hs1;
    F1_STAMP(b3);
    F1_ACC(2, b3 - b2);
    // S(t+1): a short tile's missing keys; the seed of S(t+2) when its key source changes
    const int kl1 = klen_of(t + 1, blk_s1);
    if (kl1 < kKT) {
      asm volatile("");
      if constexpr (kRegSplit) hazard_pad(o, s[nxt][0], s[nxt][1], cb);
      mask_tail(s[nxt][0], 0, kl1);
      mask_tail(s[nxt][1], 1, kl1);
    }
    if constexpr (kPool) {
      if (t + 2 == ntm) {   // tile t+2 is the first pooled tile: seed += the pooled keys' bias
        asm volatile("");
#pragma unroll
        for (int r = 0; r < 16; ++r) cb[r] += p.pool_bias_l2;
        if constexpr (kRegSplit) hazard_pad(o, s[nxt][0], s[nxt][1], cb);
      }
    }
    blk_s1 = blk_s2;
    blk_dma = blk_dma_next;
    F1_STAMP(b4);
    F1_ACC(3, b4 - b3);
  };

  // the body instantiated once per (ring slot, S parity) phase: every LDS offset an immediate
  auto run_phase = [&](int t0, auto U) __attribute__((always_inline)) {
    if (t0 + decltype(U)::value < ntiles) body(t0 + decltype(U)::value, U);
  };
  for (int t0 = 0; t0 < ntiles; t0 += kPeriod)
    for_phases([&](auto U) __attribute__((always_inline)) { run_phase(t0, U); },
               std::make_integer_sequence<int, kPeriod>{});
  // P(n-1) . V(n-1), k-steps 2 and 3
  lgkm_wait(vlo23, vhi23);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o_mma(o[dt], join8<T>(vlo23[kk][dt], vhi23[kk][dt]), pp[kk]);
  if constexpr (kRegSplit) hazard_pad(o, s[0][0], s[0][1], cb);   // the epilogue's VALU reads O
  if constexpr (!kProd) VB_WAIT_VMCNT(0);   // the zero-extent DMAs issued past the last tile retire
  F1_STAMP(e0);

  // ---- epilogue (attn_fwd_kernel's: 16-byte row stores through permlane32_swap) -------------------
  (void)m;   // no LSE output: the running max only drives the rescales
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
#if VB_DIAG
  VB_WAIT_VMCNT(0);
  F1_STAMP(e1);
  F1_ACC(5, e1 - e0);
  if (lane == 0) {
    for (int i = 0; i < 6; ++i) atomicAdd(&g_fwd1_stamp[i], st_acc[i]);
    atomicAdd(&g_fwd1_stamp[8], (unsigned long long)ntiles);
    atomicAdd(&g_fwd1_stamp[9], 1ull);
  }
#endif
}

// Launches the one-wave-per-SIMD kernel when it covers the call (inference: no LSE, no varlen, no
// head_mask_type, K/V contiguous in the reordered order); returns 1 if it did not launch.
template <int D, class T>
static int launch_fwd1_t(const FwdParams& p, bool pool, hipStream_t stream) {
  const dim3 grid(p.nbq * p.B * p.H);
  constexpr int occ = D == 64 ? VB_FWD1_OCC64 : 1;
  constexpr bool prod = D == 64 && VB_FWD1_PROD64;
  const dim3 block(prod ? 2 * kThreads : kThreads);
  if (pool) hipLaunchKernelGGL((attn_fwd1_kernel<D, T, true, occ, prod>), grid, block, 0, stream, p);
  else hipLaunchKernelGGL((attn_fwd1_kernel<D, T, false, occ, prod>), grid, block, 0, stream, p);
  return check_launch("attn_fwd1_kernel");
}

#if VB_DIAG
extern "C" int vb_fwd1_stamps(unsigned long long* host16, int reset) {
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(host16, HIP_SYMBOL(g_fwd1_stamp), sizeof(unsigned long long) * 16);
  if (reset) {
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fwd1_stamp), z, sizeof(z));
  }
  return 0;
}
#endif

int launch_fwd1(const FwdParams& p, int D, int dtype, bool pool, hipStream_t stream, bool& launched) {
  launched = false;
  if (p.lse || p.kv_rows || p.cu_q || p.head_mask_type || p.Lpad || !p.use_main) return 0;
  // main and pooled keys must share their row strides (one set of per-lane DMA offsets)
  if (pool && (p.ks[2] != p.kps[2] || p.vs[2] != p.vps[2])) return 0;
  launched = true;
  if (dtype == VB_DTYPE_BF16) {
    if (D == 64) return launch_fwd1_t<64, BF16>(p, pool, stream);
    if (D == 128) return launch_fwd1_t<128, BF16>(p, pool, stream);
  } else if (dtype == VB_DTYPE_F16) {
    if (D == 64) return launch_fwd1_t<64, F16>(p, pool, stream);
    if (D == 128) return launch_fwd1_t<128, F16>(p, pool, stream);
  }
  launched = false;
  return 0;
}

}  // namespace vb

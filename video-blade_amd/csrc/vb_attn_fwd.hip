// Block-sparse FMHA forward for gfx950 (MI355X), bf16/f16 in, fp32 softmax/accumulate.
//
// Replaces the external block_sparse_attn_func forward (mit-han-lab/Block-Sparse-Attention) as the
// reference calls it (cogvideox/train/special_attentions_local/TrainRelated/cogvideo_blocksparseattn.py:
// 293-324, 106-109) and fuses the pooled-KV branch + LSE combine (:367-393) into the same softmax.
//
// Geometry: one 256-thread workgroup (4 waves) per (b, h, 128-row q-block); each wave owns 32
// query rows. Keys stream through LDS in 64-key tiles (two per kept 128-key mask block, then the
// pooled keys), double-buffered: the next tile's global loads are issued before the current
// tile's MFMAs and written to the other LDS buffer after them (one barrier per tile).
//
// Per wave and tile:
//   S^T (64 keys x 32 q) = K . Q^T       v_mfma_f32_32x32x16: A = K rows (ds_read_b128 of an
//                                        XOR-swizzled image), B = Q fragment held in VGPRs
//   online softmax in the exp2 domain    query on the lane: row max = in-lane fmax over 32
//                                        values + one v_permlane32_swap
//   O^T (D x 32 q) += V^T . P^T          A = V^T via ds_read_b64_tr_b16 (hardware transpose of the
//                                        row-major, granule-swizzled V image), B = P packed from
//                                        the S^T accumulator registers (no LDS round trip)
// Gilbert reorder: q/k/v rows are gathered through q_rows / kv_rows and O/LSE scattered through
// q_rows, so the reference's index_select + cat + reverse (:141-161) cost no pass of their own.
#include <cstdlib>
#include <type_traits>

#include "vb_attn_fwd.hpp"
#include "vb_trace.hpp"

#ifndef VB_ATTN_TRACE
#define VB_ATTN_TRACE 0   // diagnostic builds only (tools/diag/attn_trace.py): per-workgroup timeline
#endif
#if VB_ATTN_TRACE
namespace vb { __device__ TraceBuf g_attn_trace; }
#define VB_ATRACE_START(k) trace_start(g_attn_trace, k, (unsigned)vblk)
#define VB_ATRACE_END() trace_end(g_attn_trace, (unsigned)vblk)
#else
#define VB_ATRACE_START(k)
#define VB_ATRACE_END()
#endif

namespace vb {

#ifndef VB_LAZY_COUNT
#define VB_LAZY_COUNT 0   // diagnostic builds: count lazy-max slow paths (g_vb_stamp[10]) per tile half ([11])
#endif
#ifndef VB_LAZY_NOCHECK
#define VB_LAZY_NOCHECK 0   // diagnostic builds only: no overflow check (timing of the fast path alone)
#endif
#ifndef VB_NODMA
#define VB_NODMA 0   // diagnostic: tiles past the first ring fill are not loaded (stale LDS)
#endif
#if VB_DIAG || VB_LAZY_COUNT
__device__ unsigned long long g_vb_stamp[16];
#endif
#if VB_DIAG
// diagnostic-only cycle stamps (never in the product build): per-segment sums of s_memtime
__device__ __forceinline__ unsigned long long vb_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define VB_STAMP(var) const unsigned long long var = vb_stamp()
#define VB_ACC(i, d) acc_st[i] += (d)
#else
#define VB_STAMP(var)
#define VB_ACC(i, d)
#endif

// LDS of one attention workgroup: the K/V ring, the kept-block list and its count, and (gathered
// K/V) the kv_rows entry ring
template <int D, bool kKvRows>
constexpr int fwd_smem_bytes() {
  return ((D == 64) ? 3 : 2) * 2 * kKT * D * 2 + kMaxBlocks * 2 + 16 + (kKvRows ? 4 * 512 : 0);
}

// Persistent dispatch (vb_attn_args.work_queue; vb_common.hpp): the launch is resident-sized and
// every workgroup pulls work items from per-XCD queue heads. Item v (a "virtual blockIdx" in [0,
// total)) belongs to queue v % 8, in increasing v: the same items, in the same per-XCD order, as one
// workgroup per item dealt round-robin over the XCDs. A workgroup drains its own XCD's queue (w % 8
// shares an XCD, like blockIdx % 8 of the one-per-item grid), then takes the remaining items of the
// other queues, so no XCD idles while another still has work.

// One work item: the (b, h, 128-row q-block) of virtual blockIdx `vblk`. With a work queue, lane 0
// of wave 0 claims the workgroup's next item after the tile loop (`next`), so the claim's round
// trip overlaps the epilogue.
template <int D, class T, bool kPool, bool kKvRows, bool kML, bool kCBias, bool kWQ>
__device__ __forceinline__ void attn_fwd_item(const FwdParams& p, const int vblk, int& next) {
  constexpr int KS = D / 16;                   // k-steps of the QK^T product
  constexpr int DT = D / 32;                   // 32-wide d tiles of the output
  constexpr bool kSplitPV = VB_FWD_SPLIT_PV && D == 64;   // measured: +0.8 % at D=64, -1.4 % at D=128
  // kCBias (inference launches: no LSE output): the S accumulator starts at (bias - m) instead of 0
  // and Q is pre-scaled by scale*log2(e), so every score leaves the MFMA as the exp2 argument itself:
  // no per-score v_fma before the v_exp (the D=64 loop is VALU-issue-bound). The extra rounding of
  // q*scale to 16 bits stays within the stated tolerance; launches that return the LSE for a
  // backward keep the unscaled Q so forward and backward see the same scores.
  constexpr bool kLazy = kCBias && VB_FWD_LAZY && !VB_MFMA_ROWSUM && !VB_DIAG;
  // s_setprio around the MFMA chains of the lazy (inference) loop: with two waves per SIMD (D=128)
  // the wave in its MFMA phase keeps the matrix pipe fed while the other runs its softmax VALU
  // (Wan +4 %); the LSE-returning loop and the 3-wave D=64 kernel measured slower with it
  constexpr int kPrio = !kLazy ? 0 : D == 64 ? VB_FWD_PRIO64 : VB_FWD_PRIO128;
  constexpr float kLazyBound = std::is_same<T, BF16>::value ? kLazyBoundBF16 : kLazyBoundF16;
  constexpr int kRowB = D * 2;                 // bytes per key row
  constexpr int kMatBytes = kKT * kRowB;       // one 64-key K (or V) tile
  constexpr int kBufBytes = 2 * kMatBytes;     // K image then V image
  constexpr int kBufs = (D == 64) ? 3 : 2;     // LDS ring: tile t read, t+1 (and t+2) in flight
  constexpr int kChunks = kRowB / 16;          // 16-byte chunks per row
  constexpr int kRowsPerInst = 1024 / kRowB;   // rows one 1-KiB LDS-DMA wave-instruction fills
  constexpr int kInstPerMat = kMatBytes / 1024;
  constexpr int kInstPerWave = 2 * kInstPerMat / 4;
  // declared here, not passed in from the kernel: hipcc's waitcnt pass then still sees which LDS
  // bytes each LDS-DMA writes and each read reads (through a pointer parameter it puts a vmcnt wait,
  // draining the ring, in front of every LDS read of the loop)
  __shared__ __attribute__((aligned(16))) uint8_t smem[fwd_smem_bytes<D, kKvRows>()];
  static_assert(fwd_smem_bytes<D, kKvRows>() == kBufs * kBufBytes + kMaxBlocks * 2 + 16 + (kKvRows ? 4 * 512 : 0), "LDS layout");
  static_assert(!(kML && (kPool || kKvRows)), "multi-level mode reads the KV pyramids only");
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + kBufs * kBufBytes);
  int* list_n = reinterpret_cast<int*>(smem + kBufs * kBufBytes + kMaxBlocks * 2);

  // Persistent launches (kWQ) launder the thread id per item: otherwise the item loop hoists the
  // lane-derived addresses (DMA chunks, LDS fragment bases) out of it and spills them across it.
  // The mask keeps its range known (0..255), so hipcc's waitcnt pass still separates a ring slot's
  // LDS-DMA from the reads of another slot.
  int tid = threadIdx.x;
  if constexpr (kWQ) {
    asm volatile("" : "+v"(tid));
    tid &= kThreads - 1;
  }
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int half = lane >> 5;
  const int l32 = lane & 31;

  // Work order (placement only affects speed, never results). Workgroups are dealt round-robin
  // over the 8 XCDs (blockIdx % 8 share one XCD and its 4 MiB L2).
  //  phase 1: the `heavy_rows` last q-block rows of every head (CogVideoX's dense text rows, the
  //           longest workgroups) go first, spread over all XCDs;
  //  phase 2: every XCD takes a contiguous, head-major range of the remaining (head, q-block)
  //           work, so the pooled K/V and the kept K/V blocks of the one or two heads an XCD is
  //           working on are re-read from its own L2 instead of the Infinity Cache / HBM.
  VB_ATRACE_START(0);
  const int BH = p.B * p.H;
  const int hr = min(p.heavy_rows, p.nbq);
  const int n_heavy = hr * BH;
  int qblk, bh;
  if (vblk < n_heavy) {
    qblk = p.nbq - 1 - vblk / BH;
    bh = vblk % BH;
  } else {
    const int rows_left = p.nbq - hr;
    int lin = xcd_linear(vblk - n_heavy, rows_left * BH);
    if (p.q_order) lin = __builtin_amdgcn_readfirstlane(p.q_order[lin]);   // longest first (attn_order_kernel)
    bh = lin / rows_left;
    qblk = rows_left - 1 - lin % rows_left;
  }
  const int b = bh / p.H, h = bh % p.H;

  int Lq = p.Lq, Lk = p.Lk;
  int64_t qrow0 = 0, krow0 = 0;
  if (p.cu_q) {
    qrow0 = p.cu_q[b];
    Lq = p.cu_q[b + 1] - p.cu_q[b];
    krow0 = p.cu_k[b];
    Lk = p.cu_k[b + 1] - p.cu_k[b];
  }
  const int q0 = qblk * kQBlk;
  if (q0 >= Lq) return;
  const int nbk = (Lk + kQBlk - 1) / kQBlk;

  // ---- which key blocks this q-block keeps ------------------------------------------------------
  const uint8_t* mrow = nullptr;
  bool dense = true;
  bool nan_head = false;
  if (p.use_main) {
    const uint8_t* mh = head_mask_base(p.mask, p.ms, p.head_mask_type, p.H, b, h, nan_head, p.hm_mode);
    if (mh) {
      dense = false;
      mrow = mh + (int64_t)qblk * p.ms[2];
    }
  }
  if (kML) {
    // multi-level: per-level lists of key blocks (levels 1, 2, 4, 8, in that order), built in two
    // passes over the mask row (counts, then positions) so they share the one kMaxBlocks array
    if (tid < 64) {
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
      if (lane < 4) list_n[lane] = cnt[0] * (lane == 0) + cnt[1] * (lane == 1) + cnt[2] * (lane == 2) + cnt[3] * (lane == 3);
    }
  } else if (tid < 64) {
    int n = 0;
    int dpos = -1;   // list position of the diagonal block (key block qblk), if kept
    if (p.use_main) {
      for (int j0 = 0; j0 < nbk; j0 += 64) {
        const int j = j0 + lane;
        const bool keep = (j < nbk) && (dense || mrow[j] != 0);
        const unsigned long long bal = __ballot(keep);
        if (keep) {
          const int pos = n + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
          list[pos] = (uint16_t)j;
          if (j == qblk) dpos = pos;
        }
        n += __popcll(bal);
      }
      // Diagonal block first: in the Gilbert order a q-block's own key block usually holds its
      // largest scores, so the running max is set once on the first tile (fewer rescales; the
      // lazy-max launches rarely leave their fast path). Placement only: same sum, other order.
      // The last key block keeps its place (a half-empty tail tile must stay the last tile).
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

  // ---- Q fragment (B operand of S^T = K.Q^T): row l32 of this wave, d = 16s + 8*half + j --------
  const int qg = q0 + wave * 32 + l32;               // reordered query position
  const bool qvalid = qg < Lq;
  int qrow = qvalid ? qg : Lq - 1;
  if (p.q_rows) qrow = p.q_rows[qrow];
  const uint8_t* qbase = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + qrow0 * p.qs[2]);
  typename T::vec8 qf[KS];
  auto load_q = [&]() __attribute__((always_inline)) {
    const uint8_t* qp = qbase + (int64_t)qrow * 2 * p.qs[2];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      qf[s] = *reinterpret_cast<const typename T::vec8*>(qp + (16 * s + 8 * half) * 2);
    if constexpr (kCBias) {
      // scores in the exp2 domain straight out of the MFMA: Q carries the softmax scale * log2(e)
      // (one extra rounding of q to the storage type; the stated tolerance covers it)
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int e = 0; e < 8; ++e) qf[s][e] = T::from_f32(T::to_f32(qf[s][e]) * p.c);
    }
    // Launder the Q fragment through an empty asm: the loop's MFMAs then depend on the asm, not
    // on the global loads, so hipcc's waitcnt pass does not count them against the DMA ring.
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(qf[s]));
  };
  // kQLate: the Q fragment is loaded after the ring's first DMAs are issued (below), so its round
  // trip and theirs overlap; only the q_rows entry (issued above) and the mask row precede the
  // barrier. Otherwise Q is loaded first and retired before the DMA ring starts.
  constexpr bool kQLate = D == 64 ? VB_FWD_QLATE64 : (kLazy && !kKvRows) ? VB_FWD_QLATE128_LAZY : VB_FWD_QLATE128;
  if constexpr (kQLate) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // wave 0's list writes
    __builtin_amdgcn_s_barrier();                           // kept-block list visible
    asm volatile("" ::: "memory");
  } else {
    load_q();
    __syncthreads();
  }
  const int nkept = __builtin_amdgcn_readfirstlane(*list_n);
  // main tiles: two 64-key halves per kept block, minus an empty second half of the last block
  int ntm = 2 * nkept;
  if (nkept > 0 && list[nkept - 1] == nbk - 1 && (nbk - 1) * kQBlk + kKT >= Lk && !(kML && p.ref_tail)) ntm -= 1;
  const int ntp = kPool ? (p.Lkp + kKT - 1) / kKT : 0;
  // multi-level tiles (64 pyramid rows, one level each): level 1 as above, one tile per level-2
  // block, two level-4 blocks and four level-8 blocks per tile (a short last tile is masked)
  int n2 = 0, n4 = 0, n8 = 0, T12 = 0, T124 = 0;
  if (kML) {
    n2 = __builtin_amdgcn_readfirstlane(list_n[1]);
    n4 = __builtin_amdgcn_readfirstlane(list_n[2]);
    n8 = __builtin_amdgcn_readfirstlane(list_n[3]);
    T12 = ntm + n2;
    T124 = T12 + (n4 + 1) / 2;
  }
  const int ntiles = kML ? T124 + (n8 + 3) / 4 : ntm + ntp;

  const uint8_t* kbase = reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1] + krow0 * p.ks[2]);
  const uint8_t* vbase = reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1] + krow0 * p.vs[2]);
  const uint8_t* kpbase = nullptr;
  const uint8_t* vpbase = nullptr;
  if (kPool) {
    kpbase = reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1]);
    vpbase = reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1]);
  }

  // where tile t's keys come from; `blk_raw` = list[t >> 1] (read ahead by the caller)
  auto tile_src = [&](int t, int blk_raw) __attribute__((always_inline)) -> TileSrc {
    TileSrc s;
    if (t < ntm) {
      const int blk = __builtin_amdgcn_readfirstlane(blk_raw);  // provably wave-uniform
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

  // multi-level: pyramid rows of tile t's two quarters for this wave's half (packed block ids `raw`
  // from ml_list_at, read one tile ahead like list_at)
  const int off4 = p.Lpad + p.Lpad / 2, off8 = off4 + p.Lpad / 4;
  const int my_half = (wave & 1) * 32;
  auto ml_tile_src = [&](int t, int raw) __attribute__((always_inline)) -> MlTileSrc {
    MlTileSrc s;
    const int a = __builtin_amdgcn_readfirstlane(raw & 0xFFFF);
    const int c = __builtin_amdgcn_readfirstlane(raw >> 16);
    if (t < ntm) {
      const int kstart = a * kQBlk + (t & 1) * kKT;
      s.srcA = kstart + my_half;
      s.klen = p.ref_tail ? kKT : min(kKT, Lk - kstart);
      s.lvl = 0;
    } else if (t < T12) {
      s.srcA = p.Lpad + a * 64 + my_half;
      s.klen = kKT;
      s.lvl = 1;
    } else if (t < T124) {
      s.srcA = off4 + a * 32;
      s.klen = min(kKT, (n4 - 2 * (t - T12)) * 32);
      s.lvl = 2;
    } else {
      s.srcA = off8 + a * 16;
      s.klen = min(kKT, (n8 - 4 * (t - T124)) * 16);
      s.lvl = 3;
    }
    s.srcB = (t >= T124) ? off8 + c * 16 : s.srcA + 16;
    return s;
  };
  auto ml_list_at = [&](int t) __attribute__((always_inline)) -> int {
    int e0, e1;
    if (t < ntm) {
      e0 = e1 = t >> 1;
    } else if (t < T12) {
      e0 = e1 = nkept + (t - ntm);
    } else if (t < T124) {
      e0 = e1 = nkept + n2 + min(2 * (t - T12) + (wave & 1), n4 - 1);
    } else {
      const int e = 4 * (t - T124) + 2 * (wave & 1);
      e0 = nkept + n2 + n4 + min(e, n8 - 1);
      e1 = nkept + n2 + n4 + min(e + 1, n8 - 1);
    }
    e0 = min(max(e0, 0), kMaxBlocks - 1);
    e1 = min(max(e1, 0), kMaxBlocks - 1);
    return (int)list[e0] | ((int)list[e1] << 16);
  };

  // Tile t -> LDS ring slot t % kBufs by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
  // wave-instruction, written linearly). The images' XOR swizzles (k_off / v_off_bytes) are
  // applied to each lane's SOURCE chunk instead: LDS slot `sl` of row r holds the chunk that
  // k_off / v_off_bytes would have placed there. Waves 0-1 (D=64) fill K, waves 2-3 fill V.
  // every wave fills ONE matrix: waves 0-1 -> K, waves 2-3 -> V (kInstPerWave*2 == kInstPerMat)
  static_assert(2 * kInstPerWave == kInstPerMat, "DMA split assumes two waves per matrix");
  const int my_mat = wave >> 1;
  const uint8_t* my_base = my_mat == 0 ? kbase : vbase;
  const int64_t my_stride = 2 * (my_mat == 0 ? p.ks[2] : p.vs[2]);
  const uint8_t* my_pbase = my_mat == 0 ? kpbase : vpbase;
  const int64_t my_pstride = kPool ? 2 * (my_mat == 0 ? p.kps[2] : p.vps[2]) : 0;
  // source chunk of every DMA lane (fixed: the image row of lane L is a function of L only)
  int my_chunk[kInstPerWave];
  int my_row[kInstPerWave];
#pragma unroll
  for (int i = 0; i < kInstPerWave; ++i) {
    const int mi = (wave & 1) * kInstPerWave + i;
    const int r = mi * kRowsPerInst + lane / kChunks;
    const int sl = lane % kChunks;
    my_row[i] = r;
    if (my_mat == 0) {
      my_chunk[i] = sl ^ ((D == 64) ? ((r >> 1) & 7) : (r & 15));
    } else {
      const int vsw = (D == 64) ? ((r >> 1) & 1) : (r & 3);
      my_chunk[i] = (((sl >> 2) ^ vsw) << 2) | (sl & 3);
    }
  }
  // Buffer descriptors of this wave's matrix for the (b,h) slice (main and pooled keys): the DMA
  // then needs no 64-bit per-lane address math — the lane's fixed part (row within the tile,
  // source chunk) is a precomputed 32-bit voffset and the tile's first key a scalar soffset.
  // The host guarantees every slice spans < 2^31 bytes.
  const int my_rowb = (int)my_stride;
  const int my_prowb = (int)my_pstride;
  const int src_rows = kML ? 15 * (p.Lpad / 8) : Lk;   // pyramid rows in multi-level mode
  const srd_t my_rsrc = make_srd(my_base, p.use_main ? (int)((int64_t)(src_rows - 1) * my_stride + kRowB) : 0);
  const srd_t my_prsrc = make_srd(kPool ? my_pbase : my_base, kPool ? (int)((int64_t)(p.Lkp - 1) * my_pstride + kRowB) : 0);
  // multi-level: per-lane voffsets, rows relative to the instruction's 16-row quarter (its start
  // is the soffset). Otherwise only the swizzled chunk is kept per instruction: instruction i's
  // row is my_row0 + i*kRowsPerInst, so its voffset is my_row0*rowb + chunk (one VALU per tile and
  // instruction) and the i*kRowsPerInst*rowb part goes to the scalar soffset. Fewer live VGPRs
  // than one offset per instruction and key source (a spilled one stalled the D=128 DMA ring).
  int my_voff[kInstPerWave];
  int my_rc[kInstPerWave];
  const int my_row0 = my_row[0];
#pragma unroll
  for (int i = 0; i < kInstPerWave; ++i) {
    my_rc[i] = my_chunk[i] * 16;
    if constexpr (kML) my_voff[i] = (my_row[i] & 15) * my_rowb + my_chunk[i] * 16;
  }
  auto ml_issue = [&](const MlTileSrc src, int slot) __attribute__((always_inline)) {
    uint8_t* dst = smem + slot * kBufBytes + my_mat * kMatBytes + (wave & 1) * kInstPerWave * 1024;
    const int soffA = __builtin_amdgcn_readfirstlane(src.srcA * my_rowb);
    const int soffB = __builtin_amdgcn_readfirstlane(src.srcB * my_rowb);
#pragma unroll
    for (int i = 0; i < kInstPerWave; ++i)
      if constexpr (kWQ && VB_FWD_DMA_UNSCOPED) dma16_unscoped(my_rsrc, dst + i * 1024, my_voff[i], (i * kRowsPerInst >= 16) ? soffB : soffA);
      else dma16(my_rsrc, dst + i * 1024, my_voff[i], (i * kRowsPerInst >= 16) ? soffB : soffA);
  };
  // Gathered K/V rows (kv_rows: reordered key -> caller row; the module's path on the caller's own
  // k/v). Per tile every wave DMAs the kv_rows entries of its own 32 rows into a 4-slot LDS ring
  // one DMA stage ahead of the rows themselves (lane 32 lanes, entry j*kIPW + i = the row of DMA
  // instruction i for lanes with row j), reads its kIPW entries back with one or two ds_read_b128
  // and issues the row DMAs with per-lane voffsets row * stride + chunk (v_mad_u32_u24). Every
  // body issues one offset DMA and kIPW row DMAs, past the last tile too, so the vmcnt counts are
  // constants (see the body).
  const int gather_key = ((wave & 1) * kInstPerWave + (lane % kInstPerWave)) * kRowsPerInst + lane / kInstPerWave;
  const srd_t rows_srd = make_srd(kKvRows ? p.kv_rows : nullptr, kKvRows ? Lk * 4 : 0);
  uint8_t* const ibase = smem + kBufs * kBufBytes + kMaxBlocks * 2 + 16 + wave * 128;   // [4][4 waves][32]
  auto issue_idx = [&](int t, int blk_raw) __attribute__((always_inline)) {
    int voff = 0;   // pooled tiles and tiles past the end: a harmless entry
    if (t < ntm) {
      const int kstart = __builtin_amdgcn_readfirstlane(blk_raw) * kQBlk + (t & 1) * kKT;
      voff = 4 * (kstart + min(gather_key, min(kKT, Lk - kstart) - 1));
    }
    if (lane < 32) {
      uint8_t* dst = ibase + (t & 3) * 512;
      if constexpr (kWQ && VB_FWD_DMA_UNSCOPED) {   // as dma16_unscoped
        uint32_t a = __builtin_amdgcn_readfirstlane(
            static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)dst)));
        asm("" : "+s"(a));
        dst = (uint8_t*)(__attribute__((address_space(3))) uint8_t*)(uintptr_t)a;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(rows_srd.base), (short)0, rows_srd.bytes, 0x00020000),
          (__attribute__((address_space(3))) void*)dst, 4, voff, 0, 0, 0);
    }
  };
  auto issue = [&](const TileSrc src, int slot, int t = 0) __attribute__((always_inline)) {
    uint8_t* dst = smem + slot * kBufBytes + my_mat * kMatBytes + (wave & 1) * kInstPerWave * 1024;
    // this wave's i-th 1 KiB piece of the tile
    auto piece = [&](int i, srd_t sd, int voff, int soff) __attribute__((always_inline)) {
      if constexpr (kWQ && VB_FWD_DMA_UNSCOPED) dma16_unscoped(sd, dst + i * 1024, voff, soff);
      else dma16(sd, dst + i * 1024, voff, soff);
    };
    const bool pooled = kPool && src.pooled;
    if (kKvRows && !pooled) {
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      int o[kInstPerWave];
      const uint8_t* ib = ibase + (t & 3) * 512 + 4 * kInstPerWave * (lane / kChunks);
#pragma unroll
      for (int c = 0; c < kInstPerWave; c += 4) {
        const i32x4 w = *reinterpret_cast<const i32x4*>(ib + 4 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[c + e] = w[e];
      }
#pragma unroll
      for (int i = 0; i < kInstPerWave; ++i) {
        int voff;   // row * stride + chunk: rows < 2^24 and strides < 2^24 bytes (host-checked)
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(voff) : "v"(o[i]), "s"(my_rowb), "v"(my_chunk[i] * 16));
        piece(i, my_rsrc, voff, 0);
      }
      return;
    }
    const int rowb = pooled ? my_prowb : my_rowb;
    const int soff = __builtin_amdgcn_readfirstlane(src.kstart * rowb);
    if (src.klen == kKT) {
      // 24-bit multiply (full rate; v_mul_lo_u32 is a quarter-rate op on every tile): the row is
      // < 64 and the host rejects row strides of 2^24 bytes or more
      const int vb0 = (int)__umul24((unsigned)my_row0, (unsigned)rowb);
#pragma unroll
      for (int i = 0; i < kInstPerWave; ++i)
        piece(i, pooled ? my_prsrc : my_rsrc, vb0 + my_rc[i], __builtin_amdgcn_readfirstlane(soff + i * kRowsPerInst * rowb));
    } else {   // tail tile: clamp rows to the last valid key (replicated rows are masked later)
#pragma unroll
      for (int i = 0; i < kInstPerWave; ++i) {
        const int r = min(my_row0 + i * kRowsPerInst, src.klen - 1);
        piece(i, pooled ? my_prsrc : my_rsrc, r * rowb + my_rc[i], soff);
      }
    }
  };

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = kCBias ? 0.f : -INFINITY;  // running max (exp2 domain) of this lane's query row
  float l = 0.f;        // running partial row sum (this half's keys)
  // kCBias: cb = cur_bias - m in every register (the first QK^T MFMA's C operand); `first` forces
  // the first tile to set m from its own maximum
  f32x16 cb;
#pragma unroll
  for (int r = 0; r < 16; ++r) cb[r] = 0.f;
  int cur_bias_bits = 0;   // bit pattern of the bias folded into cb (0.0f)
  bool first = true;
#if VB_MFMA_ROWSUM
  // Row sums on the matrix core (D=64 is VALU-bound): lsum += ones . P^T, every register of the
  // accumulator = the lane's full row sum of the bf16 P that also feeds O (no VALU adds).
  f32x16 lsum;
#pragma unroll
  for (int r = 0; r < 16; ++r) lsum[r] = 0.f;
  typename T::vec8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = T::from_f32(1.0f);
#endif

  const int vrow = 4 * half + (lane & 15) / 4;
  const int vcol = 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
#if VB_DIAG
  unsigned long long acc_st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif

  // Loop-invariant per-lane LDS addresses: the images' XOR swizzles depend only on the lane's own
  // row bits (K: row l32 [+32 kt]; V: row vrow [+16 k + 8]), so every K/V fragment read of every
  // tile and ring slot is one of these bases plus a compile-time immediate offset.
  int k_lane[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) k_lane[ks] = k_off<D>(l32, 2 * ks + half);
  uint32_t v_lane[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
    v_lane[dt] = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
                     (__attribute__((address_space(3))) const uint8_t*)smem)) +
                 v_off_bytes<D>(vrow, dt * 32 + vcol);

  // One 64-key tile in ring slot U: S^T = K.Q^T, online softmax, O^T += V^T.P^T.
  // bias_bits: the tile's logit bias (exp2 domain) as a bit pattern, chosen by the caller with scalar
  // selects (a float select would be a v_cndmask + v_readfirstlane on every tile)
  auto tile_step = [&](auto U, int bias_bits, int klen) __attribute__((always_inline)) {
    constexpr int kSlot = decltype(U)::value;
    const uint8_t* kl = smem + kSlot * kBufBytes;
    const float bias = __int_as_float(bias_bits);
    f32x16 s[2];
    if constexpr (kCBias) {
      // wave-uniform; only where the tile source changes (pooled, levels). Compared as bit patterns
      // in SGPRs (a scalar compare; a float compare would run on the VALU every tile)
      if (bias_bits != cur_bias_bits) {
        asm volatile("");
        const float db = bias - __int_as_float(cur_bias_bits);
#pragma unroll
        for (int r = 0; r < 16; ++r) cb[r] += db;
        cur_bias_bits = bias_bits;
      }
    }
    // V^T fragments (ds_read_b64_tr_b16) for the first VPRE k-steps, issued before the softmax
    // VALU so they land while it runs; the rest are fetched one k-step ahead inside the PV loop.
    constexpr int VPRE = (D == 64 && !VB_MFMA_ROWSUM) ? (kKvRows ? VB_VPRE64_ROWS : VB_VPRE64) : 2;
    s16x4 vlo[4][DT], vhi[4][DT];
    auto read_v = [&](int kk) __attribute__((always_inline)) {
      const int row0 = (kk >> 1) * 32 + 16 * (kk & 1);   // + vrow (in v_lane)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        vlo[kk][dt] = lds_tr4_asm(v_lane[dt], kSlot * kBufBytes + kMatBytes + row0 * kRowB);
        vhi[kk][dt] = lds_tr4_asm(v_lane[dt], kSlot * kBufBytes + kMatBytes + (row0 + 8) * kRowB);
      }
    };
    auto wait_v = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(vlo[kk][dt]), "+v"(vhi[kk][dt]));
    };
    auto mask_tail = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= klen) s[kt][r] = -INFINITY;
    };
    // row max of one 32-key half (this lane's 16 values): 7 v_max3 + 1 v_max
    auto half_max = [&](const f32x16& x) __attribute__((always_inline)) -> float {
      const float a = max3f(max3f(max3f(x[0], x[1], x[2]), x[3], x[4]), x[5], x[6]);
      const float c = max3f(max3f(max3f(x[8], x[9], x[10]), x[11], x[12]), x[13], x[14]);
      return max3f(a, c, fmaxf(x[7], x[15]));
    };
    auto compute_s = [&]() __attribute__((always_inline)) {
      if constexpr (kPrio & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        typename T::vec8 kf[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kf[ks] = lds_b128<T>(kl + kt * 32 * kRowB, k_lane[ks]);
        if constexpr (kCBias) {
          s[kt] = T::mfma32(kf[0], qf[0], cb);
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[kt][r] = 0.f;
          s[kt] = T::mfma32(kf[0], qf[0], s[kt]);
        }
#pragma unroll
        for (int ks = 1; ks < KS; ++ks) s[kt] = T::mfma32(kf[ks], qf[ks], s[kt]);
      }
      if constexpr (kPrio & 1) __builtin_amdgcn_s_setprio(0);
    };
    // P = exp2(S) of one half packed to the storage type (the PV operands of k-steps 2kt, 2kt+1)
    // WITHOUT overwriting S; returns the lane's fp32 sum (four independent chains)
    auto exp_pack = [&](const f32x16& x, typename T::vec8& p0, typename T::vec8& p1) __attribute__((always_inline)) -> float {
      float e[16];
      float h4[4];
      if constexpr (kPrio & 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        e[r] = exp2_fast(x[r]);
        h4[r & 3] = r < 4 ? e[r] : h4[r & 3] + e[r];   // chains start at their first value (no 0 + e)
      }
      u32x4 u0, u1;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        u0[w] = pack2<T>(e[2 * w], e[2 * w + 1]);
        u1[w] = pack2<T>(e[8 + 2 * w], e[8 + 2 * w + 1]);
      }
      p0 = __builtin_bit_cast(typename T::vec8, u0);
      p1 = __builtin_bit_cast(typename T::vec8, u1);
      if constexpr (kPrio & 4) __builtin_amdgcn_s_setprio(0);
      return (h4[0] + h4[1]) + (h4[2] + h4[3]);
    };
    auto pv_pk = [&](int kk, const typename T::vec8& pf) __attribute__((always_inline)) {
      wait_v(kk);
      if (kk + VPRE < 4) read_v(kk + VPRE);
      if constexpr (kPrio & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] = T::mfma32(join8<T>(vlo[kk][dt], vhi[kk][dt]), pf, o[dt]);
      if constexpr (kPrio & 2) __builtin_amdgcn_s_setprio(0);
    };
    // raise m by the rows' max mt of S (if > 0), rescaling O, l, the C seed and the S halves >= kt0
    // (a half whose P is already in O is dead: touching it would keep it live)
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
        if (kt0 == 0) s[0][r] -= delta;
        s[1][r] -= delta;
      }
    };
    if constexpr (kLazy) {
      // Lazy running max (inference launches). The first tile takes its exact row max; after that
      // no per-tile max is computed: P = exp2(S - m) uses the standing m, and the row sum of each
      // half-tile (>= each of its P) is checked against kLazyBound. A passing check bounds every P,
      // and so O and l, far from overflow. P is packed into separate registers, so S survives the
      // exp: a failing check (rare, wave-uniform) raises m to the rows' max of that S, rescales O
      // and l, and redoes the exp. m never exceeds the true running max, so l >= 1 after the first
      // tile, and P's bf16 rounding is relative: the result equals the exact-max form up to
      // rounding.
      compute_s();
#pragma unroll
      for (int kk = 0; kk < VPRE; ++kk) read_v(kk);
      if (klen < kKT) {
        asm volatile("");
        mask_tail(0);
        mask_tail(1);
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
      typename T::vec8 pf[4];
      if constexpr (kSplitPV) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          float hs = exp_pack(s[kt], pf[2 * kt], pf[2 * kt + 1]);
          if (!VB_LAZY_NOCHECK && !__all(hs <= kLazyBound)) {
            asm volatile("");
#if VB_LAZY_COUNT
            if (lane == 0) atomicAdd(&g_vb_stamp[10], 1ull);
#endif
            // O and l already hold the first half's P when kt = 1: they are rescaled with the rest
            if (kt == 0) raise_m(half_max(s[0]), std::integral_constant<int, 0>{});
            else raise_m(half_max(s[1]), std::integral_constant<int, 1>{});
            hs = exp_pack(s[kt], pf[2 * kt], pf[2 * kt + 1]);
          }
          l += hs;
          pv_pk(2 * kt, pf[2 * kt]);
          pv_pk(2 * kt + 1, pf[2 * kt + 1]);
        }
      } else {
        float h0 = exp_pack(s[0], pf[0], pf[1]);
        float h1 = exp_pack(s[1], pf[2], pf[3]);
        if (!VB_LAZY_NOCHECK && !__all(fmaxf(h0, h1) <= kLazyBound)) {
          asm volatile("");
#if VB_LAZY_COUNT
          if (lane == 0) atomicAdd(&g_vb_stamp[10], 1ull);
#endif
          raise_m(fmaxf(half_max(s[0]), half_max(s[1])), std::integral_constant<int, 0>{});
          h0 = exp_pack(s[0], pf[0], pf[1]);
          h1 = exp_pack(s[1], pf[2], pf[3]);
        }
        l += h0 + h1;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) pv_pk(kk, pf[kk]);
      }
#if VB_LAZY_COUNT
      if (lane == 0) atomicAdd(&g_vb_stamp[11], kSplitPV ? 2ull : 1ull);
#endif
      return;
    }
    compute_s();
#pragma unroll
    for (int kk = 0; kk < VPRE; ++kk) read_v(kk);
    VB_STAMP(s1);
    if (klen < kKT) {   // tail tile only; the volatile asm keeps it a real (wave-uniform) branch
      asm volatile("");
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half >= klen) s[kt][r] = -INFINITY;
    }
    // row max: four independent chains (short dependency chains, max3-friendly)
    float mq[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {   // 16 v_max3 for 32 values (the minimum), depth 6
      const f32x16& x = s[c >> 1];
      const int o = 8 * (c & 1);
      mq[c] = max3f(max3f(max3f(x[o], x[o + 1], x[o + 2]), x[o + 3], x[o + 4]), x[o + 5], x[o + 6]);
    }
    const float f1 = max3f(mq[0], mq[1], s[0][7]);
    const float f2 = max3f(mq[2], mq[3], s[0][15]);
    float mt = max3f(max3f(f1, f2, s[1][7]), s[1][15], s[1][15]);
    if constexpr (kCBias) mt = max_xor32(mt);  // tile row max relative to m (bias included)
    else mt = max_xor32(mt) * p.c + bias;       // tile row max, exp2 domain
    // Deferred rescale (guide T13): the running max m is raised only when some row's tile max
    // exceeds it by more than kRescaleSlack (log2 units), so P = exp2(s - m) <= 2^kRescaleSlack.
    // O and l always share the same m, so the result is exact up to rounding; without the slack
    // nearly every tile of a 32-row wave rescales (some row's max grows), a 40-VALU O-wide pass.
    // The empty volatile asm keeps hipcc from if-converting this block into every iteration.
    if (kCBias) {
      if (first || !__all(mt <= kRescaleSlack)) {
        asm volatile("");
        // first tile: m := the tile's max (O and l are still zero; alpha would be meaningless)
        const float delta = first ? mt : fmaxf(mt, 0.f);
        const float alpha = first ? 0.f : exp2_fast(-delta);
        m += delta;
        l *= alpha;
#if VB_MFMA_ROWSUM
#pragma unroll
        for (int r = 0; r < 16; ++r) lsum[r] *= alpha;
#endif
#pragma unroll
        for (int i = 0; i < DT; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) s[kt][r] -= delta;
#pragma unroll
        for (int r = 0; r < 16; ++r) cb[r] -= delta;
        first = false;
      }
    } else if (!__all(mt <= m + kRescaleSlack)) {
      asm volatile("");
      const float mn = fmaxf(m, mt);
      const float alpha = exp2_fast(m - mn);
      m = mn;
      l *= alpha;
#if VB_MFMA_ROWSUM
#pragma unroll
      for (int r = 0; r < 16; ++r) lsum[r] *= alpha;
#endif
#pragma unroll
      for (int i = 0; i < DT; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
    }
    const float nbias = bias - m;
    float ls = 0.f;
    if (VB_DIAG && (p.dbg & 1)) {   // diagnostic: no exp
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = kCBias ? s[kt][r] : fmaf(s[kt][r], p.c, nbias);
          s[kt][r] = e;
          ls += e;
        }
    } else if (VB_MFMA_ROWSUM) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kt][r] = exp2_fast(kCBias ? s[kt][r] : fmaf(s[kt][r], p.c, nbias));
    } else if (kSplitPV) {
      // exp of the first 32 keys, their P.V k-steps, then the second 32: the PV MFMAs of the first
      // half overlap the second half's exp VALU (same sums, same order: bit-identical results)
      float lq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = exp2_fast(kCBias ? s[kt][r] : fmaf(s[kt][r], p.c, nbias));
          s[kt][r] = e;
          lq[(2 * kt + r) & 3] = (kt == 0 && r < 4) ? e : lq[(2 * kt + r) & 3] + e;   // no 0 + e
        }
#pragma unroll
        for (int kk = 2 * kt; kk < 2 * kt + 2; ++kk) {
          wait_v(kk);
          if (kk + VPRE < 4) read_v(kk + VPRE);
          const typename T::vec8 pf = pack8<T>(s[kk >> 1], 8 * (kk & 1));
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] = T::mfma32(join8<T>(vlo[kk][dt], vhi[kk][dt]), pf, o[dt]);
        }
      }
      ls = (lq[0] + lq[1]) + (lq[2] + lq[3]);
    } else {
      float lq[4] = {0.f, 0.f, 0.f, 0.f};   // four independent partial sums
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = exp2_fast(kCBias ? s[kt][r] : fmaf(s[kt][r], p.c, nbias));
          s[kt][r] = e;
          lq[(2 * kt + r) & 3] = (kt == 0 && r < 4) ? e : lq[(2 * kt + r) & 3] + e;
        }
      ls = (lq[0] + lq[1]) + (lq[2] + lq[3]);
    }
    l += ls;
    VB_STAMP(s2);
    VB_ACC(3, s2 - s1);
    // O^T += V^T . P^T : 4 k-steps of 16 keys (done above in the split form)
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kSplitPV && !(VB_DIAG && (p.dbg & 1)) && !VB_MFMA_ROWSUM) break;
      wait_v(kk);
      if (kk + VPRE < 4) read_v(kk + VPRE);
      const typename T::vec8 pf = pack8<T>(s[kk >> 1], 8 * (kk & 1));
      if constexpr (kPrio & 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] = T::mfma32(join8<T>(vlo[kk][dt], vhi[kk][dt]), pf, o[dt]);
      if constexpr (kPrio & 2) __builtin_amdgcn_s_setprio(0);
#if VB_MFMA_ROWSUM
      lsum = T::mfma32(ones, pf, lsum);
#endif
    }
    VB_STAMP(s3);
    VB_ACC(4, s3 - s2);
  };

  // Each ring slot remembers its tile's source (SGPRs, written when the tile is issued), and the
  // kept-block index of the next tile to issue is read from LDS one tile ahead, so no LDS round
  // trip sits between a barrier and the tile's first MFMA.
  auto list_at = [&](int t) __attribute__((always_inline)) -> int {
    return t < ntm ? (int)list[min(t >> 1, kMaxBlocks - 1)] : 0;
  };
  using Src = std::conditional_t<kML, MlTileSrc, TileSrc>;
  auto any_list_at = [&](int t) __attribute__((always_inline)) -> int {
    if constexpr (kML) return ml_list_at(t);
    else return list_at(t);
  };
  auto any_tile_src = [&](int t, int raw) __attribute__((always_inline)) -> Src {
    if constexpr (kML) return ml_tile_src(t, raw);
    else return tile_src(t, raw);
  };
  auto any_issue = [&](const Src src, int slot) __attribute__((always_inline)) {
    if constexpr (kML) ml_issue(src, slot);
    else issue(src, slot);
  };
  Src slot_src[kBufs];
  const int pool_bias_bits = __builtin_amdgcn_readfirstlane(__float_as_int(p.pool_bias_l2));
  int next_blk, idx_blk = 0;
  if constexpr (kKvRows) {
    // I0 .. I(kBufs-1), then the rows of tiles 0 .. kBufs-2, each once its offsets have landed
    // (younger than I(s): I(s+1) .. I(kBufs-1) and the s row stages already issued)
#pragma unroll
    for (int s0 = 0; s0 < kBufs; ++s0) issue_idx(s0, list_at(s0));
    slot_src[0] = tile_src(0, list_at(0));
    VB_WAIT_VMCNT(kBufs - 1);
    asm volatile("" ::: "memory");
    issue(slot_src[0], 0, 0);
    if constexpr (kBufs > 2) {
      slot_src[1] = tile_src(1, list_at(1));
      VB_WAIT_VMCNT(kBufs - 2 + kInstPerWave);
      asm volatile("" ::: "memory");
      issue(slot_src[1], 1, 1);
    }
    next_blk = list_at(kBufs - 1);
    idx_blk = list_at(kBufs);
  } else {
    slot_src[0] = any_tile_src(0, any_list_at(0));
    if (ntiles > 0) any_issue(slot_src[0], 0);
    if constexpr (kBufs > 2) {
      slot_src[1] = any_tile_src(1, any_list_at(1));
      if (ntiles > 1) any_issue(slot_src[1], 1);
    }
    next_blk = any_list_at(kBufs - 1);
  }
  if constexpr (kQLate) load_q();   // its wait (vmcnt 0) also lands the ring's first tiles
  // The loop body is instantiated once per ring slot (compile-time U), so every LDS address is a
  // loop-invariant lane base + immediate offset: no address VALU inside the loop.
  auto body = [&](int t, auto U) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    constexpr int un = (u + kBufs - 1) % kBufs;   // slot of the tile issued during this one
    VB_STAMP(st0);
    // retire this wave's DMAs of tile t (younger tiles stay in flight); the barrier then makes
    // every wave's part visible and proves slot (t-1) % kBufs is no longer being read
    const int ti = t + kBufs - 1;
    if constexpr (kKvRows) {
      // per body: I(t+kBufs) then the rows of tile t+kBufs-1, always (past the end too). Body t
      // needs K/V(t) and I(t+kBufs-1); only the rows of tile t+1 (3-slot ring) are younger.
      if constexpr (kBufs == 3) VB_WAIT_VMCNT(kInstPerWave);
      else VB_WAIT_VMCNT(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue_idx(t + kBufs, idx_blk);
      slot_src[un] = tile_src(ti, next_blk);
      issue(slot_src[un], un, ti);
      next_blk = idx_blk;
      idx_blk = list_at(t + kBufs + 1);   // in flight during this tile's compute
    } else {
      const int younger = min(ntiles - 1 - t, kBufs - 2);
      if (younger >= 2) VB_WAIT_VMCNT(2 * kInstPerWave);
      else if (younger == 1) VB_WAIT_VMCNT(kInstPerWave);
      else VB_WAIT_VMCNT(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (ti < ntiles) {
        slot_src[un] = any_tile_src(ti, next_blk);
        if (!(VB_NODMA && ti >= kBufs)) any_issue(slot_src[un], un);   // VB_NODMA: timing diagnostic only
        next_blk = any_list_at(ti + 1);   // in flight during this tile's compute
      }
    }
    VB_STAMP(st1);
    VB_ACC(0, st1 - st0);
    VB_STAMP(st2);
    VB_ACC(1, st2 - st1);
    const Src src = slot_src[u];
    int bias_bits;
    if constexpr (kML) {   // + ln(p) in the exp2 domain: log2(p) in {0, 1, 2, 3}
      bias_bits = src.lvl == 0 ? 0 : src.lvl == 1 ? 0x3F800000 : src.lvl == 2 ? 0x40000000 : 0x40400000;
    } else {
      bias_bits = (kPool && src.pooled) ? pool_bias_bits : 0;
    }
    bias_bits = __builtin_amdgcn_readfirstlane(bias_bits);
    if (VB_DIAG && (p.dbg & 2)) return;   // diagnostic: stream tiles only
    tile_step(U, bias_bits, src.klen);
    VB_STAMP(st3);
    VB_ACC(2, st3 - st2);
  };
  for (int t0 = 0; t0 < ntiles; t0 += kBufs) {
    body(t0, std::integral_constant<int, 0>{});
    if (t0 + 1 < ntiles) body(t0 + 1, std::integral_constant<int, 1>{});
    if constexpr (kBufs > 2)
      if (t0 + 2 < ntiles) body(t0 + 2, std::integral_constant<int, 2>{});
  }
  // the stages issued past the last tile land before exit; persistent launches always wait here (a
  // no-op at run time: every tile has landed): across the item loop's back edge hipcc's waitcnt pass
  // would otherwise count LDS-DMA as possibly in flight and wait (drain the ring) before the next
  // item's LDS reads
  if constexpr (kKvRows || kWQ) VB_WAIT_VMCNT(0);
  // The next item is claimed here, after the tile loop and before the epilogue's arithmetic and
  // stores, so its round trip overlaps them. Not inside the loop: the claim's wait for its own
  // result (and the waits hipcc then places after the branch) would drain the DMA ring every round.
  if (kWQ && tid == 0) next = wq_fetch(p.work_queue, blockIdx.x & 7, p.n_items);
#if VB_DIAG
  if (lane == 0) {
    for (int i = 0; i < 5; ++i) atomicAdd(&g_vb_stamp[i], acc_st[i]);
    atomicAdd(&g_vb_stamp[8], (unsigned long long)ntiles);
  }
#endif

  // ---- epilogue -----------------------------------------------------------------------------------
#if VB_MFMA_ROWSUM
  const float lt = lsum[0];
#else
  const float lt = add_xor32(l);
#endif
  const float inv = (lt > 0.f) ? 1.0f / lt : 0.f;
  // streaming heads (unsupported) are flagged with NaN outputs written as bit patterns: this
  // translation unit is compiled with -fno-honor-nans, so no float arithmetic may produce them
  constexpr uint32_t kNaN2 = std::is_same<T, BF16>::value ? 0x7FC07FC0u : 0x7E007E00u;
  if (qvalid) {
    uint8_t* obase = reinterpret_cast<uint8_t*>(p.out) +
                     2 * (b * p.os[0] + h * p.os[1] + (qrow0 + qrow) * p.os[2]);
    // Each lane holds half of its row's 8-column groups (lane l: columns 8g..8g+3, lane l+32:
    // 8g+4..8g+7). One v_permlane32_swap per dword pairs groups 2p and 2p+1 so every lane owns 16
    // contiguous bytes: half the store instructions of the 8-byte form (guide T21).
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        u32x2 a, c;
        a[0] = pack2<T>(o[dt][8 * pr + 0] * inv, o[dt][8 * pr + 1] * inv);
        a[1] = pack2<T>(o[dt][8 * pr + 2] * inv, o[dt][8 * pr + 3] * inv);
        c[0] = pack2<T>(o[dt][8 * pr + 4] * inv, o[dt][8 * pr + 5] * inv);
        c[1] = pack2<T>(o[dt][8 * pr + 6] * inv, o[dt][8 * pr + 7] * inv);
        if (nan_head) a[0] = a[1] = c[0] = c[1] = kNaN2;
        const auto sx = __builtin_amdgcn_permlane32_swap(a[0], c[0], false, false);
        const auto sy = __builtin_amdgcn_permlane32_swap(a[1], c[1], false, false);
        const u32x4 w = {sx[0], sy[0], sx[1], sy[1]};
        *reinterpret_cast<u32x4*>(obase + (dt * 32 + 16 * pr + 8 * half) * 2) = w;
      }
    if (p.lse && half == 0) {
      const float v = (m + __log2f(lt)) * kLn2;
      float* dst = p.lse + b * p.lse_s[0] + h * p.lse_s[1] + (p.cu_q ? qg : qrow);
      if (nan_head) *reinterpret_cast<uint32_t*>(dst) = 0x7FC00000u;
      // a row with no kept key: -inf on the module path; +inf on the reference-signature entry
      // (cu_q set), FlashAttention-2's convention for an empty softmax (normalize_softmax_lse)
      else *dst = (p.cu_q && !(lt > 0.f)) ? INFINITY : v;
    }
  }
  VB_ATRACE_END();
}

template <int D, class T, bool kPool, bool kKvRows, bool kML = false, bool kCBias = false, bool kPersist = false>
__global__ void __launch_bounds__(kThreads, (D == 64 ? VB_FWD_WAVES_D64 : 2)) attn_fwd_kernel(const FwdParams p) {
  if constexpr (!kPersist) {   // one workgroup per item
    int next;
    attn_fwd_item<D, T, kPool, kKvRows, kML, kCBias, false>(p, blockIdx.x, next);
  } else {
    // persistent: a resident-sized grid, every item (the first one too) from the work queue
    __shared__ int next_s;
    int* const wq = p.work_queue;
    if (threadIdx.x == 0) next_s = wq_fetch(wq, blockIdx.x & 7, p.n_items);
    __syncthreads();
    int item = next_s;
    while (item >= 0) {
      int next = -2;   // -2: not claimed during the item (it returned before its tile loop)
      attn_fwd_item<D, T, kPool, kKvRows, kML, kCBias, true>(p, item, next);
      // every wave is done with this item's LDS (ring, list) before the next item's prologue writes it
      if (threadIdx.x == 0) next_s = next == -2 ? wq_fetch(wq, blockIdx.x & 7, p.n_items) : next;
      __syncthreads();
      item = next_s;
      __syncthreads();   // next_s is read by every wave before lane 0 may overwrite it
    }
    if (threadIdx.x == 0) wq_finish(wq);   // the last workgroup re-zeroes the queue
  }
}

// Dispatch order of the attention kernel's phase 2 (longest-processing-time first, per XCD): the
// kernel deals workgroups round-robin over the 8 XCDs and gives XCD x the contiguous range of
// linear work items xcd_linear assigns it (head-major). Each XCD drains its range in order, so its
// last workgroups set the kernel's tail. One workgroup per XCD range re-sorts the range by (head,
// kept key blocks descending): the head-major grouping (the L2 reuse of a head's K/V) stays, and
// within every head the longest q-blocks go first and the shortest last. Counting sort over
// (head, length) bins in LDS; the order inside a bin follows the atomics (placement only: every
// q-block's output is the same whatever the order). order[start + rank] = item.
constexpr int kOrderBins = 8192;
__global__ void __launch_bounds__(1024) attn_order_kernel(const FwdParams p, int32_t* order) {
  __shared__ int bins[kOrderBins];
  const int BH = p.B * p.H;
  const int hr = min(p.heavy_rows, p.nbq);
  const int rows_left = p.nbq - hr;
  const int nwg = rows_left * BH;
  const int x = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  int start = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
  const int count_x = q8 + (x < r8 ? 1 : 0);
  if (count_x <= 0) return;
  // only the range's last `order_window` items are re-ordered (the rest keep their place)
  const int skip = (p.order_window > 0 && p.order_window < count_x) ? count_x - p.order_window : 0;
  for (int i = threadIdx.x; i < skip; i += blockDim.x) order[start + i] = start + i;
  start += skip;
  const int count = count_x - skip;
  const int bh0 = start / rows_left;
  const int nh = (start + count - 1) / rows_left - bh0 + 1;
  const int nl = p.nbk + 1;   // kept counts 0..nbk
  // (head, length) bins; a range spanning more heads than LDS has bins for sorts by length alone
  // (longest first over the whole range: the tail is still the shortest items, the head-major
  // grouping is given up). nl <= kMaxBlocks + 1 < kOrderBins always fits.
  const bool by_head = (int64_t)nh * nl <= kOrderBins;
  const int nbins = by_head ? nh * nl : nl;
  for (int i = threadIdx.x; i < nbins; i += blockDim.x) bins[i] = 0;
  __syncthreads();
  auto key_of = [&](int lin) -> int {
    const int bh = lin / rows_left, qblk = rows_left - 1 - lin % rows_left;
    bool nan_head = false;
    const uint8_t* mh = head_mask_base(p.mask, p.ms, p.head_mask_type, p.H, bh / p.H, bh % p.H, nan_head, p.hm_mode);
    int kept = p.nbk;
    if (p.q_len) {
      kept = min(max(p.q_len[(int64_t)bh * p.nbq + qblk], 0), p.nbk);
    } else if (mh) {
      const uint8_t* mrow = mh + (int64_t)qblk * p.ms[2];
      kept = 0;
      for (int j = 0; j < p.nbk; ++j) kept += mrow[j] != 0;
    }
    return (by_head ? (bh - bh0) * nl : 0) + (p.nbk - kept);   // head ascending, kept count descending
  };
  for (int i = threadIdx.x; i < count; i += blockDim.x) atomicAdd(&bins[key_of(start + i)], 1);
  __syncthreads();
  {   // exclusive prefix over the bins: every thread a run of C bins, a scan of the runs' sums
    __shared__ int wsum[16];
    const int C = (nbins + 1023) / 1024;
    const int b0 = threadIdx.x * C;
    int run = 0;
    for (int i = 0; i < C; ++i) run += (b0 + i < nbins) ? bins[b0 + i] : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = run;   // inclusive scan within the wave
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int wbase = 0;
    for (int i = 0; i < w; ++i) wbase += wsum[i];
    int pos = wbase + incl - run;   // exclusive prefix of this thread's run
    for (int i = 0; i < C; ++i) {
      if (b0 + i < nbins) {
        const int c = bins[b0 + i];
        bins[b0 + i] = pos;
        pos += c;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < count; i += blockDim.x) {
    const int lin = start + i;
    order[start + atomicAdd(&bins[key_of(lin)], 1)] = lin;
  }
}

// Grid of one launch: one workgroup per item, or (work queue) as many as are resident at once —
// the occupancy of this instantiation times the device's CUs (host queries, cached per kernel and
// device; no device synchronisation), a multiple of 8 so every XCD gets the same number.
// Grid of one launch: one workgroup per item, or (persistent instantiation, with a work queue) as
// many as are resident at once (resident_grid: occupancy x CUs, a multiple of 8).
template <auto Kern, auto KernP>
static int launch_one(FwdParams p, hipStream_t stream, const char* what) {
  const unsigned items = (unsigned)(p.nbq * p.B * p.H);
  p.n_items = (int)items;
  if (p.work_queue) {
    const unsigned slots = (unsigned)resident_grid(reinterpret_cast<const void*>(KernP), kThreads, 0);
    hipLaunchKernelGGL(KernP, dim3(slots < items ? slots : items), dim3(kThreads), 0, stream, p);
  } else {
    hipLaunchKernelGGL(Kern, dim3(items), dim3(kThreads), 0, stream, p);
  }
  return check_launch(what);
}

template <int D, class T>
static int launch_fwd(const FwdParams& p, bool pool, hipStream_t stream) {
  const bool rows = p.kv_rows != nullptr;
  const bool cbias = VB_FWD_CBIAS && p.lse == nullptr;
  const char* w = "attn_fwd_kernel";
  if (cbias && pool && rows) return launch_one<attn_fwd_kernel<D, T, true, true, false, true, false>, attn_fwd_kernel<D, T, true, true, false, true, true>>(p, stream, w);
  if (cbias && rows) return launch_one<attn_fwd_kernel<D, T, false, true, false, true, false>, attn_fwd_kernel<D, T, false, true, false, true, true>>(p, stream, w);
  if (cbias && pool) return launch_one<attn_fwd_kernel<D, T, true, false, false, true, false>, attn_fwd_kernel<D, T, true, false, false, true, true>>(p, stream, w);
  if (cbias) return launch_one<attn_fwd_kernel<D, T, false, false, false, true, false>, attn_fwd_kernel<D, T, false, false, false, true, true>>(p, stream, w);
  if (pool && rows) return launch_one<attn_fwd_kernel<D, T, true, true, false, false, false>, attn_fwd_kernel<D, T, true, true, false, false, true>>(p, stream, w);
  if (pool) return launch_one<attn_fwd_kernel<D, T, true, false, false, false, false>, attn_fwd_kernel<D, T, true, false, false, false, true>>(p, stream, w);
  if (rows) return launch_one<attn_fwd_kernel<D, T, false, true, false, false, false>, attn_fwd_kernel<D, T, false, true, false, false, true>>(p, stream, w);
  return launch_one<attn_fwd_kernel<D, T, false, false, false, false, false>, attn_fwd_kernel<D, T, false, false, false, false, true>>(p, stream, w);
}

static int dispatch_fwd(const FwdParams& p, int D, int dtype, bool pool, hipStream_t stream) {
  if (dtype == VB_DTYPE_BF16) {
    if (D == 64) return launch_fwd<64, BF16>(p, pool, stream);
    if (D == 128) return launch_fwd<128, BF16>(p, pool, stream);
  } else if (dtype == VB_DTYPE_F16) {
    if (D == 64) return launch_fwd<64, F16>(p, pool, stream);
    if (D == 128) return launch_fwd<128, F16>(p, pool, stream);
  } else {
    return fail(VB_ERR_INVALID, "attn: unknown dtype");
  }
  return fail(VB_ERR_UNSUPPORTED, "attn: head_dim must be 64 or 128, got " + std::to_string(D));
}

static bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }


}  // namespace vb

#if VB_DIAG || VB_LAZY_COUNT
extern "C" int vb_diag_stamps(unsigned long long* host16, int reset) {
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(host16, HIP_SYMBOL(vb::g_vb_stamp), sizeof(unsigned long long) * 16);
  if (reset) {
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(vb::g_vb_stamp), z, sizeof(z));
  }
  return 0;
}
#endif

extern "C" int vb_attn_fwd(const vb_attn_args* a, void* stream) {
  using namespace vb;
  if (!a) return fail(VB_ERR_INVALID, "vb_attn_fwd: null args");
  if (a->B <= 0 || a->H <= 0 || a->Lq <= 0 || a->D <= 0)
    return fail(VB_ERR_INVALID, "vb_attn_fwd: B, H, Lq, D must be positive");
  if (!a->q || !a->out || (a->use_main && (!a->k || !a->v || a->Lk <= 0)))
    return fail(VB_ERR_INVALID, "vb_attn_fwd: missing q/k/v/out");
  const bool pool = a->kp != nullptr;
  if (!a->use_main && !pool) return fail(VB_ERR_INVALID, "vb_attn_fwd: nothing to attend to");
  if (pool && (!a->vp || a->Lkp <= 0)) return fail(VB_ERR_INVALID, "vb_attn_fwd: pooled branch needs vp and Lkp > 0");
  const int nbq = (a->Lq + kQBlk - 1) / kQBlk;
  const int nbk = a->use_main ? (a->Lk + kQBlk - 1) / kQBlk : 0;
  if (nbk > kMaxBlocks) return fail(VB_ERR_UNSUPPORTED, "vb_attn_fwd: Lk too long");
  for (int i = 0; i < 3; ++i) {
    if ((a->q_stride[i] | a->out_stride[i]) & 7) return fail(VB_ERR_INVALID, "vb_attn_fwd: q/out strides must be multiples of 8 elements");
    if (a->use_main && ((a->k_stride[i] | a->v_stride[i]) & 7)) return fail(VB_ERR_INVALID, "vb_attn_fwd: k/v strides must be multiples of 8 elements");
    if (pool && ((a->kp_stride[i] | a->vp_stride[i]) & 7)) return fail(VB_ERR_INVALID, "vb_attn_fwd: kp/vp strides must be multiples of 8 elements");
  }
  if (a->kv_rows && a->Lk >= (1 << 24))
    return fail(VB_ERR_UNSUPPORTED, "vb_attn_fwd: kv_rows needs Lk < 2^24");
  // the tile DMA offsets use 24-bit multiplies: row strides below 2^24 bytes (16 MiB per row)
  if ((a->use_main && (a->k_stride[2] * 2 >= (1 << 24) || a->v_stride[2] * 2 >= (1 << 24))) ||
      (pool && (a->kp_stride[2] * 2 >= (1 << 24) || a->vp_stride[2] * 2 >= (1 << 24))))
    return fail(VB_ERR_UNSUPPORTED, "vb_attn_fwd: k/v/kp/vp row strides must be < 2^24 bytes");
  const int64_t kLim = int64_t(1) << 31;   // one (b,h) slice must be addressable by a 32-bit buffer offset
  if (a->use_main && ((int64_t)(a->Lk - 1) * 2 * (a->k_stride[2] > a->v_stride[2] ? a->k_stride[2] : a->v_stride[2]) + 2 * a->D >= kLim))
    return fail(VB_ERR_UNSUPPORTED, "vb_attn_fwd: a k/v (b,h) slice spans >= 2 GiB");
  if (pool && ((int64_t)(a->Lkp - 1) * 2 * (a->kp_stride[2] > a->vp_stride[2] ? a->kp_stride[2] : a->vp_stride[2]) + 2 * a->D >= kLim))
    return fail(VB_ERR_UNSUPPORTED, "vb_attn_fwd: a kp/vp (b,h) slice spans >= 2 GiB");
  if (!aligned16(a->q) || !aligned16(a->out) || (a->use_main && (!aligned16(a->k) || !aligned16(a->v))) ||
      (pool && (!aligned16(a->kp) || !aligned16(a->vp))))
    return fail(VB_ERR_INVALID, "vb_attn_fwd: tensors must be 16-byte aligned");
  FwdParams p{};
  p.q = a->q; p.k = a->k; p.v = a->v;
  for (int i = 0; i < 3; ++i) {
    p.qs[i] = a->q_stride[i]; p.ks[i] = a->k_stride[i]; p.vs[i] = a->v_stride[i];
    p.ms[i] = a->mask_stride[i]; p.kps[i] = a->kp_stride[i]; p.vps[i] = a->vp_stride[i];
    p.os[i] = a->out_stride[i];
  }
  p.q_rows = a->q_rows; p.kv_rows = a->kv_rows;
  p.use_main = a->use_main;
  p.mask = a->block_mask;
  p.kp = a->kp; p.vp = a->vp; p.Lkp = a->Lkp;
  p.pool_bias_l2 = a->kp_log_bias * kLog2e;
  p.out = a->out; p.lse = a->lse;
  p.lse_s[0] = (int64_t)a->H * a->Lq; p.lse_s[1] = a->Lq;
  p.B = a->B; p.H = a->H; p.Lq = a->Lq; p.Lk = a->use_main ? a->Lk : 1; p.nbq = nbq; p.nbk = nbk;
  const float scale = a->scale > 0.f ? a->scale : (float)(1.0 / sqrt((double)a->D));
  p.c = scale * kLog2e;
  p.heavy_rows = a->heavy_rows;
#if VB_DIAG
  if (const char* d = getenv("VB_DEBUG_ATTN")) p.dbg = atoi(d);
#endif
  p.q_len = a->q_lengths;
  p.order_window = a->order_window;
  p.work_queue = a->work_queue;
  if (a->q_order && p.use_main && p.mask) {   // longest-first dispatch order (scheduling only)
    hipLaunchKernelGGL(attn_order_kernel, dim3(8), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream), p,
                       a->q_order);
    if (int rc = check_launch("attn_order_kernel")) return rc;
    p.q_order = a->q_order;
  }
  return dispatch_fwd(p, a->D, a->dtype, pool, reinterpret_cast<hipStream_t>(stream));
}

#if VB_ATTN_TRACE
VB_TRACE_GETTER(vb_debug_attn_trace, vb::g_attn_trace)
#endif

extern "C" int vb_kv_pyramid_rows(int L) {
  const int lpad = (L + vb::kQBlk - 1) / vb::kQBlk * vb::kQBlk;
  return 15 * (lpad / 8);
}

extern "C" int vb_ml_attn_fwd(const vb_ml_attn_args* a, void* stream) {
  using namespace vb;
  if (!a) return fail(VB_ERR_INVALID, "vb_ml_attn_fwd: null args");
  if (a->B <= 0 || a->H <= 0 || a->L <= 0) return fail(VB_ERR_INVALID, "vb_ml_attn_fwd: B, H, L must be positive");
  if (!a->q || !a->kpyr || !a->vpyr || !a->level_mask || !a->out)
    return fail(VB_ERR_INVALID, "vb_ml_attn_fwd: missing q/kpyr/vpyr/level_mask/out");
  if (a->D != 64 && a->D != 128)
    return fail(VB_ERR_UNSUPPORTED, "vb_ml_attn_fwd: head_dim must be 64 or 128, got " + std::to_string(a->D));
  const int nb = (a->L + kQBlk - 1) / kQBlk;
  if (nb > kMaxBlocks) return fail(VB_ERR_UNSUPPORTED, "vb_ml_attn_fwd: L too long");
  for (int i = 0; i < 3; ++i)
    if ((a->q_stride[i] | a->out_stride[i]) & 7) return fail(VB_ERR_INVALID, "vb_ml_attn_fwd: q/out strides must be multiples of 8 elements");
  const int R = vb_kv_pyramid_rows(a->L);
  if ((int64_t)R * 2 * a->D >= (int64_t(1) << 31)) return fail(VB_ERR_UNSUPPORTED, "vb_ml_attn_fwd: a pyramid (b,h) slice spans >= 2 GiB");
  if (!aligned16(a->q) || !aligned16(a->out) || !aligned16(a->kpyr) || !aligned16(a->vpyr))
    return fail(VB_ERR_INVALID, "vb_ml_attn_fwd: tensors must be 16-byte aligned");
  FwdParams p{};
  p.q = a->q; p.k = a->kpyr; p.v = a->vpyr;
  for (int i = 0; i < 3; ++i) {
    p.qs[i] = a->q_stride[i]; p.os[i] = a->out_stride[i]; p.ms[i] = a->mask_stride[i];
  }
  p.ks[0] = p.vs[0] = (int64_t)a->H * R * a->D;
  p.ks[1] = p.vs[1] = (int64_t)R * a->D;
  p.ks[2] = p.vs[2] = a->D;
  p.q_rows = a->q_rows;
  p.use_main = 1;
  p.mask = a->level_mask;
  p.out = a->out; p.lse = a->lse;
  p.lse_s[0] = (int64_t)a->H * a->L; p.lse_s[1] = a->L;
  p.B = a->B; p.H = a->H; p.Lq = a->L; p.Lk = a->L; p.nbq = nb; p.nbk = nb;
  p.Lpad = nb * kQBlk;
  p.ref_tail = a->ref_tail ? 1 : 0;
  const float scale = a->scale > 0.f ? a->scale : (float)(1.0 / sqrt((double)a->D));
  p.c = scale * kLog2e;
  p.heavy_rows = a->heavy_rows;
  p.work_queue = a->work_queue;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool cb = VB_FWD_CBIAS && p.lse == nullptr;   // inference launches (see kCBias)
  const char* w = "attn_fwd_kernel (multi-level)";
  if (a->dtype == VB_DTYPE_BF16) {
    if (a->D == 64 && cb) return launch_one<attn_fwd_kernel<64, BF16, false, false, true, true, false>, attn_fwd_kernel<64, BF16, false, false, true, true, true>>(p, st, w);
    if (a->D == 64) return launch_one<attn_fwd_kernel<64, BF16, false, false, true, false, false>, attn_fwd_kernel<64, BF16, false, false, true, false, true>>(p, st, w);
    if (cb) return launch_one<attn_fwd_kernel<128, BF16, false, false, true, true, false>, attn_fwd_kernel<128, BF16, false, false, true, true, true>>(p, st, w);
    return launch_one<attn_fwd_kernel<128, BF16, false, false, true, false, false>, attn_fwd_kernel<128, BF16, false, false, true, false, true>>(p, st, w);
  }
  if (a->dtype == VB_DTYPE_F16) {
    if (a->D == 64 && cb) return launch_one<attn_fwd_kernel<64, F16, false, false, true, true, false>, attn_fwd_kernel<64, F16, false, false, true, true, true>>(p, st, w);
    if (a->D == 64) return launch_one<attn_fwd_kernel<64, F16, false, false, true, false, false>, attn_fwd_kernel<64, F16, false, false, true, false, true>>(p, st, w);
    if (cb) return launch_one<attn_fwd_kernel<128, F16, false, false, true, true, false>, attn_fwd_kernel<128, F16, false, false, true, true, true>>(p, st, w);
    return launch_one<attn_fwd_kernel<128, F16, false, false, true, false, false>, attn_fwd_kernel<128, F16, false, false, true, false, true>>(p, st, w);
  }
  return fail(VB_ERR_INVALID, "vb_ml_attn_fwd: unknown dtype");
}

extern "C" int vb_block_sparse_attn_fwd(const void* q_unpad, const void* k_unpad, const void* v_unpad,
                                        const int32_t* cu_seqlens_q, const int32_t* cu_seqlens_k,
                                        const int32_t* head_mask_type, const int32_t* streaming_info,
                                        const uint8_t* base_blockmask, int batch, int num_heads, int head_dim,
                                        int max_seqlen_q, int max_seqlen_k, float p_dropout, int deterministic,
                                        float softmax_scale, int is_causal, int exact_streaming, int dtype,
                                        void* out_unpad, float* softmax_lse, int mask_head_mode, void* stream) {
  using namespace vb;
  (void)streaming_info;
  (void)deterministic;
  if (p_dropout != 0.f) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_fwd: p_dropout must be 0");
  if (is_causal || exact_streaming) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_fwd: causal/streaming not supported");
  if (mask_head_mode != VB_MASK_HEAD_PER_HEAD && mask_head_mode != VB_MASK_HEAD_SHARED0)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_fwd: unknown mask_head_mode");
  if (!q_unpad || !k_unpad || !v_unpad || !cu_seqlens_q || !cu_seqlens_k || !out_unpad)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_fwd: null tensor");
  if (batch <= 0 || num_heads <= 0 || max_seqlen_q <= 0 || max_seqlen_k <= 0)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_fwd: bad sizes");
  const int nbq = (max_seqlen_q + kQBlk - 1) / kQBlk;
  const int nbk = (max_seqlen_k + kQBlk - 1) / kQBlk;
  if (nbk > kMaxBlocks) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_fwd: max_seqlen_k too long");
  if ((int64_t)(max_seqlen_k - 1) * 2 * num_heads * head_dim + 2 * head_dim >= (int64_t(1) << 31))
    return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_fwd: a sequence's k/v span >= 2 GiB");
  FwdParams p{};
  p.q = q_unpad; p.k = k_unpad; p.v = v_unpad;
  const int64_t row = (int64_t)num_heads * head_dim;
  p.qs[0] = p.ks[0] = p.vs[0] = p.os[0] = 0;
  p.qs[1] = p.ks[1] = p.vs[1] = p.os[1] = head_dim;
  p.qs[2] = p.ks[2] = p.vs[2] = p.os[2] = row;
  p.cu_q = cu_seqlens_q; p.cu_k = cu_seqlens_k;
  p.head_mask_type = head_mask_type;
  p.hm_mode = mask_head_mode;
  p.use_main = 1;
  p.mask = base_blockmask;  // may be NULL: dense
  // base_blockmask [batch, n_sparse, nbq, nbk]: n_sparse (= number of heads whose mask id is 1) is
  // counted on the device from head_mask_type (no host read of device memory, no sync).
  p.ms[0] = head_mask_type ? -1 : (int64_t)num_heads * nbq * nbk;
  p.ms[1] = (int64_t)nbq * nbk; p.ms[2] = nbk;
  p.out = out_unpad; p.lse = softmax_lse;
  p.lse_s[0] = (int64_t)num_heads * max_seqlen_q; p.lse_s[1] = max_seqlen_q;
  p.B = batch; p.H = num_heads; p.Lq = max_seqlen_q; p.Lk = max_seqlen_k; p.nbq = nbq; p.nbk = nbk;
  const float scale = softmax_scale > 0.f ? softmax_scale : (float)(1.0 / sqrt((double)head_dim));
  p.c = scale * kLog2e;
  return dispatch_fwd(p, head_dim, dtype, false, reinterpret_cast<hipStream_t>(stream));
}

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
#include "vb_common.hpp"

namespace vb {

struct FwdParams {
  const void* q; const void* k; const void* v;
  int64_t qs[3], ks[3], vs[3];
  const int32_t* q_rows; const int32_t* kv_rows;
  const int32_t* cu_q; const int32_t* cu_k;   // varlen row offsets (reference API), nullable
  const int32_t* head_mask_type;              // reference API, nullable
  int use_main;
  const uint8_t* mask; int64_t ms[3];
  const void* kp; const void* vp; int64_t kps[3], vps[3];
  int Lkp; float pool_bias_l2;                 // bias in the exp2 domain (log2 gap)
  void* out; int64_t os[3];
  float* lse; int64_t lse_s[2];               // row stride 1
  int B, H, Lq, Lk, nbq, nbk;
  float c;                                    // softmax scale * log2(e)
};

constexpr int kThreads = 256;
constexpr int kQBlk = 128;   // rows per workgroup (4 waves x 32)
constexpr int kKT = 64;      // keys per LDS tile
constexpr int kMaxBlocks = 1024;  // keys <= 131072

// ---- LDS images --------------------------------------------------------------------------------
// K: [64 rows][D] with 16-byte chunks XOR-swizzled so a ds_read_b128 column slice (32 rows, one
//    chunk) hits 16 distinct bank slots per lane group (guide T2).
template <int D>
__device__ __forceinline__ int k_off(int row, int ch) {
  constexpr int kRowBytes = D * 2;
  const int sw = (D == 64) ? ((row >> 1) & 7) : (row & 15);
  return row * kRowBytes + 16 * (ch ^ sw);
}
// V: [64 rows][D] row-major, 64-byte granules XOR-swizzled so the 4-row x 64-byte footprint of
//    a half-wave's ds_read_b64_tr_b16 covers a full 256-byte bank row.
template <int D>
__device__ __forceinline__ int v_off_bytes(int row, int col) {
  constexpr int kRowBytes = D * 2;
  const int g = col >> 5;
  const int sw = (D == 64) ? ((row >> 1) & 1) : (row & 3);
  return row * kRowBytes + 64 * (g ^ sw) + (col & 31) * 2;
}

template <class T>
__device__ __forceinline__ typename T::vec8 lds_b128(const uint8_t* base, int off) {
  return *reinterpret_cast<const typename T::vec8*>(base + off);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4 lds_tr4(const uint8_t* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + off));
}

template <class T>
__device__ __forceinline__ typename T::vec8 join8(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(typename T::vec8, r);
}

template <class T>
__device__ __forceinline__ typename T::vec8 pack8(const f32x16& acc, int base) {
  u32x4 u;
  u[0] = pack2<T>(acc[base + 0], acc[base + 1]);
  u[1] = pack2<T>(acc[base + 2], acc[base + 3]);
  u[2] = pack2<T>(acc[base + 4], acc[base + 5]);
  u[3] = pack2<T>(acc[base + 6], acc[base + 7]);
  return __builtin_bit_cast(typename T::vec8, u);
}

// Global -> register staging of one 64-key tile of K and V (each thread: CH*64/256 chunks).
template <int D>
struct Stage {
  static constexpr int CH = D / 8;                      // 16-byte chunks per row
  static constexpr int N = kKT * CH / kThreads;         // chunks per thread per matrix (2 or 4)
  u32x4 kr[N];
  u32x4 vr[N];
};

template <int D>
__device__ __forceinline__ void stage_load(Stage<D>& st, const uint8_t* kbase, const uint8_t* vbase,
                                           int64_t krow_stride, int64_t vrow_stride,
                                           const int32_t* rows, int kstart, int klen) {
  constexpr int CH = Stage<D>::CH;
#pragma unroll
  for (int i = 0; i < Stage<D>::N; ++i) {
    const int c = threadIdx.x + i * kThreads;
    const int r = c / CH, ch = c % CH;
    int kr = kstart + min(r, klen - 1);
    if (rows) kr = rows[kr];
    st.kr[i] = *reinterpret_cast<const u32x4*>(kbase + (int64_t)kr * krow_stride + ch * 16);
    st.vr[i] = *reinterpret_cast<const u32x4*>(vbase + (int64_t)kr * vrow_stride + ch * 16);
  }
}

template <int D>
__device__ __forceinline__ void stage_store(const Stage<D>& st, uint8_t* kl, uint8_t* vl) {
  constexpr int CH = Stage<D>::CH;
#pragma unroll
  for (int i = 0; i < Stage<D>::N; ++i) {
    const int c = threadIdx.x + i * kThreads;
    const int r = c / CH, ch = c % CH;
    *reinterpret_cast<u32x4*>(kl + k_off<D>(r, ch)) = st.kr[i];
    *reinterpret_cast<u32x4*>(vl + v_off_bytes<D>(r, ch * 8)) = st.vr[i];
  }
}

// Describes where tile t's keys come from.
struct TileSrc {
  int pooled;   // 0 = main (block-masked) keys, 1 = pooled keys
  int kstart;   // first key (reordered index for main, pooled index otherwise)
  int klen;     // valid keys in this tile (1..64)
};

template <int D, class T, bool kPool>
__global__ void __launch_bounds__(kThreads, 2) attn_fwd_kernel(const FwdParams p) {
  constexpr int KS = D / 16;   // k-steps of the QK^T product
  constexpr int DT = D / 32;   // 32-wide d tiles of the output
  constexpr int kTileBytes = kKT * D * 2;
  __shared__ __attribute__((aligned(16))) uint8_t smem[4 * kTileBytes + kMaxBlocks * 2 + 16];
  // buffer i: K image at smem + 2*i*kTileBytes, V image right after it
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + 4 * kTileBytes);
  int* list_n = reinterpret_cast<int*>(smem + 4 * kTileBytes + kMaxBlocks * 2);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int half = lane >> 5;
  const int l32 = lane & 31;

  // heavy-first order: the last q-blocks (CogVideoX's dense text rows) of every head first
  const int BH = p.B * p.H;
  const int qblk = p.nbq - 1 - (int)(blockIdx.x / BH);
  const int bh = blockIdx.x % BH;
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
  bool dense = (p.mask == nullptr);
  bool nan_head = false;
  if (p.use_main && !dense) {
    int mh = h;
    if (p.head_mask_type) {
      const int t = p.head_mask_type[h];
      if (t == 0) dense = true;
      else if (t < 0) nan_head = true;
      else if (t == 1) {
        int cnt = 0;
        for (int i = 0; i <= h; ++i) cnt += (p.head_mask_type[i] == 1);
        mh = cnt - 1;
      } else {
        mh = t - 1;
      }
    }
    int64_t mb = p.ms[0];
    if (mb < 0) {  // reference API: batch stride = (#heads with mask id 1) * nbq * nbk
      int ones = 0;
      for (int i = 0; i < p.H; ++i) ones += (p.head_mask_type[i] == 1);
      mb = (int64_t)ones * p.ms[1];
    }
    mrow = p.mask + b * mb + (int64_t)mh * p.ms[1] + (int64_t)qblk * p.ms[2];
  }
  if (threadIdx.x < 64) {
    int n = 0;
    if (p.use_main) {
      for (int j0 = 0; j0 < nbk; j0 += 64) {
        const int j = j0 + lane;
        const bool keep = (j < nbk) && (dense || mrow[j] != 0);
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
  __syncthreads();
  const int nkept = *list_n;
  // main tiles: two 64-key halves per kept block, minus an empty second half of the last block
  int ntm = 2 * nkept;
  if (nkept > 0 && list[nkept - 1] == nbk - 1 && (nbk - 1) * kQBlk + kKT >= Lk) ntm -= 1;
  const int ntp = kPool ? (p.Lkp + kKT - 1) / kKT : 0;
  const int ntiles = ntm + ntp;

  const uint8_t* qbase = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1] + qrow0 * p.qs[2]);
  const uint8_t* kbase = reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1] + krow0 * p.ks[2]);
  const uint8_t* vbase = reinterpret_cast<const uint8_t*>(p.v) + 2 * (b * p.vs[0] + h * p.vs[1] + krow0 * p.vs[2]);
  const uint8_t* kpbase = nullptr;
  const uint8_t* vpbase = nullptr;
  if (kPool) {
    kpbase = reinterpret_cast<const uint8_t*>(p.kp) + 2 * (b * p.kps[0] + h * p.kps[1]);
    vpbase = reinterpret_cast<const uint8_t*>(p.vp) + 2 * (b * p.vps[0] + h * p.vps[1]);
  }

  auto tile_src = [&](int t) -> TileSrc {
    TileSrc s;
    if (t < ntm) {
      const int blk = list[t >> 1];
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
  auto load_tile = [&](Stage<D>& st, int t) {
    const TileSrc s = tile_src(t);
    if (!kPool || !s.pooled)
      stage_load<D>(st, kbase, vbase, 2 * p.ks[2], 2 * p.vs[2], p.kv_rows, s.kstart, s.klen);
    else
      stage_load<D>(st, kpbase, vpbase, 2 * p.kps[2], 2 * p.vps[2], nullptr, s.kstart, s.klen);
  };

  // ---- Q fragment (B operand of S^T = K.Q^T): row l32 of this wave, d = 16s + 8*half + j --------
  const int qg = q0 + wave * 32 + l32;               // reordered query position
  const bool qvalid = qg < Lq;
  int qrow = qvalid ? qg : Lq - 1;
  if (p.q_rows) qrow = p.q_rows[qrow];
  typename T::vec8 qf[KS];
  {
    const uint8_t* qp = qbase + (int64_t)qrow * 2 * p.qs[2];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      qf[s] = *reinterpret_cast<const typename T::vec8*>(qp + (16 * s + 8 * half) * 2);
  }

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY;  // running max (exp2 domain) of this lane's query row
  float l = 0.f;        // running partial row sum (this half's keys)

  Stage<D> st;
  if (ntiles > 0) {
    load_tile(st, 0);
    stage_store<D>(st, smem, smem + kTileBytes);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load_tile(st, t + 1);
    const TileSrc src = tile_src(t);
    const float bias = (kPool && src.pooled) ? p.pool_bias_l2 : 0.f;
    const uint8_t* kl = smem + cur * 2 * kTileBytes;
    const uint8_t* vl = kl + kTileBytes;

    // S^T = K . Q^T : two 32-key output tiles
    f32x16 s[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kt][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const typename T::vec8 a = lds_b128<T>(kl, k_off<D>(kt * 32 + l32, 2 * ks + half));
        s[kt] = T::mfma32(a, qf[ks], s[kt]);
      }
    }
    // scale, bias, tail mask, row max
    float mt = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        float x = s[kt][r] * p.c + bias;
        if (key >= src.klen) x = -INFINITY;
        s[kt][r] = x;
        mt = fmaxf(mt, x);
      }
    mt = max_xor32(mt);
    const float mn = fmaxf(m, mt);
    const float alpha = exp2_fast(m - mn);
    m = mn;
    float ls = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = exp2_fast(s[kt][r] - mn);
        s[kt][r] = e;
        ls += e;
      }
    l = l * alpha + ls;
#pragma unroll
    for (int i = 0; i < DT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[i][r] *= alpha;

    // O^T += V^T . P^T : 4 k-steps of 16 keys
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kt = kk >> 1, sp = kk & 1;
      const typename T::vec8 pf = pack8<T>(s[kt], 8 * sp);
      const int kb = kt * 32 + 16 * sp + 4 * half + (lane & 15) / 4;  // this lane's block row
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
        const s16x4 lo = lds_tr4(vl, v_off_bytes<D>(kb, col));
        const s16x4 hi = lds_tr4(vl, v_off_bytes<D>(kb + 8, col));
        o[dt] = T::mfma32(join8<T>(lo, hi), pf, o[dt]);
      }
    }

    if (t + 1 < ntiles) {
      uint8_t* kn = smem + (cur ^ 1) * 2 * kTileBytes;
      stage_store<D>(st, kn, kn + kTileBytes);
    }
    __syncthreads();
  }

  // ---- epilogue -----------------------------------------------------------------------------------
  const float lt = add_xor32(l);
  float inv = (lt > 0.f) ? 1.0f / lt : 0.f;
  if (nan_head) inv = __builtin_nanf("");
  if (qvalid) {
    uint8_t* obase = reinterpret_cast<uint8_t*>(p.out) +
                     2 * (b * p.os[0] + h * p.os[1] + (qrow0 + qrow) * p.os[2]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = dt * 32 + 8 * g4 + 4 * half;
        u32x2 w;
        w[0] = pack2<T>(o[dt][4 * g4 + 0] * inv, o[dt][4 * g4 + 1] * inv);
        w[1] = pack2<T>(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv);
        *reinterpret_cast<u32x2*>(obase + d * 2) = w;
      }
    if (p.lse && half == 0) {
      float v = (m + __log2f(lt)) * kLn2;
      if (nan_head) v = __builtin_nanf("");
      p.lse[b * p.lse_s[0] + h * p.lse_s[1] + (p.cu_q ? qg : qrow)] = v;
    }
  }
}

template <int D, class T>
static int launch_fwd(const FwdParams& p, bool pool, hipStream_t stream) {
  const dim3 grid(p.nbq * p.B * p.H);
  if (pool)
    hipLaunchKernelGGL((attn_fwd_kernel<D, T, true>), grid, dim3(kThreads), 0, stream, p);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<D, T, false>), grid, dim3(kThreads), 0, stream, p);
  return check_launch("attn_fwd_kernel");
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
  return dispatch_fwd(p, a->D, a->dtype, pool, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int vb_block_sparse_attn_fwd(const void* q_unpad, const void* k_unpad, const void* v_unpad,
                                        const int32_t* cu_seqlens_q, const int32_t* cu_seqlens_k,
                                        const int32_t* head_mask_type, const int32_t* streaming_info,
                                        const uint8_t* base_blockmask, int batch, int num_heads, int head_dim,
                                        int max_seqlen_q, int max_seqlen_k, float p_dropout, int deterministic,
                                        float softmax_scale, int is_causal, int exact_streaming, int dtype,
                                        void* out_unpad, float* softmax_lse, void* stream) {
  using namespace vb;
  (void)streaming_info;
  (void)deterministic;
  if (p_dropout != 0.f) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_fwd: p_dropout must be 0");
  if (is_causal || exact_streaming) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_fwd: causal/streaming not supported");
  if (!q_unpad || !k_unpad || !v_unpad || !cu_seqlens_q || !cu_seqlens_k || !out_unpad)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_fwd: null tensor");
  if (batch <= 0 || num_heads <= 0 || max_seqlen_q <= 0 || max_seqlen_k <= 0)
    return fail(VB_ERR_INVALID, "vb_block_sparse_attn_fwd: bad sizes");
  const int nbq = (max_seqlen_q + kQBlk - 1) / kQBlk;
  const int nbk = (max_seqlen_k + kQBlk - 1) / kQBlk;
  if (nbk > kMaxBlocks) return fail(VB_ERR_UNSUPPORTED, "vb_block_sparse_attn_fwd: max_seqlen_k too long");
  FwdParams p{};
  p.q = q_unpad; p.k = k_unpad; p.v = v_unpad;
  const int64_t row = (int64_t)num_heads * head_dim;
  p.qs[0] = p.ks[0] = p.vs[0] = p.os[0] = 0;
  p.qs[1] = p.ks[1] = p.vs[1] = p.os[1] = head_dim;
  p.qs[2] = p.ks[2] = p.vs[2] = p.os[2] = row;
  p.cu_q = cu_seqlens_q; p.cu_k = cu_seqlens_k;
  p.head_mask_type = head_mask_type;
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

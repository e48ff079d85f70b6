// Mask predictor, mean pooling and the reference-faithful LSE combine for gfx950.
//
// vb_mask_predict fuses, per (b, h) and group of four 32-row sampled q-blocks:
//   * efficient_attn_with_pooling: replicate pad + per-block token sampling
//     (cogvideox/train/special_attentions_local/TrainRelated/cogvideo_blocksparseattn.py:20-82),
//     done as row-index arithmetic on the caller's (un-reordered) q/k through the Gilbert rows;
//   * the Triton pooled-score kernel (TrainRelated/attn_pooling_kernel.py:17-255): per sampled row
//     the max logit of every 32-key sampled block (MFMA 32x32x16, query on the lane), rounded to the
//     storage dtype (R), the running fp32 row max m, then Po[i,j] = max_rows exp2(R - m) and the
//     storage-dtype row normalisation;
//   * transfer_attn_to_mask(mode="energy") (:177-249; wanx_blocksparseattn.py:162-233): stable
//     descending rank, fp32-accumulated cumsum rounded to the storage dtype per prefix, the first
//     crossing of storage(total * thr), clamp to [min_keep, max_keep], forced tail rows/cols.
// Nothing but Po and the mask reaches HBM (R stays in LDS).
#include "vb_common.hpp"

namespace vb {

constexpr int kPThreads = 256;
constexpr int kPWaves = 4;
constexpr int kMaxNb = 320;        // sampled blocks per side (L <= 40960 at block 128)
constexpr int kKeysPerTile = 64;   // two 32-key sampled blocks per LDS tile

struct PredParams {
  const void* q; const void* k;
  int64_t qs[3], ks[3];
  const int32_t* rows;
  const int32_t* q_off; const int32_t* k_off;
  int B, H, L, D, block, nb;
  float c;             // fp32(scale) * fp32(1.44269504), as the Triton kernel forms qk_scale
  float thr;
  int min_keep, max_keep, force_tail;
  void* po;
  uint8_t* mask;
  unsigned long long* count;
};

// caller row holding reordered-padded position `pos` of a (b,h) stream
__device__ __forceinline__ int sampled_row(int blk, int off, int block, int L, const int32_t* rows) {
  int pos = blk * block + off;
  pos = min(pos, L - 1);  // replicate padding (F.pad mode='replicate')
  return rows ? rows[pos] : pos;
}

// Energy rule on one row of nc normalised scores held (storage-rounded, as f32) in LDS `val`.
// `scratch` has room for nc floats. Executed by one full wave. Returns kept count via mask bytes.
template <class T>
__device__ int energy_row(const float* val, float* sorted, uint8_t* mrow, int nc, float thr,
                          int min_keep, int max_keep, int force_cols, bool force_all) {
  const int lane = threadIdx.x & 63;
  // stable descending rank: larger first, equal values lower index first
  int rank[kMaxNb / 64 + 1];
#pragma unroll
  for (int u = 0; u < kMaxNb / 64 + 1; ++u) {
    const int j = lane + 64 * u;
    rank[u] = 0;
    if (j < nc) {
      const float v = val[j];
      int rk = 0;
      for (int t = 0; t < nc; ++t) {
        const float w = val[t];
        rk += (w > v) || (w == v && t < j);
      }
      rank[u] = rk;
      sorted[rk] = v;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  int k = 0;
  if (lane == 0) {
    float acc = 0.f;
    for (int t = 0; t < nc; ++t) acc += sorted[t];
    const float total = round_to<T>(acc);
    const float th = round_to<T>(total * thr);
    acc = 0.f;
    k = nc;
    for (int t = 0; t < nc; ++t) {
      acc += sorted[t];
      if (round_to<T>(acc) >= th) { k = t; break; }
    }
    k = min(max(k, min_keep), max_keep);
  }
  k = __shfl(k, 0);
  int kept = 0;
#pragma unroll
  for (int u = 0; u < kMaxNb / 64 + 1; ++u) {
    const int j = lane + 64 * u;
    if (j < nc) {
      const bool keep = force_all || rank[u] < k || j >= nc - force_cols;
      mrow[j] = keep ? 1 : 0;
      kept += keep;
    }
  }
  // wave sum of kept
  for (int o = 32; o > 0; o >>= 1) kept += __shfl_xor(kept, o);
  return kept;
}

template <int D, class T>
__global__ void __launch_bounds__(kPThreads, 1) mask_predict_kernel(const PredParams p) {
  constexpr int KS = D / 16;
  constexpr int CH = D / 8;
  constexpr int kTileBytes = kKeysPerTile * D * 2;
  constexpr int kN = kKeysPerTile * CH / kPThreads;  // staged chunks per thread
  // LDS: R [4 waves][32 rows][nb] storage dtype | m [4][32] f32 | K tile x2 | row scratch
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int nb = p.nb;
  const int rstride = (nb + 7) & ~7;
  typename T::raw* R = reinterpret_cast<typename T::raw*>(smem);
  const int r_bytes = (kPWaves * 32 * rstride * 2 + 15) & ~15;
  float* mrow_s = reinterpret_cast<float*>(smem + r_bytes);
  uint8_t* ktile = smem + r_bytes + kPWaves * 32 * 4;
  float* rowbuf = reinterpret_cast<float*>(ktile + 2 * kTileBytes);  // [4][2][kMaxNb]

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int half = lane >> 5;
  const int l32 = lane & 31;
  const int bh = blockIdx.y;
  const int b = bh / p.H, h = bh % p.H;
  const int qb = blockIdx.x * kPWaves + wave;  // this wave's sampled q-block
  const bool wave_active = qb < nb;

  const uint8_t* qbase = reinterpret_cast<const uint8_t*>(p.q) + 2 * (b * p.qs[0] + h * p.qs[1]);
  const uint8_t* kbase = reinterpret_cast<const uint8_t*>(p.k) + 2 * (b * p.ks[0] + h * p.ks[1]);
  const int32_t* qoff = p.q_off + (int64_t)bh * 32;
  const int32_t* koff = p.k_off + (int64_t)bh * 32;

  // Q fragment of this lane's sampled row (B operand of S^T = K_s . Q_s^T)
  typename T::vec8 qf[KS];
  {
    const int row = sampled_row(wave_active ? qb : 0, qoff[l32], p.block, p.L, p.rows);
    const uint8_t* qp = qbase + (int64_t)row * 2 * p.qs[2];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      qf[s] = *reinterpret_cast<const typename T::vec8*>(qp + (16 * s + 8 * half) * 2);
  }
  float m = -INFINITY;

  const int ntiles = (nb + 1) / 2;
  u32x4 stg[kN];
  auto load = [&](int t) {
#pragma unroll
    for (int i = 0; i < kN; ++i) {
      const int c = threadIdx.x + i * kPThreads;
      const int r = c / CH, ch = c % CH;            // r: key within tile (0..63)
      const int blk = min(2 * t + (r >> 5), nb - 1);
      const int row = sampled_row(blk, koff[r & 31], p.block, p.L, p.rows);
      stg[i] = *reinterpret_cast<const u32x4*>(kbase + (int64_t)row * 2 * p.ks[2] + ch * 16);
    }
  };
  auto store = [&](uint8_t* dst) {
#pragma unroll
    for (int i = 0; i < kN; ++i) {
      const int c = threadIdx.x + i * kPThreads;
      const int r = c / CH, ch = c % CH;
      const int sw = (D == 64) ? ((r >> 1) & 7) : (r & 15);
      *reinterpret_cast<u32x4*>(dst + r * D * 2 + 16 * (ch ^ sw)) = stg[i];
    }
  };

  load(0);
  store(ktile);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntiles) load(t + 1);
    const uint8_t* kl = ktile + cur * kTileBytes;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      const int j = 2 * t + kt;
      f32x16 s;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int row = kt * 32 + l32;
        const int sw = (D == 64) ? ((row >> 1) & 7) : (row & 15);
        const typename T::vec8 a =
            *reinterpret_cast<const typename T::vec8*>(kl + row * D * 2 + 16 * ((2 * ks + half) ^ sw));
        s = T::mfma32(a, qf[ks], s);
      }
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[r]);
      mx = max_xor32(mx) * p.c;                       // tl.max(qk, 1) * qk_scale
      if (j < nb) {
        m = fmaxf(m, mx);
        if (half == kt) R[(wave * 32 + l32) * rstride + j] = T::from_f32(mx);
      }
    }
    if (t + 1 < ntiles) store(ktile + (cur ^ 1) * kTileBytes);
    __syncthreads();
  }
  if (half == 0) mrow_s[wave * 32 + l32] = m;
  __syncthreads();
  if (!wave_active) return;

  // Po[qb, j] = storage(max_r exp2(R[r][j] - m_r)); then storage-dtype row normalisation
  float* val = rowbuf + wave * 2 * kMaxNb;
  float* sorted = val + kMaxNb;
  const float* mw = mrow_s + wave * 32;
  const typename T::raw* Rw = R + wave * 32 * rstride;
  float part = 0.f;
  for (int j = lane; j < nb; j += 64) {
    float cm = 0.f;
    for (int r = 0; r < 32; ++r) cm = fmaxf(cm, exp2_fast(T::to_f32(Rw[r * rstride + j]) - mw[r]));
    cm = round_to<T>(cm);
    val[j] = cm;
    part += cm;
  }
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
  const float tot = round_to<T>(part);
  typename T::raw* po = reinterpret_cast<typename T::raw*>(p.po) + ((int64_t)bh * nb + qb) * nb;
  for (int j = lane; j < nb; j += 64) {
    const float v = round_to<T>(val[j] / tot);
    val[j] = v;
    po[j] = T::from_f32(v);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  uint8_t* mrow = p.mask + ((int64_t)bh * nb + qb) * nb;
  const bool force_all = p.force_tail > 0 && qb >= nb - p.force_tail;
  const int kept = energy_row<T>(val, sorted, mrow, nb, p.thr, p.min_keep, p.max_keep, p.force_tail, force_all);
  if (p.count && lane == 0) atomicAdd(p.count, (unsigned long long)kept);
}

template <class T>
__global__ void __launch_bounds__(256) energy_mask_kernel(const void* po, int rows_total, int nc, float thr,
                                                          int min_keep, int max_keep, int force_tail, int nr,
                                                          uint8_t* mask, unsigned long long* count) {
  __shared__ float buf[4][2 * kMaxNb];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows_total) return;
  const typename T::raw* src = reinterpret_cast<const typename T::raw*>(po) + (int64_t)row * nc;
  float* val = buf[wave];
  for (int j = lane; j < nc; j += 64) val[j] = T::to_f32(src[j]);
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  const int i = row % nr;
  const bool force_all = force_tail > 0 && i >= nr - force_tail;
  const int kept = energy_row<T>(val, val + kMaxNb, mask + (int64_t)row * nc, nc, thr, min_keep, max_keep,
                                 force_tail, force_all);
  if (count && lane == 0) atomicAdd(count, (unsigned long long)kept);
}

// simple_pooling of K and V: one thread per 16-byte chunk of a pooled row
template <class T>
__global__ void __launch_bounds__(256) pool_kv_kernel(const uint8_t* k, const uint8_t* v, int64_t ks0, int64_t ks1,
                                                      int64_t ks2, int64_t vs0, int64_t vs1, int64_t vs2,
                                                      const int32_t* rows, int B, int H, int L, int D, int gap,
                                                      int Lp, uint8_t* kp, uint8_t* vp) {
  const int CH = D / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)B * H * Lp * CH;
  if (idx >= total) return;
  const int ch = idx % CH;
  const int64_t prow = idx / CH;        // (b*H + h)*Lp + pr
  const int pr = prow % Lp;
  const int bh = prow / Lp;
  const int b = bh / H, h = bh % H;
  float ak[8], av[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ak[e] = av[e] = 0.f;
  for (int t = 0; t < gap; ++t) {
    int pos = min(pr * gap + t, L - 1);  // replicate padding
    if (rows) pos = rows[pos];
    const u32x4 xk = *reinterpret_cast<const u32x4*>(k + 2 * (b * ks0 + h * ks1 + (int64_t)pos * ks2) + ch * 16);
    const u32x4 xv = *reinterpret_cast<const u32x4*>(v + 2 * (b * vs0 + h * vs1 + (int64_t)pos * vs2) + ch * 16);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ak[2 * e] += T::bits_to_f32(xk[e] & 0xffff);
      ak[2 * e + 1] += T::bits_to_f32(xk[e] >> 16);
      av[2 * e] += T::bits_to_f32(xv[e] & 0xffff);
      av[2 * e + 1] += T::bits_to_f32(xv[e] >> 16);
    }
  }
  const float f = 1.0f / (float)gap;  // mean = sum * (1/N), as ATen's MeanOps
  u32x4 ok, ov;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ok[e] = pack2<T>(ak[2 * e] * f, ak[2 * e + 1] * f);
    ov[e] = pack2<T>(av[2 * e] * f, av[2 * e + 1] * f);
  }
  *reinterpret_cast<u32x4*>(kp + (prow * D + ch * 8) * 2) = ok;
  *reinterpret_cast<u32x4*>(vp + (prow * D + ch * 8) * 2) = ov;
}

// adaptive_block_sparse_attn's combine (cogvideo_blocksparseattn.py:374-393), eager-op rounding
template <class T>
__global__ void __launch_bounds__(256) lse_combine_kernel(const uint8_t* out1, const float* lse1, const uint8_t* out2,
                                                          const float* lse2, int64_t rows, int D, float gap,
                                                          uint8_t* out, float* alpha_out) {
  const int CH = D / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * CH) return;
  const int64_t row = idx / CH;
  const int ch = idx % CH;
  const float l1 = round_to<T>(lse1[row]);
  const float l2 = round_to<T>(lse2[row]);
  const float log_g = round_to<T>(logf(round_to<T>(gap)));
  const float w2 = round_to<T>(l2 + log_g);
  const float mx = fmaxf(l1, w2);
  const float e1 = round_to<T>(expf(round_to<T>(l1 - mx)));
  const float e2 = round_to<T>(expf(round_to<T>(w2 - mx)));
  const float a = round_to<T>(e1 / round_to<T>(e1 + e2));
  const float b = round_to<T>(1.0f - a);
  if (alpha_out && ch == 0) alpha_out[row] = a;
  const u32x4 x1 = *reinterpret_cast<const u32x4*>(out1 + (row * D + ch * 8) * 2);
  const u32x4 x2 = *reinterpret_cast<const u32x4*>(out2 + (row * D + ch * 8) * 2);
  u32x4 y;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float r[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const float v1 = T::bits_to_f32((x1[e] >> (16 * s)) & 0xffff);
      const float v2 = T::bits_to_f32((x2[e] >> (16 * s)) & 0xffff);
      r[s] = round_to<T>(round_to<T>(v1 * a) + round_to<T>(v2 * b));
    }
    y[e] = pack2<T>(r[0], r[1]);
  }
  *reinterpret_cast<u32x4*>(out + (row * D + ch * 8) * 2) = y;
}

static size_t predict_smem_bytes(int nb, int D) {
  const int rstride = (nb + 7) & ~7;
  const size_t r_bytes = ((size_t)kPWaves * 32 * rstride * 2 + 15) & ~size_t(15);
  return r_bytes + kPWaves * 32 * 4 + 2 * (size_t)kKeysPerTile * D * 2 + (size_t)kPWaves * 2 * kMaxNb * 4;
}

template <int D, class T>
static int launch_predict(const PredParams& p, hipStream_t stream) {
  const size_t smem = predict_smem_bytes(p.nb, D);
  auto kern = mask_predict_kernel<D, T>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)smem) != hipSuccess)
    return fail(VB_ERR_LAUNCH, "mask_predict: cannot reserve LDS");
  const dim3 grid((p.nb + kPWaves - 1) / kPWaves, p.B * p.H);
  hipLaunchKernelGGL(kern, grid, dim3(kPThreads), smem, stream, p);
  return check_launch("mask_predict_kernel");
}

}  // namespace vb

extern "C" int vb_mask_predict(const vb_predict_args* a, void* stream) {
  using namespace vb;
  if (!a || !a->q || !a->k || !a->q_off || !a->k_off || !a->po || !a->mask)
    return fail(VB_ERR_INVALID, "vb_mask_predict: null argument");
  if (a->B <= 0 || a->H <= 0 || a->L <= 0) return fail(VB_ERR_INVALID, "vb_mask_predict: bad sizes");
  if (a->block != 128 || a->num_keep != 32)
    return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: block must be 128 and num_keep 32 (the reference's values)");
  const int nb = (a->L + a->block - 1) / a->block;
  if (nb > kMaxNb) return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: sequence too long");
  if (a->min_keep < 1 || a->max_keep < 1) return fail(VB_ERR_INVALID, "vb_mask_predict: keep counts must be >= 1");
  for (int i = 0; i < 3; ++i)
    if ((a->q_stride[i] | a->k_stride[i]) & 7) return fail(VB_ERR_INVALID, "vb_mask_predict: strides must be multiples of 8");
  PredParams p{};
  p.q = a->q; p.k = a->k;
  for (int i = 0; i < 3; ++i) { p.qs[i] = a->q_stride[i]; p.ks[i] = a->k_stride[i]; }
  p.rows = a->rows; p.q_off = a->q_off; p.k_off = a->k_off;
  p.B = a->B; p.H = a->H; p.L = a->L; p.D = a->D; p.block = a->block; p.nb = nb;
  const float scale = a->scale > 0.f ? a->scale : (float)(1.0 / sqrt((double)a->D));
  p.c = scale * 1.44269504f;
  p.thr = a->energy_threshold;
  p.min_keep = a->min_keep; p.max_keep = a->max_keep; p.force_tail = a->force_tail;
  p.po = a->po; p.mask = a->mask; p.count = a->mask_count;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a->dtype == VB_DTYPE_BF16) {
    if (a->D == 64) return launch_predict<64, BF16>(p, s);
    if (a->D == 128) return launch_predict<128, BF16>(p, s);
  } else if (a->dtype == VB_DTYPE_F16) {
    if (a->D == 64) return launch_predict<64, F16>(p, s);
    if (a->D == 128) return launch_predict<128, F16>(p, s);
  } else {
    return fail(VB_ERR_INVALID, "vb_mask_predict: unknown dtype");
  }
  return fail(VB_ERR_UNSUPPORTED, "vb_mask_predict: head_dim must be 64 or 128");
}

extern "C" int vb_energy_mask(const void* po, int B, int H, int nr, int nc, float energy_threshold, int min_keep,
                              int max_keep, int force_tail, int dtype, uint8_t* mask,
                              unsigned long long* mask_count, void* stream) {
  using namespace vb;
  if (!po || !mask) return fail(VB_ERR_INVALID, "vb_energy_mask: null argument");
  if (B <= 0 || H <= 0 || nr <= 0 || nc <= 0) return fail(VB_ERR_INVALID, "vb_energy_mask: bad sizes");
  if (nc > kMaxNb) return fail(VB_ERR_UNSUPPORTED, "vb_energy_mask: too many columns");
  if (min_keep < 1 || max_keep < 1) return fail(VB_ERR_INVALID, "vb_energy_mask: keep counts must be >= 1");
  const int rows = B * H * nr;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((rows + 3) / 4);
  if (dtype == VB_DTYPE_BF16)
    hipLaunchKernelGGL(energy_mask_kernel<BF16>, grid, dim3(256), 0, s, po, rows, nc, energy_threshold, min_keep,
                       max_keep, force_tail, nr, mask, mask_count);
  else if (dtype == VB_DTYPE_F16)
    hipLaunchKernelGGL(energy_mask_kernel<F16>, grid, dim3(256), 0, s, po, rows, nc, energy_threshold, min_keep,
                       max_keep, force_tail, nr, mask, mask_count);
  else
    return fail(VB_ERR_INVALID, "vb_energy_mask: unknown dtype");
  return check_launch("energy_mask_kernel");
}

extern "C" int vb_pool_kv(const void* k, const void* v, const int64_t* k_stride, const int64_t* v_stride,
                          const int32_t* rows, int B, int H, int L, int D, int gap, int dtype, void* kp, void* vp,
                          void* stream) {
  using namespace vb;
  if (!k || !v || !k_stride || !v_stride || !kp || !vp) return fail(VB_ERR_INVALID, "vb_pool_kv: null argument");
  if (B <= 0 || H <= 0 || L <= 0 || gap <= 0 || D % 8) return fail(VB_ERR_INVALID, "vb_pool_kv: bad sizes");
  for (int i = 0; i < 3; ++i)
    if ((k_stride[i] | v_stride[i]) & 7) return fail(VB_ERR_INVALID, "vb_pool_kv: strides must be multiples of 8");
  const int Lp = (L + gap - 1) / gap;
  const int64_t total = (int64_t)B * H * Lp * (D / 8);
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto* kb = reinterpret_cast<const uint8_t*>(k);
  auto* vb_ = reinterpret_cast<const uint8_t*>(v);
  if (dtype == VB_DTYPE_BF16)
    hipLaunchKernelGGL(pool_kv_kernel<BF16>, grid, dim3(256), 0, s, kb, vb_, k_stride[0], k_stride[1], k_stride[2],
                       v_stride[0], v_stride[1], v_stride[2], rows, B, H, L, D, gap, Lp,
                       reinterpret_cast<uint8_t*>(kp), reinterpret_cast<uint8_t*>(vp));
  else if (dtype == VB_DTYPE_F16)
    hipLaunchKernelGGL(pool_kv_kernel<F16>, grid, dim3(256), 0, s, kb, vb_, k_stride[0], k_stride[1], k_stride[2],
                       v_stride[0], v_stride[1], v_stride[2], rows, B, H, L, D, gap, Lp,
                       reinterpret_cast<uint8_t*>(kp), reinterpret_cast<uint8_t*>(vp));
  else
    return fail(VB_ERR_INVALID, "vb_pool_kv: unknown dtype");
  return check_launch("pool_kv_kernel");
}

extern "C" int vb_lse_combine(const void* out1, const float* lse1, const void* out2, const float* lse2, int B, int H,
                              int L, int D, float gap, int dtype, void* out, float* alpha, void* stream) {
  using namespace vb;
  if (!out1 || !lse1 || !out2 || !lse2 || !out) return fail(VB_ERR_INVALID, "vb_lse_combine: null argument");
  if (B <= 0 || H <= 0 || L <= 0 || D % 8) return fail(VB_ERR_INVALID, "vb_lse_combine: bad sizes");
  const int64_t rows = (int64_t)B * H * L;
  const dim3 grid((unsigned)((rows * (D / 8) + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto* o1 = reinterpret_cast<const uint8_t*>(out1);
  auto* o2 = reinterpret_cast<const uint8_t*>(out2);
  auto* o = reinterpret_cast<uint8_t*>(out);
  if (dtype == VB_DTYPE_BF16)
    hipLaunchKernelGGL(lse_combine_kernel<BF16>, grid, dim3(256), 0, s, o1, lse1, o2, lse2, rows, D, gap, o, alpha);
  else if (dtype == VB_DTYPE_F16)
    hipLaunchKernelGGL(lse_combine_kernel<F16>, grid, dim3(256), 0, s, o1, lse1, o2, lse2, rows, D, gap, o, alpha);
  else
    return fail(VB_ERR_INVALID, "vb_lse_combine: unknown dtype");
  return check_launch("lse_combine_kernel");
}

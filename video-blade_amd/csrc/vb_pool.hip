// Mean pooling of K/V (fused with the Gilbert-ordered K/V copies) and the reference-faithful LSE
// combine for gfx950: the two HBM-bound element passes of the adaptive path.
//   simple_pooling (cogvideox/train/special_attentions_local/TrainRelated/cogvideo_blocksparseattn.py:83-88)
//   + the rearrange gathers (:148-150); the bf16 combine of adaptive_block_sparse_attn (:374-393).
#include <cstdlib>

#include "vb_pool.hpp"

namespace vb {

// simple_pooling of K and V (+ the Gilbert-ordered copies): pool_kv_span (vb_pool.hpp), grid-strided
template <class T>
__global__ void __launch_bounds__(256) pool_kv_kernel(const PoolTask t) {
  pool_kv_span<T>(t, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// Workgroups of an HBM-bound pass that runs beside the predictor's score kernel on another stream:
// a capped, grid-strided launch leaves most CUs to the MFMA-bound kernel instead of flooding the
// dispatcher (the build's VB_POOL_WGS_DEFAULT; 0 = one workgroup per 256 chunks).
unsigned pool_grid(int64_t work_items) {
  constexpr int cap = kPoolWgsDefault;
  const int64_t n = (work_items + 255) / 256;
  return (unsigned)((cap > 0 && n > cap) ? cap : n);
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

}  // namespace vb

extern "C" int vb_pool_kv(const void* k, const void* v, const int64_t* k_stride, const int64_t* v_stride,
                          const int32_t* rows, int B, int H, int L, int D, int gap, int dtype, void* kp, void* vp,
                          void* k_r, void* v_r, void* stream) {
  using namespace vb;
  if (!k || !v || !k_stride || !v_stride || !kp || !vp) return fail(VB_ERR_INVALID, "vb_pool_kv: null argument");
  if ((k_r == nullptr) != (v_r == nullptr)) return fail(VB_ERR_INVALID, "vb_pool_kv: give both k_r and v_r or neither");
  if (B <= 0 || H <= 0 || L <= 0 || gap <= 0 || D % 8) return fail(VB_ERR_INVALID, "vb_pool_kv: bad sizes");
  for (int i = 0; i < 3; ++i)
    if ((k_stride[i] | v_stride[i]) & 7) return fail(VB_ERR_INVALID, "vb_pool_kv: strides must be multiples of 8");
  PoolTask t{};
  t.k = reinterpret_cast<const uint8_t*>(k); t.v = reinterpret_cast<const uint8_t*>(v);
  for (int i = 0; i < 3; ++i) { t.ks[i] = k_stride[i]; t.vs[i] = v_stride[i]; }
  t.rows = rows; t.B = B; t.H = H; t.L = L; t.D = D; t.gap = gap; t.Lp = (L + gap - 1) / gap;
  t.kp = reinterpret_cast<uint8_t*>(kp); t.vp = reinterpret_cast<uint8_t*>(vp);
  t.k_r = reinterpret_cast<uint8_t*>(k_r); t.v_r = reinterpret_cast<uint8_t*>(v_r);
  const dim3 grid(pool_grid((int64_t)B * H * t.Lp * (D / 8)));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == VB_DTYPE_BF16)
    hipLaunchKernelGGL(pool_kv_kernel<BF16>, grid, dim3(256), 0, s, t);
  else if (dtype == VB_DTYPE_F16)
    hipLaunchKernelGGL(pool_kv_kernel<F16>, grid, dim3(256), 0, s, t);
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

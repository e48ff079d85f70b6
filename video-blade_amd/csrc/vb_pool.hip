// Mean pooling of K/V (fused with the Gilbert-ordered K/V copies) and the reference-faithful LSE
// combine for gfx950: the two HBM-bound element passes of the adaptive path.
//   simple_pooling (cogvideox/train/special_attentions_local/TrainRelated/cogvideo_blocksparseattn.py:83-88)
//   + the rearrange gathers (:148-150); the bf16 combine of adaptive_block_sparse_attn (:374-393).
#include <cstdlib>

#include "vb_common.hpp"

namespace vb {

// simple_pooling of K and V: one thread per 16-byte chunk of a pooled row. Every reordered row
// is read by exactly one thread, which (when k_r/v_r are given) also writes it to the contiguous
// Gilbert-ordered copies the attention kernel streams (the reference's index_select, fused).
template <class T>
__global__ void __launch_bounds__(256) pool_kv_kernel(const uint8_t* k, const uint8_t* v, int64_t ks0, int64_t ks1,
                                                      int64_t ks2, int64_t vs0, int64_t vs1, int64_t vs2,
                                                      const int32_t* rows, int B, int H, int L, int D, int gap,
                                                      int Lp, uint8_t* kp, uint8_t* vp, uint8_t* k_r,
                                                      uint8_t* v_r) {
  const int CH = D / 8;
  const int64_t total = (int64_t)B * H * Lp * CH;
  // grid-stride: the launch may use fewer workgroups than chunks (see pool_grid below)
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
  const int ch = idx % CH;
  const int64_t prow = idx / CH;        // (b*H + h)*Lp + pr
  const int pr = prow % Lp;
  const int bh = prow / Lp;
  const int b = bh / H, h = bh % H;
  float ak[8], av[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) ak[e] = av[e] = 0.f;
  for (int t = 0; t < gap; ++t) {
    const int g = pr * gap + t;
    int pos = min(g, L - 1);  // replicate padding
    if (rows) pos = rows[pos];
    const u32x4 xk = *reinterpret_cast<const u32x4*>(k + 2 * (b * ks0 + h * ks1 + (int64_t)pos * ks2) + ch * 16);
    const u32x4 xv = *reinterpret_cast<const u32x4*>(v + 2 * (b * vs0 + h * vs1 + (int64_t)pos * vs2) + ch * 16);
    if (k_r && g < L) {
      const int64_t o = ((int64_t)bh * L + g) * D * 2 + ch * 16;
      *reinterpret_cast<u32x4*>(k_r + o) = xk;
      *reinterpret_cast<u32x4*>(v_r + o) = xv;
    }
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
}

// Workgroups of an HBM-bound pass that runs beside the predictor's score kernel on another stream:
// a capped, grid-strided launch leaves most CUs to the MFMA-bound kernel instead of flooding the
// dispatcher (VB_POOL_WGS overrides; 0 = one workgroup per 256 chunks).
unsigned pool_grid(int64_t work_items) {
  static const int cap = [] {
    const char* e = getenv("VB_POOL_WGS");
    return e ? atoi(e) : kPoolWgsDefault;
  }();
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
  const int Lp = (L + gap - 1) / gap;
  const int64_t total = (int64_t)B * H * Lp * (D / 8);
  const dim3 grid(pool_grid(total));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto* kb = reinterpret_cast<const uint8_t*>(k);
  auto* vb_ = reinterpret_cast<const uint8_t*>(v);
  if (dtype == VB_DTYPE_BF16)
    hipLaunchKernelGGL(pool_kv_kernel<BF16>, grid, dim3(256), 0, s, kb, vb_, k_stride[0], k_stride[1], k_stride[2],
                       v_stride[0], v_stride[1], v_stride[2], rows, B, H, L, D, gap, Lp,
                       reinterpret_cast<uint8_t*>(kp), reinterpret_cast<uint8_t*>(vp),
                       reinterpret_cast<uint8_t*>(k_r), reinterpret_cast<uint8_t*>(v_r));
  else if (dtype == VB_DTYPE_F16)
    hipLaunchKernelGGL(pool_kv_kernel<F16>, grid, dim3(256), 0, s, kb, vb_, k_stride[0], k_stride[1], k_stride[2],
                       v_stride[0], v_stride[1], v_stride[2], rows, B, H, L, D, gap, Lp,
                       reinterpret_cast<uint8_t*>(kp), reinterpret_cast<uint8_t*>(vp),
                       reinterpret_cast<uint8_t*>(k_r), reinterpret_cast<uint8_t*>(v_r));
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

// Multi-level path helpers (gfx950): the KV pyramid and the rank-band level mask.
//
// Reference: cogvideox/sample_evaluate/Triton/kernels/block_sparse_attn_kernel_with_backward_9_10.py
// (_forward :1311-1320 builds k_2/k_4/k_8 with pad_to_multiple :1239-1250 and pooling :1252-1270)
// and cogvideox/sample_evaluate/Triton/cogvideo_newattn.py transfer_attn_to_mask (:154-207).
#include "vb_common.hpp"
#include "vb_pyr.hpp"

namespace vb {

// ---- KV pyramid ---------------------------------------------------------------------------------
// The stand-alone launch of kv_pyramid_span (vb_pyr.hpp), grid-strided (pool_grid).
template <int D, class T>
__global__ void __launch_bounds__(256) kv_pyramid_kernel(const PyrTask t) {
  kv_pyramid_span<D, T>(t, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// ---- level mask ----------------------------------------------------------------------------------
// One wave per score row. Each score's 16-bit storage pattern is mapped to an order-preserving
// key and packed with its inverted column index, so key_i > key_j <=> (po_i > po_j) or (equal and
// i < j): the stable descending rank of column j is the number of larger keys in the row.
constexpr int kLmMaxBands = 8;
struct LevelBands {
  int n;
  int value[kLmMaxBands];
  int start[kLmMaxBands];
  int end[kLmMaxBands];
};

template <class T>
__device__ __forceinline__ uint32_t order_key16(uint16_t u) {
  // IEEE-like 16-bit float (bf16 / fp16): flip all bits of negatives, the sign bit of positives
  return (u & 0x8000u) ? (uint32_t)(~u & 0xFFFFu) : (uint32_t)(u | 0x8000u);
}

template <class T>
__global__ void __launch_bounds__(256) level_mask_kernel(const uint16_t* __restrict__ po, int rows_total, int nr, int nc,
                                                         LevelBands bands, uint8_t* __restrict__ mask) {
  extern __shared__ uint32_t keys_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows_total) return;
  uint32_t* keys = keys_lds + wave * nc;
  const uint16_t* src = po + (int64_t)row * nc;
  for (int j = lane; j < nc; j += 64) keys[j] = (order_key16<T>(src[j]) << 16) | (uint32_t)(0xFFFF - j);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int i = row % nr;
  uint8_t* dst = mask + (int64_t)row * nc;
  for (int j = lane; j < nc; j += 64) {
    const uint32_t kj = keys[j];
    int rank = 0;
    for (int t = 0; t < nc; ++t) rank += keys[t] > kj;
    int lv = 0;
    for (int bnd = 0; bnd < bands.n; ++bnd)
      if (rank >= bands.start[bnd] && rank < bands.end[bnd]) lv = bands.value[bnd];
    if (j >= nc - 2 || i >= nr - 2) lv = 1;
    dst[j] = (uint8_t)lv;
  }
}

}  // namespace vb

extern "C" int vb_kv_pyramid(const void* k, const void* v, const int64_t* k_stride, const int64_t* v_stride,
                             const int32_t* rows, int B, int H, int L, int D, int dtype, void* kpyr, void* vpyr,
                             void* stream) {
  using namespace vb;
  if (!k || !v || !k_stride || !v_stride || !kpyr || !vpyr) return fail(VB_ERR_INVALID, "vb_kv_pyramid: null argument");
  if (B <= 0 || H <= 0 || L <= 0) return fail(VB_ERR_INVALID, "vb_kv_pyramid: B, H, L must be positive");
  if (D != 64 && D != 128) return fail(VB_ERR_UNSUPPORTED, "vb_kv_pyramid: head_dim must be 64 or 128");
  for (int i = 0; i < 3; ++i)
    if ((k_stride[i] | v_stride[i]) & 7) return fail(VB_ERR_INVALID, "vb_kv_pyramid: strides must be multiples of 8 elements");
  if (((reinterpret_cast<uintptr_t>(k) | reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(kpyr) |
        reinterpret_cast<uintptr_t>(vpyr)) & 15) != 0)
    return fail(VB_ERR_INVALID, "vb_kv_pyramid: tensors must be 16-byte aligned");
  const int Lpad = (L + 127) / 128 * 128;
  const int64_t total = (int64_t)B * H * (Lpad / 8) * (D / 8);
  const dim3 grid(pool_grid(total));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  PyrTask t{};
  t.k = static_cast<const uint8_t*>(k); t.v = static_cast<const uint8_t*>(v);
  for (int i = 0; i < 3; ++i) { t.ks[i] = k_stride[i]; t.vs[i] = v_stride[i]; }
  t.rows = rows; t.B = B; t.H = H; t.L = L; t.Lpad = Lpad;
  t.kpyr = static_cast<uint8_t*>(kpyr); t.vpyr = static_cast<uint8_t*>(vpyr);
#define VB_PYR(DD, TT) hipLaunchKernelGGL((kv_pyramid_kernel<DD, TT>), grid, dim3(256), 0, st, t)
  if (dtype == VB_DTYPE_BF16) {
    if (D == 64) VB_PYR(64, BF16); else VB_PYR(128, BF16);
  } else if (dtype == VB_DTYPE_F16) {
    if (D == 64) VB_PYR(64, F16); else VB_PYR(128, F16);
  } else {
    return fail(VB_ERR_INVALID, "vb_kv_pyramid: unknown dtype");
  }
#undef VB_PYR
  return check_launch("kv_pyramid_kernel");
}

extern "C" int vb_level_mask(const void* po, int B, int H, int nr, int nc, int n_bands, const int32_t* band_value,
                             const double* band_start, const double* band_end, int dtype, uint8_t* mask,
                             void* stream) {
  using namespace vb;
  if (!po || !mask) return fail(VB_ERR_INVALID, "vb_level_mask: null tensor");
  if (B <= 0 || H <= 0 || nr <= 0 || nc <= 0) return fail(VB_ERR_INVALID, "vb_level_mask: sizes must be positive");
  if (nc > 4096) return fail(VB_ERR_UNSUPPORTED, "vb_level_mask: nc > 4096");
  if (n_bands < 0 || n_bands > kLmMaxBands || (n_bands > 0 && (!band_value || !band_start || !band_end)))
    return fail(VB_ERR_INVALID, "vb_level_mask: 0..8 bands with value/start/end arrays");
  LevelBands bands{};
  bands.n = n_bands;
  for (int i = 0; i < n_bands; ++i) {
    const int val = band_value[i];
    if (val != 0 && val != 1 && val != 2 && val != 4 && val != 8)
      return fail(VB_ERR_INVALID, "vb_level_mask: band values must be 0, 1, 2, 4 or 8");
    bands.value[i] = val;
    // max(0, int(seq * start)), min(seq, int(seq * end)) in double, as the reference's Python
    double a = (double)nc * band_start[i], b = (double)nc * band_end[i];
    int ia = (int)a, ib = (int)b;   // truncation toward zero, as int()
    bands.start[i] = ia < 0 ? 0 : ia;
    bands.end[i] = ib > nc ? nc : ib;
  }
  const int rows_total = B * H * nr;
  const dim3 grid((rows_total + 3) / 4);
  const size_t lds = (size_t)4 * nc * sizeof(uint32_t);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint16_t* p = static_cast<const uint16_t*>(po);
  if (dtype == VB_DTYPE_BF16)
    hipLaunchKernelGGL((level_mask_kernel<BF16>), grid, dim3(256), lds, st, p, rows_total, nr, nc, bands, mask);
  else if (dtype == VB_DTYPE_F16)
    hipLaunchKernelGGL((level_mask_kernel<F16>), grid, dim3(256), lds, st, p, rows_total, nr, nc, bands, mask);
  else
    return fail(VB_ERR_INVALID, "vb_level_mask: unknown dtype");
  return check_launch("level_mask_kernel");
}

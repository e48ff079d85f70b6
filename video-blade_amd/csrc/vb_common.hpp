// Shared device/host helpers for the Video-BLADE MI355X (gfx950) attention library.
// Wave64 throughout; MFMA v_mfma_f32_32x32x16_{bf16,f16}; no CUDA idioms.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "vblade.h"

namespace vb {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ---------------------------------------------------------------- element types
struct BF16 {
  using raw = __bf16;
  using vec8 = bf16x8;
  static __device__ __forceinline__ float to_f32(raw x) { return static_cast<float>(x); }
  static __device__ __forceinline__ raw from_f32(float x) { return static_cast<raw>(x); }
  static __device__ __forceinline__ f32x16 mfma32(vec8 a, vec8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mfma16(vec8 a, vec8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  // bit pattern of a 16-bit element -> f32
  static __device__ __forceinline__ float bits_to_f32(uint16_t u) {
    return __uint_as_float(static_cast<uint32_t>(u) << 16);
  }
};

struct F16 {
  using raw = _Float16;
  using vec8 = f16x8;
  static __device__ __forceinline__ float to_f32(raw x) { return static_cast<float>(x); }
  static __device__ __forceinline__ raw from_f32(float x) { return static_cast<raw>(x); }
  static __device__ __forceinline__ f32x16 mfma32(vec8 a, vec8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f32x4 mfma16(vec8 a, vec8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ float bits_to_f32(uint16_t u) {
    _Float16 h;
    __builtin_memcpy(&h, &u, 2);
    return static_cast<float>(h);
  }
};

// round an f32 to the storage type and back (emulates a store/load in that dtype)
template <class T>
__device__ __forceinline__ float round_to(float x) {
  return T::to_f32(T::from_f32(x));
}

// pack two f32 into one dword of two 16-bit elements (lo = a), round-to-nearest-even;
// __builtin_convertvector lowers to ONE v_cvt_pk_bf16_f32 (two scalar casts + or would be three)
template <class T>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef typename T::raw r2 __attribute__((ext_vector_type(2)));
  const f32x2 x = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, r2));
}

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// symmetric combine of lane l with lane l^32 (v_permlane32_swap; no LDS)
__device__ __forceinline__ float max_xor32(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float add_xor32(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }

// ---------------------------------------------------------------- HBM passes beside the predictor
#ifndef VB_POOL_WGS_DEFAULT
#define VB_POOL_WGS_DEFAULT 0
#endif
constexpr int kPoolWgsDefault = VB_POOL_WGS_DEFAULT;
unsigned pool_grid(int64_t work_items);   // vb_pool.hip

// ---------------------------------------------------------------- persistent work queues (ABI 4)
// The caller's int32[VB_WORK_QUEUE_INTS] queue: heads 0-7 per XCD (work item v is in queue v % 8),
// word kWqDone the finished workgroups. Words are 128 bytes apart. The last workgroup to finish a
// launch zeroes every word (wq_finish), so each launch finds the queue at zero.
constexpr int kWqStride = 32;
constexpr int kWqDone = 8 * kWqStride;
static_assert(kWqDone < VB_WORK_QUEUE_INTS, "work queue words");
__device__ __forceinline__ int wq_pop(int* wq, int word) {
  return __hip_atomic_fetch_add(wq + word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// next item of a per-XCD queue set over `total` items: the home XCD's queue first, then the others'
__device__ __forceinline__ int wq_fetch(int* wq, int home, int total) {
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    const int x = (home + i) & 7;
    const int cnt = (total - x + 7) >> 3;   // items x, x + 8, x + 16, ...
    if (cnt > 0) {
      const int j = wq_pop(wq, x * kWqStride);
      if (j < cnt) return x + 8 * j;
    }
  }
  return -1;
}
// called once per workgroup by one thread, after its last (failed) fetch has returned
__device__ __forceinline__ void wq_finish(int* wq) {
  const int done = wq_pop(wq, kWqDone);
  if (done == (int)gridDim.x - 1)
    for (int x = 0; x <= kWqDone / kWqStride; ++x)
      __hip_atomic_store(wq + x * kWqStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// resident workgroups of `kernel` at `smem` bytes of dynamic LDS on the current device (host; no sync)
int resident_grid(const void* kernel, int threads, size_t smem);

// ---------------------------------------------------------------- host error plumbing
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int check_launch(const char* what);

}  // namespace vb

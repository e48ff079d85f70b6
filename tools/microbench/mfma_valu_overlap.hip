// Microbenchmark: do MFMAs of one wave and the exp/add VALU stream of another wave on the same SIMD
// overlap on gfx950? (the D=64 attention forward looked serialised.)
//
// One 512-thread workgroup per CU (8 waves, two per SIMD: waves w and w+4 share one). Modes:
//   mfma   waves 0-3: N x 16 v_mfma_f32_32x32x16_bf16 (4 independent accumulators); waves 4-7 exit
//   valu   waves 0-3: N x (32 v_exp_f32 + 32 v_add_f32 + 16 v_cvt_pk_bf16_f32); waves 4-7 exit
//   both   waves 0-3 the MFMA stream, waves 4-7 the VALU stream, concurrently
//   mixed  waves 0-3 alone, each iteration interleaving the MFMA group and the VALU group in one wave
// Overlap shows as t(both) close to max(t(mfma), t(valu)); serialisation as t(both) ~ t(mfma) + t(valu).
// The per-iteration instruction mix is the attention forward's per 64-key tile at D=64.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o mfma_valu_overlap mfma_valu_overlap.hip
// Run:   ./mfma_valu_overlap [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void mfma_group(f32x16 (&acc)[4], bf16x8 a, bf16x8 b) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
}

__device__ __forceinline__ void valu_group(float (&x)[32], float& sum, uint32_t& pk) {
  // x is made opaque every iteration (no instruction), so the exps cannot be hoisted
#pragma unroll
  for (int r = 0; r < 32; ++r) asm volatile("" : "+v"(x[r]));
  float e[32];
#pragma unroll
  for (int r = 0; r < 32; ++r) e[r] = __builtin_amdgcn_exp2f(x[r]);
  float h[4] = {e[0], e[1], e[2], e[3]};
#pragma unroll
  for (int r = 4; r < 32; ++r) h[r & 3] += e[r];
  sum += (h[0] + h[1]) + (h[2] + h[3]);
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const f32x2 v = {e[2 * w], e[2 * w + 1]};
    const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
    asm volatile("" :: "v"(u));   // keep the pack (no instruction)
  }
  (void)pk;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
// the same FLOPs as mfma_group with v_mfma_f32_16x16x32_bf16: 32 instructions of 16 cycles
__device__ __forceinline__ void mfma16_group(f32x4 (&acc)[8], bf16x8 a, bf16x8 b) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
}

// modes 4 (16x16x32 alone), 5 (16x16x32 + VALU in one wave), 6 (16x16x32 and VALU in two waves)
template <int kMode>
__global__ void __launch_bounds__(512, 1) overlap16_kernel(int iters, float* out) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const bool grp_mfma = wave < 4;
  float res = 0.f;
  if (grp_mfma) {
    bf16x8 a, b;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] = (__bf16)(0.01f * (lane + e));
      b[e] = (__bf16)(0.02f * (lane - e));
    }
    f32x4 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[j][r] = 0.f;
    float x[32];
    float sum = 0.f;
    uint32_t pk = 0;
#pragma unroll
    for (int r = 0; r < 32; ++r) x[r] = -0.01f * (r + lane);
    for (int it = 0; it < iters; ++it) {
      mfma16_group(acc, a, b);
      if (kMode == 5) valu_group(x, sum, pk);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) res += acc[j][r];
    res += sum;
  }
  if (kMode == 6 && !grp_mfma) {
    float x[32];
    float sum = 0.f;
    uint32_t pk = 0;
#pragma unroll
    for (int r = 0; r < 32; ++r) x[r] = -0.01f * (r + lane);
    for (int it = 0; it < iters; ++it) valu_group(x, sum, pk);
    res += sum;
  }
  out[blockIdx.x * 512 + threadIdx.x] = res;
}

template <int kMode>
__global__ void __launch_bounds__(512, 1) overlap_kernel(int iters, float* out) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const bool grp_mfma = wave < 4;
  float res = 0.f;
  if ((kMode == 0 || kMode == 2 || kMode == 3) && grp_mfma) {
    bf16x8 a, b;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] = (__bf16)(0.01f * (lane + e));
      b[e] = (__bf16)(0.02f * (lane - e));
    }
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    float x[32];
    float sum = 0.f;
    uint32_t pk = 0;
#pragma unroll
    for (int r = 0; r < 32; ++r) x[r] = -0.01f * (r + lane);
    for (int it = 0; it < iters; ++it) {
      mfma_group(acc, a, b);
      if (kMode == 3) valu_group(x, sum, pk);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) res += acc[j][r];
    res += sum + (float)(pk & 1);
  }
  if ((kMode == 1 && grp_mfma) || (kMode == 2 && !grp_mfma)) {
    float x[32];
    float sum = 0.f;
    uint32_t pk = 0;
#pragma unroll
    for (int r = 0; r < 32; ++r) x[r] = -0.01f * (r + lane);
    for (int it = 0; it < iters; ++it) valu_group(x, sum, pk);
    res += sum + (float)(pk & 1);
  }
  out[blockIdx.x * 512 + threadIdx.x] = res;
}

template <int kMode>
static float run16(int iters, float* d_out, int nwg) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(overlap16_kernel<kMode>, dim3(nwg), dim3(512), 0, 0, iters, d_out);   // warm
  (void)hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(overlap16_kernel<kMode>, dim3(nwg), dim3(512), 0, 0, iters, d_out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

template <int kMode>
static float run(int iters, float* d_out, int nwg) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(overlap_kernel<kMode>, dim3(nwg), dim3(512), 0, 0, iters, d_out);   // warm
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(overlap_kernel<kMode>, dim3(nwg), dim3(512), 0, 0, iters, d_out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int nwg = ncu;   // one 8-wave workgroup per CU
  float* d_out = nullptr;
  hipMalloc(&d_out, sizeof(float) * nwg * 512);
  const float tm = run<0>(iters, d_out, nwg);
  const float tv = run<1>(iters, d_out, nwg);
  const float tb = run<2>(iters, d_out, nwg);
  const float tx = run<3>(iters, d_out, nwg);
  const float t16 = run16<4>(iters, d_out, nwg);
  const float t16x = run16<5>(iters, d_out, nwg);
  const float t16b = run16<6>(iters, d_out, nwg);
  printf("{\"iters\": %d, \"mfma16_ms\": %.4f, \"mfma16_mixed_one_wave_ms\": %.4f, "
         "\"mfma16_both_two_waves_ms\": %.4f, \"mfma16_over_mfma32\": %.3f, \"mixed16_over_mixed32\": %.3f}\n",
         iters, t16, t16x, t16b, t16 / tm, t16x / tx);
  // per iteration and SIMD: 16 MFMAs (512 matrix cycles at 32 each) vs 80 VALU
  printf("{\"iters\": %d, \"cus\": %d, \"mfma_ms\": %.4f, \"valu_ms\": %.4f, \"both_two_waves_ms\": %.4f, "
         "\"mixed_one_wave_ms\": %.4f, \"both_over_max\": %.3f, \"both_over_sum\": %.3f, "
         "\"mixed_over_sum\": %.3f}\n",
         iters, ncu, tm, tv, tb, tx, tb / (tm > tv ? tm : tv), tb / (tm + tv), tx / (tm + tv));
  hipFree(d_out);
  return 0;
}

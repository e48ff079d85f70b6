// Microbenchmark: what a one-wave-per-SIMD MFMA stream pays for fillers placed in its gaps (gfx950).
//
// One 256-thread workgroup per CU (4 waves, one per SIMD), every wave the same loop: per iteration
// 16 v_mfma_f32_32x32x16_bf16 with a fixed set of fillers pinned after each MFMA by sched_barrier
// (the structure of the round-4 one-wave-per-SIMD forward experiment, removed from the library in round 5; profiles/archive/r04_fwd1_experiments.md). Modes vary the
// accumulator chaining and the filler mix:
//   acc:   1 = one dependent chain, 2 = two alternating, 4 = four round-robin
//   fill:  0 = none, 1 = 2 v_exp_f32, 2 = 2 v_add_f32 + 1 v_cvt_pk, 3 = 2 exp + 2 add + 1 pack,
//          4 = 1 exp + 2 add + 1 pack, 5 = 3 + two ds_read_b128
// Prints ns per MFMA per SIMD and the cycles at the clock passed as argv[2] (GHz).
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_gap_fill tools/microbench/mfma_gap_fill.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));

template <int kAcc, int kFill>
__global__ void __launch_bounds__(256, 1) gapfill(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[96 * 1024];   // one workgroup per CU
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (lane + i));
    b[i] = (__bf16)(0.002f * (lane - i));
  }
  f32x16 acc[4];
  for (int j = 0; j < 4; ++j)
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float x[32];
  for (int r = 0; r < 32; ++r) x[r] = 0.01f * (r - lane);
  float h[4] = {0.f, 0.f, 0.f, 0.f};
  uint32_t pk = 0;
  bf16x8 rd[2];
  rd[0] = rd[1] = a;
  const int off = (lane * 16) & 0x3FFF;
  if (threadIdx.x == 0) lds[0] = 0;
  __syncthreads();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 32; ++r) asm volatile("" : "+v"(x[r]));
    float e[32];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int j = kAcc == 1 ? 0 : (kAcc == 2 ? (g & 1) : (g & 3));
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, (g & 1) ? b : rd[g & 1], acc[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (kFill == 1 || kFill == 3 || kFill == 5) {
        e[2 * g] = __builtin_amdgcn_exp2f(x[2 * g]);
        e[2 * g + 1] = __builtin_amdgcn_exp2f(x[2 * g + 1]);
      }
      if (kFill == 4) {
        e[2 * g] = __builtin_amdgcn_exp2f(x[2 * g]);
        e[2 * g + 1] = x[2 * g + 1];
      }
      if (kFill == 2) {
        e[2 * g] = x[2 * g];
        e[2 * g + 1] = x[2 * g + 1];
      }
      if (kFill >= 2 && g > 0) {
        h[(2 * g) & 3] += e[2 * g - 2];
        h[(2 * g + 1) & 3] += e[2 * g - 1];
        const f32x2 v = {e[2 * g - 2], e[2 * g - 1]};
        pk ^= __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b2));
        asm volatile("" : "+v"(pk));
      }
      if (kFill == 5) {
        rd[g & 1] = *reinterpret_cast<const bf16x8*>(lds + ((off + 1024 * g) & 0x7FFF));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (kFill == 1) h[0] += e[0] + e[31];
  }
  float s = h[0] + h[1] + h[2] + h[3] + (float)pk;
  for (int j = 0; j < 4; ++j) s += acc[j][0];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int kAcc, int kFill>
static float run(float* out, int cus, int iters) {
  hipLaunchKernelGGL((gapfill<kAcc, kFill>), dim3(cus), dim3(256), 0, 0, out, iters);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((gapfill<kAcc, kFill>), dim3(cus), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const double ghz = argc > 2 ? atof(argv[2]) : 2.1;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  hipMalloc(&out, sizeof(float) * 256 * cus);
  const char* fills[] = {"none", "2 exp", "2 add + pack", "2 exp + 2 add + pack", "1 exp + 2 add + pack",
                         "2 exp + 2 add + pack + 2 ds_read_b128"};
  float t[3][6];
#define ROW(A, AI)                   \
  t[AI][0] = run<A, 0>(out, cus, iters); \
  t[AI][1] = run<A, 1>(out, cus, iters); \
  t[AI][2] = run<A, 2>(out, cus, iters); \
  t[AI][3] = run<A, 3>(out, cus, iters); \
  t[AI][4] = run<A, 4>(out, cus, iters); \
  t[AI][5] = run<A, 5>(out, cus, iters);
  ROW(1, 0)
  ROW(2, 1)
  ROW(4, 2)
  const int accs[3] = {1, 2, 4};
  printf("{\"iters\": %d, \"cus\": %d, \"ghz_assumed\": %.2f, \"rows\": [\n", iters, cus, ghz);
  for (int ai = 0; ai < 3; ++ai)
    for (int f = 0; f < 6; ++f) {
      const double ns = t[ai][f] * 1e6 / (5.0 * 0 + 1) / ((double)iters * 16);
      printf("  {\"acc\": %d, \"fill\": \"%s\", \"ms\": %.4f, \"ns_per_mfma\": %.3f, \"cycles_per_mfma\": %.1f}%s\n",
             accs[ai], fills[f], t[ai][f], ns, ns * ghz, (ai == 2 && f == 5) ? "" : ",");
    }
  printf("]}\n");
  hipFree(out);
  return 0;
}

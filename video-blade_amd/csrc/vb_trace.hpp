// Diagnostic-only per-workgroup timeline (never in the product build): start time, the end time of
// every wave, HW_ID, XCC_ID, a kind tag, and the shader-clock cycles over the workgroup, so a tool
// can see dispatch, residency per CU, workgroup lengths, the tail and the clock
// (tools/diag/pred_trace.py, tools/diag/attn_trace.py). Times are s_memrealtime ticks (100 MHz).
#pragma once
#include <hip/hip_runtime.h>

namespace vb {

constexpr int kTraceWgs = 8192;
constexpr int kTraceF = 10;   // start, end of waves 0-3, HW_ID, XCC_ID, kind, clk start, clk end (wave 0)
struct TraceBuf {
  unsigned long long v[kTraceWgs][kTraceF];
};

__device__ __forceinline__ unsigned long long trace_now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned long long trace_clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
// `row`: the workgroup's record (its blockIdx, or the work item a persistent workgroup is running)
__device__ __forceinline__ void trace_start(TraceBuf& b, int kind, unsigned row = blockIdx.x) {
  if (row < kTraceWgs && threadIdx.x == 0) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    b.v[row][0] = trace_now();
    b.v[row][5] = hw;
    b.v[row][6] = xcc;
    b.v[row][7] = kind;
    b.v[row][8] = trace_clk();
  }
}
__device__ __forceinline__ void trace_end(TraceBuf& b, unsigned row = blockIdx.x) {
  if (row < kTraceWgs && (threadIdx.x & 63) == 0) {
    b.v[row][1 + (threadIdx.x >> 6)] = trace_now();
    if (threadIdx.x == 0) b.v[row][9] = trace_clk();
  }
}

}  // namespace vb

// host side: copy out n rows and clear the buffer
#define VB_TRACE_GETTER(fn, sym)                                                                   \
  extern "C" int fn(unsigned long long* out, int n) {                                              \
    const size_t rows = (size_t)(n < vb::kTraceWgs ? n : vb::kTraceWgs);                          \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sym), sizeof(unsigned long long) * vb::kTraceF * rows) \
        != hipSuccess)                                                                             \
      return -1;                                                                                   \
    static vb::TraceBuf z;                                                                         \
    return hipMemcpyToSymbol(HIP_SYMBOL(sym), &z, sizeof(z)) == hipSuccess ? 0 : -1;               \
  }

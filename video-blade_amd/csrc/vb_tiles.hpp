// MFMA / LDS tile idioms shared by the attention forward and backward kernels (gfx950).
//
// v_mfma_f32_32x32x16 operand maps (wave64), used throughout:
//   A [32 x 16]: lane l supplies row (l & 31), k = 8*(l >> 5) + 0..7   (one 16-byte vector)
//   B [16 x 32]: lane l supplies column (l & 31), k = 8*(l >> 5) + 0..7
//   C [32 x 32]: lane l holds column (l & 31), register r holds row (r&3) + 8*(r>>2) + 4*(l>>5)
// A C tile re-used as the B operand of the next MFMA (pack8: registers 8s..8s+7 -> one vector)
// delivers its rows in the order rho(k) = 16s + 8*((k>>2)&1) + (k&3) + 4*(k>>3); the matching A
// operand is fetched with ds_read_b64_tr_b16 at rows (16s + 4h + q) and (+8): see tr_row().
#pragma once
#include "vb_common.hpp"

namespace vb {

typedef short s16x4 __attribute__((ext_vector_type(4)));

// s_waitcnt vmcnt(n) with lgkm/exp counters left at max (gfx9 encoding)
#define VB_WAIT_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | 0x0F70)

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, kMax] (the count is an instruction
// immediate): a compile-time chain of scalar compares
template <int kMax>
__device__ __forceinline__ void wait_vmcnt_upto(int n) {
  if constexpr (kMax > 0) {
    if (n >= kMax) {
      VB_WAIT_VMCNT(kMax);
      return;
    }
    wait_vmcnt_upto<kMax - 1>(n);
  } else {
    VB_WAIT_VMCNT(0);
  }
}

template <class T>
__device__ __forceinline__ typename T::vec8 lds_b128(const uint8_t* base, int off) {
  return *reinterpret_cast<const typename T::vec8*>(base + off);
}

// ds_read_b64_tr_b16, two forms:
//  * lds_tr4 / lds_tr4_imm: the compiler builtin. hipcc's hazard recognizer and waitcnt pass see
//    it; but while LDS-DMA writes are in flight the waitcnt pass drains the whole DMA queue
//    (s_waitcnt vmcnt(0)) before it, serialising a DMA ring.
//  * lds_tr4_asm: inline asm, invisible to the waitcnt pass. Its destination is NOT ready when the
//    statement returns: wait with an `s_waitcnt lgkmcnt` asm that names the destinations before any
//    use. Only its result is asm-produced; it reads no MFMA result, so no MFMA->VALU hazard applies.
__device__ __forceinline__ s16x4 lds_tr4(const uint8_t* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(base + off));
}
__device__ __forceinline__ s16x4 lds_tr4_imm(uint32_t lane_addr, int imm) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      reinterpret_cast<__attribute__((address_space(3))) s16x4*>(static_cast<uintptr_t>(lane_addr + imm)));
}
__device__ __forceinline__ s16x4 lds_tr4_asm_at(const uint8_t* base, int off) {
  const uint32_t a = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)(base + off)));
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
__device__ __forceinline__ s16x4 lds_tr4_asm(uint32_t lane_addr, int imm) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(lane_addr), "i"(imm));
  return r;
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

// max of three floats: one v_max3_f32 when the translation unit is built with -fno-honor-nans
// (see the Makefile; otherwise hipcc canonicalises every MFMA result with an extra v_max x,x).
// Never inline asm here: an asm statement reading MFMA results is invisible to hipcc's hazard
// recognizer, which then omits the wait states between the MFMA write and the read.
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

// ---- LDS-DMA through a buffer descriptor ------------------------------------------------------------
// (base, extent) of a wave-uniform buffer; the descriptor itself is built inside dma16 (the compiler
// keeps it in SGPRs and hoists it), so host-side parsing of kernels never sees the device-only
// resource type. `bytes` < 2^31.
struct srd_t {
  const void* base;
  int bytes;
};
__device__ __forceinline__ srd_t make_srd(const void* base, int bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  return srd_t{reinterpret_cast<const void*>((static_cast<uint64_t>(hi) << 32) | lo),
               __builtin_amdgcn_readfirstlane(bytes)};
}
// 16 bytes per lane from base + voffset + soffset into lds + 16 * lane (buffer_load_dwordx4 ... lds)
__device__ __forceinline__ void dma16(srd_t srd, uint8_t* lds, int voffset, int soffset) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(srd.base), (short)0, srd.bytes, 0x00020000),
      (__attribute__((address_space(3))) void*)lds, 16, voffset, soffset, 0, 0);
}
// dma16 with the LDS address passed through an empty asm (an SGPR value the optimizer cannot trace
// to the LDS variable): the DMA's LDS store then carries no alias scope, and hipcc's waitcnt pass
// puts no vmcnt wait of its own in front of LDS reads for it. For kernels that retire every DMA
// with their own counted waits and barriers before reading its bytes.
__device__ __forceinline__ void dma16_unscoped(srd_t srd, uint8_t* lds, int voffset, int soffset) {
  uint32_t a = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)lds)));
  asm("" : "+s"(a));
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(srd.base), (short)0, srd.bytes, 0x00020000),
      (__attribute__((address_space(3))) void*)(uintptr_t)a, 16, voffset, soffset, 0, 0);
}

// 16-bit store through a buffer descriptor: lane address = base + voffset + soffset (no 64-bit
// per-lane address arithmetic on the VALU)
__device__ __forceinline__ void store16(srd_t srd, uint16_t v, int voffset, int soffset) {
  __builtin_amdgcn_raw_buffer_store_b16(
      v, __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(srd.base), (short)0, srd.bytes, 0x00020000),
      voffset, soffset, 0);
}

// ---- dual-use LDS image ---------------------------------------------------------------------------
// A [rows][D] 16-bit tile read BOTH row-wise (ds_read_b128: 16 lanes = 16 consecutive rows, one
// 16-byte chunk) and transposed (ds_read_b64_tr_b16: a half-wave = 4 consecutive rows x 64 bytes),
// conflict-free for both: chunk ch of row r lives at chunk slot ch ^ f(r).
//   D=64  (128-B rows, two rows per 256-B bank row): f = ((r>>1)&1)<<2 | ((r>>2)&3)
//         row reads: over 8 same-parity rows f takes all 8 values; tr reads: rows r, r+2 of a
//         4-row group differ in f's bit 2, i.e. their 64-byte granules land in opposite halves.
//   D=128 (256-B rows): f = (r&3)<<2 | ((r>>2)&3) (bijective over 16 rows; bits 2-3 = r&3 move
//         the 4 rows' granules to 4 distinct quarters).
template <int D>
__device__ __forceinline__ int dual_swz(int row) {
  return (D == 64) ? ((((row >> 1) & 1) << 2) | ((row >> 2) & 3)) : (((row & 3) << 2) | ((row >> 2) & 3));
}
template <int D>
__device__ __forceinline__ int dual_off(int row, int ch) {
  return row * (D * 2) + 16 * (ch ^ dual_swz<D>(row));
}
// byte address of the 4 consecutive columns col..col+3 (col % 4 == 0) of row `row`
template <int D>
__device__ __forceinline__ int dual_off_col(int row, int col) {
  return dual_off<D>(row, col >> 3) + 2 * (col & 7);
}

// Lane-relative coordinates of the transposed read (ds_read_b64_tr_b16) that fetches the A
// operand [32 cols x 16 rows] matching a packed C tile: lane 4q+p of each 16-lane group reads row
// q of its 4-row block, columns 4p..4p+3 of the group's 16.
__device__ __forceinline__ int tr_row(int lane) { return 4 * (lane >> 5) + ((lane & 15) >> 2); }
__device__ __forceinline__ int tr_col(int lane) { return 16 * ((lane >> 4) & 1) + 4 * (lane & 3); }

// ---- reference-API block-mask addressing ----------------------------------------------------------
// Block-Sparse-Attention's head_mask_type: 0 dense; m > 0 block-sparse with base_blockmask head
// m-1; m < 0 a streaming head (unsupported: NaN output). `mode` (open offline):
// VB_MASK_HEAD_PER_HEAD renumbers every 1 to 1,2,3.. in head order first (the library's
// replace_ones_with_count: ones(H) -> one mask per head); VB_MASK_HEAD_SHARED0 reads m literally
// (ones(H) -> every head uses base_blockmask head 0). ms[0] < 0 = batch stride counted on the
// device as (#heads with id 1) * ms[1]. Returns the (b, h) mask base (row 0, column 0) or nullptr
// if dense.
__device__ __forceinline__ const uint8_t* head_mask_base(const uint8_t* mask, const int64_t* ms,
                                                         const int32_t* hmt, int H, int b, int h,
                                                         bool& nan_head, int mode = VB_MASK_HEAD_PER_HEAD) {
  nan_head = false;
  if (mask == nullptr) return nullptr;
  int mh = h;
  if (hmt) {
    const int t = hmt[h];
    if (t == 0) return nullptr;
    if (t < 0) { nan_head = true; return nullptr; }
    if (t == 1 && mode == VB_MASK_HEAD_PER_HEAD) {
      int cnt = 0;
      for (int i = 0; i <= h; ++i) cnt += (hmt[i] == 1);
      mh = cnt - 1;
    } else {
      mh = t - 1;
    }
  }
  int64_t mb = ms[0];
  if (mb < 0) {
    int ones = 0;
    for (int i = 0; i < H; ++i) ones += (hmt[i] == 1);
    mb = (int64_t)ones * ms[1];
  }
  return mask + b * mb + (int64_t)mh * ms[1];
}

// XCD-aware work order: workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8 share one
// XCD and its L2); give every XCD a contiguous range of the linear work index instead.
__device__ __forceinline__ int xcd_linear(int id, int nwg) {
  const int xcd = id & 7, slot = id >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
}

}  // namespace vb

// Parameter blocks and geometry shared by the block-sparse FMHA backward kernels (vb_attn_bwd.hip,
// vb_attn_bwd_kv128.hip). See vb_attn_bwd.hip for the algorithm.
#pragma once
#include "vb_tiles.hpp"

namespace vb {

namespace bwd {
constexpr int kThreads = 256;
constexpr int kBlk = 128;       // mask block (rows and keys)
constexpr int kT = 64;          // rows (dkdv) / keys (dq) per LDS tile
constexpr int kMaxBlocks = 1024;
constexpr float kBigL = 1.0e30f;  // L' of rows that must contribute nothing (exp2(s - 1e30) = 0)
}  // namespace bwd

struct PrepParams {
  const void* q; const void* dout; const void* out; const void* out2;
  int64_t qs[3], dos[3], os[3], o2s[3];
  const float* lse; const float* lse2; const float* alpha;  // [B,H,Lq] at the caller's row
  const int32_t* q_rows; const int32_t* cu_q;
  void* q_r; void* do_r;  // [B,H,Lq,D] contiguous reordered copies (written when q_rows != NULL)
  float* stats;           // [B*H][ntile][4][64]: L'1, -Delta1, L'2, -Delta2
  int B, H, Lq, D, ntile;
};

struct BwdParams {
  const void* q; const void* dout; int64_t qs[3], dos[3];  // row g of (b,h) at qrow0 + g
  const void* k; const void* v; int64_t ks[3], vs[3];
  const void* kp; const void* vp; int64_t kps[3], vps[3];
  int Lkp;
  const int32_t* cu_q; const int32_t* cu_k; const int32_t* head_mask_type;
  int hm_mode;   // VB_MASK_HEAD_PER_HEAD / VB_MASK_HEAD_SHARED0 (head_mask_base)
  const uint8_t* mask; int64_t ms[3];
  const float* stats; int ntile;
  void* dq; int64_t dqs[3]; const int32_t* q_rows;
  void* dk; void* dv; int64_t dks[3], dvs[3]; const int32_t* kv_rows;
  float* dkp; float* dvp;  // [B,H,Lkp,D] fp32 pooled-key grads
  int psplit;              // pooled-key workgroups split the q-blocks in psplit ranges...
  float* dkp_part; float* dvp_part;  // ...into [psplit][B,H,Lkp,D] partials (== dkp/dvp if 1)
  int gap;
  int B, H, Lq, Lk, nbq, nbk, nbkp;
  float c;      // scale * log2(e)
  float scale;
  int heavy_rows;
  // multi-level mode (vb_ml_attn_bwd): k/v are the KV pyramids [B,H,15*Lpad/8,D] (contiguous),
  // mask the level mask; the pooled levels' pyramid-row grads go to dkpyr/dvpyr fp32
  // [B,H,7*Lpad/8,D] (level 2 rows, then level 4, then level 8)
  int Lpad;
  int ref_tail;
  float* dkpyr; float* dvpyr;
};

// multi-level geometry shared by the backward kernels: pyramid level regions (rows) and the
// pooled-level work items of the dK/dV pass (one 128-row pyramid block each)
struct MlGeom {
  int nb, Lpad, off[4];   // level-1/2/4/8 region starts in the pyramid
  int nblk[4];            // 128-row pyramid blocks per level: ceil(nb / p)
  __device__ __forceinline__ MlGeom(int Lpad_) {
    Lpad = Lpad_;
    nb = Lpad / 128;
    off[0] = 0; off[1] = Lpad; off[2] = Lpad + Lpad / 2; off[3] = off[2] + Lpad / 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) nblk[e] = (nb + (1 << e) - 1) >> e;
  }
};

// The hand-scheduled dK/dV kernels (vb_attn_bwd_kv.hip): returns 0 or a VB_ERR code. `pooled`
// selects the pooled-key pass (grid nbkp * B*H * psplit) over the full-resolution one (grid nbk * B*H).
int launch_dkdv_pipe(const BwdParams& p, int D, bool pooled, bool f16, hipStream_t s);
// the hand-scheduled dQ kernels (same file; grid nbq * B*H) on the ring `sel` picks
// (VB_BWD_SEL_DQ_RING4); ORs the VB_BWD_RAN_* bit of what it launched into `ran`
int launch_dq_pipe(const BwdParams& p, int D, bool pool, bool f16, hipStream_t s, int sel, int& ran);
// the multi-level dQ on the 2-slot pipeline (vb_ml_attn_bwd)
int launch_ml_dq_pipe(const BwdParams& p, int D, bool f16, hipStream_t s);
// the multi-level level-1 dK/dV on the pipeline kernel
int launch_ml_dkdv_pipe(const BwdParams& p, int D, bool f16, hipStream_t s);

}  // namespace vb

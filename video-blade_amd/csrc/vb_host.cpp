// Host-side pieces of libvblade_hip.so: error plumbing and the Gilbert 3-D curve permutation.
//
// vb_gilbert3d_perm restates the generalized Hilbert ("gilbert") space-filling curve
// (J. Cervený, BSD-2) the reference uses to reorder video tokens:
// cogvideox/train/special_attentions_local/utils/gilbert3d.py:6-167 and the coordinate->index map
// of GilbertRearranger (TrainRelated/cogvideo_blocksparseattn.py:119-140).
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "vb_common.hpp"

namespace vb {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return fail(VB_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  }
  return VB_OK;
}

// Persistent launches: the occupancy of `kernel` at `smem` bytes of dynamic LDS times the device's
// CUs, rounded down to a multiple of 8 (every XCD the same number of workgroups). Host queries only,
// cached per (kernel, device, LDS size).
int resident_grid(const void* kernel, int threads, size_t smem) {
  static std::mutex mu;
  static std::map<std::tuple<const void*, int, size_t>, int> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  const auto key = std::make_tuple(kernel, dev, smem);
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, smem) != hipSuccess) per_cu = 0;
  const int slots = cus * per_cu >= 8 ? cus * per_cu / 8 * 8 : 8;
  std::lock_guard<std::mutex> g(mu);
  cache[key] = slots;
  return slots;
}

namespace {

struct V3 {
  long x, y, z;
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline long sgn(long v) { return (v > 0) - (v < 0); }
inline V3 unit(V3 a) { return {sgn(a.x), sgn(a.y), sgn(a.z)}; }
inline long l1(V3 a) { return std::labs(a.x + a.y + a.z); }
inline long floordiv2(long v) { return v >= 0 ? v / 2 : -((-v + 1) / 2); }  // Python // 2
inline V3 half(V3 a) { return {floordiv2(a.x), floordiv2(a.y), floordiv2(a.z)}; }

struct Walker {
  long W, H;
  int32_t* out;
  long n = 0;
  void emit(V3 p) { out[n++] = static_cast<int32_t>(p.x + W * (p.y + H * p.z)); }

  // p: origin, a: major axis, b/c: the two other axes (each axis-aligned, signed)
  void box(V3 p, V3 a, V3 b, V3 c) {
    const long w = l1(a), h = l1(b), d = l1(c);
    const V3 da = unit(a), db = unit(b), dc = unit(c);
    if (h == 1 && d == 1) { for (long i = 0; i < w; ++i, p = p + da) emit(p); return; }
    if (w == 1 && d == 1) { for (long i = 0; i < h; ++i, p = p + db) emit(p); return; }
    if (w == 1 && h == 1) { for (long i = 0; i < d; ++i, p = p + dc) emit(p); return; }
    V3 a2 = half(a), b2 = half(b), c2 = half(c);
    if ((l1(a2) & 1) && w > 2) a2 = a2 + da;
    if ((l1(b2) & 1) && h > 2) b2 = b2 + db;
    if ((l1(c2) & 1) && d > 2) c2 = c2 + dc;
    const V3 ra = a - a2, rb = b - b2, rc = c - c2;
    if (2 * w > 3 * h && 2 * w > 3 * d) {
      box(p, a2, b, c);
      box(p + a2, ra, b, c);
    } else if (3 * h > 4 * d) {
      box(p, b2, c, a2);
      box(p + b2, a, rb, c);
      box(p + (a - da) + (b2 - db), -b2, c, -ra);
    } else if (3 * d > 4 * h) {
      box(p, c2, a2, b);
      box(p + c2, a, b, rc);
      box(p + (a - da) + (c2 - dc), -c2, -ra, b);
    } else {
      box(p, b2, c2, a2);
      box(p + b2, c, a2, rb);
      box(p + (b2 - db) + (c - dc), a, -b2, -rc);
      box(p + (a - da) + b2 + (c - dc), -c, -ra, rb);
      box(p + (a - da) + (b2 - db), -b2, c2, -ra);
    }
  }
};

}  // namespace
}  // namespace vb

extern "C" {

const char* vb_last_error(void) { return vb::g_last_error.c_str(); }

int vb_abi_version(void) { return VB_ABI_VERSION; }

int vb_gilbert3d_perm(int width, int height, int depth, int32_t* perm_out) {
  using vb::V3;
  if (width <= 0 || height <= 0 || depth <= 0 || !perm_out)
    return vb::fail(VB_ERR_INVALID, "vb_gilbert3d_perm: dims must be positive and perm_out non-null");
  if (static_cast<long>(width) * height * depth > (1L << 30))
    return vb::fail(VB_ERR_INVALID, "vb_gilbert3d_perm: volume too large");
  vb::Walker wk{width, height, perm_out};
  const V3 o{0, 0, 0}, X{width, 0, 0}, Y{0, height, 0}, Z{0, 0, depth};
  if (width >= height && width >= depth)
    wk.box(o, X, Y, Z);
  else if (height >= width && height >= depth)
    wk.box(o, Y, X, Z);
  else
    wk.box(o, Z, X, Y);
  if (wk.n != static_cast<long>(width) * height * depth)
    return vb::fail(VB_ERR_INVALID, "vb_gilbert3d_perm: internal error (curve length)");
  return VB_OK;
}

}  // extern "C"

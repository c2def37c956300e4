// Shared device/host helpers for the frcnn_amd HIP library (gfx950 / CDNA4).
//
// Numerics contract: every file is compiled with -ffp-contract=off and HIP's
// default correctly-rounded f32 divide/sqrt, so each arithmetic statement below
// rounds exactly once, in the same order as the reference's torch expressions.
// That is what makes IoU / assignment bit-exact against the reference CPU path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/frcnn_amd.h"

namespace frh {

// ---------------------------------------------------------------- errors
void set_error(const char* fmt, ...);
int32_t check_launch(const char* what);

#define FRH_REQUIRE(cond, ...)                 \
  do {                                         \
    if (!(cond)) {                             \
      ::frh::set_error(__VA_ARGS__);           \
      return FRH_EINVAL;                       \
    }                                          \
  } while (0)

#define FRH_HIP(call)                                                   \
  do {                                                                  \
    hipError_t e_ = (call);                                             \
    if (e_ != hipSuccess) {                                             \
      ::frh::set_error("%s failed: %s", #call, hipGetErrorString(e_));  \
      return FRH_ELAUNCH;                                               \
    }                                                                   \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Workgroups of `kernel` (block threads, dynamic LDS bytes) the current device holds at
// once: its CU count x hipOccupancyMaxActiveBlocksPerMultiprocessor, cached per (device,
// kernel).  The one-launch kernels whose workgroups wait for each other size their grids
// from it (a partitioned GPU has fewer CUs).  0 when the query fails: callers then take
// their multi-launch forms.
int resident_capacity(const void* kernel, int block, size_t dyn_lds = 0);

constexpr int kWave = 64;

// ---------------------------------------------------------------- box math
// calc_iou (reference lib/utils.py:151-172): +1 widths, intersection zeroed
// unless tl < br strictly on both axes, iou = area_i / ((area_a + area_b) - area_i).
__device__ __forceinline__ float iou_plus1(float ax1, float ay1, float ax2, float ay2,
                                           float bx1, float by1, float bx2, float by2) {
  float tlx = fmaxf(ax1, bx1), tly = fmaxf(ay1, by1);
  float brx = fminf(ax2, bx2), bry = fminf(ay2, by2);
  float iw = (brx - tlx) + 1.0f;
  float ih = (bry - tly) + 1.0f;
  float area_i = iw * ih;
  float m = (tlx < brx && tly < bry) ? 1.0f : 0.0f;
  area_i = area_i * m;
  float area_a = ((ax2 - ax1) + 1.0f) * ((ay2 - ay1) + 1.0f);
  float area_b = ((bx2 - bx1) + 1.0f) * ((by2 - by1) + 1.0f);
  return area_i / ((area_a + area_b) - area_i);
}

// torchvision.ops.nms IoU (no +1, max(0,.) clipped intersection).
__device__ __forceinline__ float iou_tv(float4 a, float area_a, float4 b, float area_b) {
  float w = fmaxf(0.0f, fminf(a.z, b.z) - fmaxf(a.x, b.x));
  float h = fmaxf(0.0f, fminf(a.w, b.w) - fmaxf(a.y, b.y));
  float inter = w * h;
  return inter / ((area_a + area_b) - inter);
}

// ------------------------------------------------------- ordered float keys
// Monotone map f32 -> u32 (NaN above +inf, -0 just below +0).
__device__ __forceinline__ uint32_t float_key(float f) {
  uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// ------------------------------------------------------------- wave utils
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t w = __shfl_xor(v, o, kWave);
    v = v > w ? v : w;
  }
  return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  return (lane_id() == 0) ? 0ull : ((~0ull) >> (kWave - lane_id()));
}

// wave-aggregated append: every lane with `take` gets a distinct slot of the
// list behind `counter` (LDS or global); -1 for the others.  Wave-uniform call.
__device__ __forceinline__ int wave_append(bool take, int* counter) {
  const uint64_t m = __ballot(take);
  if (!m) return -1;
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if (lane_id() == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader, kWave);
  return take ? base + __popcll(m & lanemask_lt()) : -1;
}

}  // namespace frh

// Shared RoIAlign / RoIPool device helpers: level descriptors, torchvision's
// bilinear tap rule, RoI geometry and CDNA4 buffer / LDS-DMA primitives.
// Reference: lib/region.py:243-306 (per-level torchvision RoIAlign, legacy
// aligned=False semantics).
#pragma once
#include "common.h"

namespace frh {

struct RoiLevels {
  const float* feat[FRH_MAX_LEVELS];
  float* grad[FRH_MAX_LEVELS];
  int32_t h[FRH_MAX_LEVELS], w[FRH_MAX_LEVELS];
  int64_t sb[FRH_MAX_LEVELS], sc[FRH_MAX_LEVELS], sy[FRH_MAX_LEVELS], sx[FRH_MAX_LEVELS];
  float scale[FRH_MAX_LEVELS];
  int L;
};

struct RoiCfg {
  const float* rois;         // [K, 5]
  const int64_t* levels;     // [K] or nullptr
  int64_t K;
  int C, ph, pw, sampling, aligned;
};

struct Tap {
  int lo, hi;
  float l, h;  // fractional part and 1 - fractional part
  int valid;
};

// One coordinate of torchvision's bilinear_interpolate / pre_calc.
__device__ __forceinline__ Tap make_tap(float v, int size) {
  Tap t;
  if (v < -1.0f || v > (float)size) {
    t.valid = 0;
    t.lo = t.hi = 0;
    t.l = t.h = 0.f;
    return t;
  }
  t.valid = 1;
  if (v <= 0.f) v = 0.f;
  int lo = (int)v, hi;
  if (lo >= size - 1) {
    hi = lo = size - 1;
    v = (float)lo;
  } else {
    hi = lo + 1;
  }
  t.lo = lo;
  t.hi = hi;
  t.l = v - (float)lo;
  t.h = 1.0f - t.l;
  return t;
}

struct RoiGeom {
  int b, lvl, gh, gw;
  float start_h, start_w, bin_h, bin_w;
  float count;
};

__device__ __forceinline__ RoiGeom roi_geom(const RoiCfg& c, const RoiLevels& lv, int64_t k) {
  RoiGeom g;
  const float* r = c.rois + k * 5;
  g.b = (int)r[0];
  g.lvl = c.levels ? (int)c.levels[k] : 0;
  const float sc = lv.scale[g.lvl];
  const float off = c.aligned ? 0.5f : 0.0f;
  float sw = r[1] * sc - off, sh = r[2] * sc - off;
  float ew = r[3] * sc - off, eh = r[4] * sc - off;
  float rw = ew - sw, rh = eh - sh;
  if (!c.aligned) {
    rw = fmaxf(rw, 1.0f);
    rh = fmaxf(rh, 1.0f);
  }
  g.start_w = sw;
  g.start_h = sh;
  g.bin_h = rh / (float)c.ph;
  g.bin_w = rw / (float)c.pw;
  g.gh = c.sampling > 0 ? c.sampling : (int)ceilf(rh / (float)c.ph);
  g.gw = c.sampling > 0 ? c.sampling : (int)ceilf(rw / (float)c.pw);
  int cnt = g.gh * g.gw;
  g.count = (float)(cnt > 1 ? cnt : 1);
  return g;
}

// fill the separable sample tables: rows [ph*gh], cols [pw*gw]
__device__ __forceinline__ float sample_y(const RoiGeom& g, int p, int i) {
  return g.start_h + (float)p * g.bin_h + ((float)i + 0.5f) * g.bin_h / (float)g.gh;
}
__device__ __forceinline__ float sample_x(const RoiGeom& g, int p, int i) {
  return g.start_w + (float)p * g.bin_w + ((float)i + 0.5f) * g.bin_w / (float)g.gw;
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, n, 0x00020000);
}

// Wave-wide min / max with DPP row ops (no LDS round trip); result in every lane.
template <bool kMin>
__device__ __forceinline__ int wave_minmax_i32(int v) {
  const int id = kMin ? 0x7fffffff : (int)0x80000000;
  auto op = [](int a, int b) { return kMin ? min(a, b) : max(a, b); };
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0xb1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x4e, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x140, 0xf, 0xf, false));  // row_mirror
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));  // row_bcast15
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));  // row_bcast31
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_min_i32(int v) { return wave_minmax_i32<true>(v); }
__device__ __forceinline__ int wave_max_i32(int v) { return wave_minmax_i32<false>(v); }

// buffer_load_dword{,x4} ... lds: kBytes per lane into LDS at lds + 4*kBytes/4 * lane.
// The 16-byte form is a gfx950 instruction the host pass of hipcc cannot check,
// hence the device-pass guard (the host never runs device code).
template <int kBytes>
__device__ __forceinline__ void lds_dma(__amdgpu_buffer_rsrc_t r, float* lds, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(kBytes == 4 || kBytes == 16, "LDS-DMA width");
  if constexpr (kBytes == 16)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
  else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, soff, 0, 0);
#endif
}

// the same with the destination given as a wave-uniform LDS byte address
template <int kBytes>
__device__ __forceinline__ void lds_dma_at(__amdgpu_buffer_rsrc_t r, uint32_t lds_addr, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(kBytes == 4 || kBytes == 16, "LDS-DMA width");
  auto* p = (__attribute__((address_space(3))) void*)(uintptr_t)lds_addr;
  if constexpr (kBytes == 16)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, p, 16, voff, soff, 0, 0);
  else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, p, 4, voff, soff, 0, 0);
#endif
}

// s_waitcnt vmcnt(N) with every other counter left alone (gfx9 encoding).  The
// compiler does not wait for LDS-DMA data before ds_reads: these are explicit.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}


}  // namespace frh

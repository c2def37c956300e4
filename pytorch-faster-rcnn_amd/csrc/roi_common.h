// Shared RoIAlign / RoIPool device helpers: level descriptors, torchvision's
// bilinear tap rule, RoI geometry and CDNA4 buffer / LDS-DMA primitives.
// Reference: lib/region.py:243-306 (per-level torchvision RoIAlign, legacy
// aligned=False semantics).
#pragma once
#include "cdna.h"

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

// roi_geom with the RoI's and its level's loads issued together (one memory round trip
// in the wave's prologue instead of two: the level pointer is selected, not branched on)
// (k wave-uniform).  The compiler would wait for the level before loading the box, so
// both scalar loads are issued by hand, followed by ONE lgkmcnt(0) wait.
__device__ __forceinline__ RoiGeom roi_geom_par(const RoiCfg& c, const RoiLevels& lv, int64_t k) {
  const float* r = c.rois + k * 5;
  const int64_t* lp = c.levels ? c.levels + k : reinterpret_cast<const int64_t*>(c.rois);
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t rq;
  uint32_t r4u, lraw;
  asm volatile(
      "s_load_dwordx4 %0, %3, 0x0\n\t"
      "s_load_dword %1, %3, 0x10\n\t"
      "s_load_dword %2, %4, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=s"(rq), "=s"(r4u), "=s"(lraw)
      : "s"(r), "s"(lp)
      : "memory");
  const float r0 = __uint_as_float(rq.x), r1 = __uint_as_float(rq.y), r2 = __uint_as_float(rq.z),
              r3 = __uint_as_float(rq.w), r4 = __uint_as_float(r4u);
  RoiGeom g;
  g.b = (int)r0;
  g.lvl = c.levels ? (int)lraw : 0;  // level index < 2^31: the low word
  const float sc = lv.scale[g.lvl];
  const float off = c.aligned ? 0.5f : 0.0f;
  float sw = r1 * sc - off, sh = r2 * sc - off;
  float ew = r3 * sc - off, eh = r4 * sc - off;
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

}  // namespace frh

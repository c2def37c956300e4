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
  int B;  // images in the batch (make_levels: no limit until the entry sets it)
};

// A RoI's image and level as indices the feature descriptors can address whatever the RoI rows
// hold: a batch index outside [0, B) or NaN and a level outside [0, L) are clamped (the reference
// would raise an IndexError; a C-ABI kernel must not address outside its tensors -- e.g. the rows
// of an aborted proposal call, NaN coordinates, reach here with garbage in them).
__device__ __forceinline__ int roi_image(const RoiLevels& lv, float b) {
  return b >= 0.0f ? (b < (float)lv.B ? (int)b : lv.B - 1) : 0;  // NaN: 0
}
__device__ __forceinline__ int roi_level(const RoiLevels& lv, int64_t l) {
  return l < 0 ? 0 : (l >= lv.L ? lv.L - 1 : (int)l);
}

struct RoiCfg {
  const float* rois;         // [K, 5]
  const int64_t* levels;     // [K] or nullptr
  int64_t K;
  int C, ph, pw, sampling, aligned;
  unsigned long long* span;  // measurement builds (kSpan): {min wave start, max wave end}, s_memrealtime
  const uint32_t* fix_max;   // fixed-point backward: bits of max|grad_out| (the call's own pass)
  int fix_hb;                // fixed-point backward: ceil(log2(K * ph * pw)), accumulation headroom
  const int32_t* rec;        // forward, kFwdSorted: RoI records in processing order, 8 words each:
                             // (x5 as written, level, original index, 0) -- roi_sort_kernel
};

// kSpan kernels: the launch's span on the 100 MHz clock, first wave start to last wave end.
// One lane per wave makes two memory-side atomics on its shard (workgroup id mod
// FRH_SPAN_SHARDS, one 128-B line each): ~64 waves per line instead of every wave of the
// launch on one line (which serialises: ~11 ns per atomic, 360 us for a cfg2 launch).
__device__ __forceinline__ void record_span(const RoiCfg& c, int64_t t_start) {
  unsigned long long* sh = c.span + (blockIdx.x % FRH_SPAN_SHARDS) * FRH_SPAN_STRIDE;
  atomicMin(&sh[0], (unsigned long long)t_start);
  atomicMax(&sh[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

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
  g.b = roi_image(lv, r[0]);
  g.lvl = c.levels ? roi_level(lv, c.levels[k]) : 0;
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

// The RoI's box and level as loaded (RoiRaw), fetched by hand-issued scalar loads: the
// compiler would wait for the level before loading the box, so the loads of one (or
// two) RoIs go out together, followed by ONE lgkmcnt(0) wait (k wave-uniform).
struct RoiRaw {
  float r0, r1, r2, r3, r4;
  int lvl;
};

typedef uint32_t roi_u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ const int64_t* roi_level_ptr(const RoiCfg& c, int64_t k) {
  return c.levels ? c.levels + k : reinterpret_cast<const int64_t*>(c.rois);  // selected, not branched on
}

__device__ __forceinline__ RoiRaw roi_raw(const RoiCfg& c, roi_u32x4_t q, uint32_t r4, uint32_t l) {
  return RoiRaw{__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w),
                __uint_as_float(r4), c.levels ? (int)l : 0};  // level index < 2^31: the low word
}

__device__ __forceinline__ RoiRaw roi_fetch(const RoiCfg& c, int64_t k) {
  roi_u32x4_t q;
  uint32_t r4, l;
  asm volatile(
      "s_load_dwordx4 %0, %3, 0x0\n\t"
      "s_load_dword %1, %3, 0x10\n\t"
      "s_load_dword %2, %4, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(q), "=&s"(r4), "=&s"(l)  // early clobber: later loads of the statement read the inputs
      : "s"(c.rois + k * 5), "s"(roi_level_ptr(c, k))
      : "memory");
  return roi_raw(c, q, r4, l);
}

// record j of c.rec (kFwdSorted): the RoI and, in *ko, the output row it belongs to
typedef uint32_t roi_u32x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ RoiRaw roi_fetch_rec(const RoiCfg& c, int64_t j, int64_t* ko) {
  roi_u32x8_t q;
  const uint64_t a = reinterpret_cast<uint64_t>(c.rec + j * 8);  // wave-uniform: made scalar
  const uint64_t as = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  asm volatile(
      "s_load_dwordx8 %0, %1, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=s"(q)
      : "s"(reinterpret_cast<const int32_t*>(as))
      : "memory");
  *ko = (int64_t)q[6];
  return RoiRaw{__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]), __uint_as_float(q[3]),
                __uint_as_float(q[4]), (int)q[5]};
}

__device__ __forceinline__ void roi_fetch2(const RoiCfg& c, int64_t k0, int64_t k1, RoiRaw* a, RoiRaw* b) {
  roi_u32x4_t q0, q1;
  uint32_t r40, r41, l0, l1;
  asm volatile(
      "s_load_dwordx4 %0, %6, 0x0\n\t"
      "s_load_dword %1, %6, 0x10\n\t"
      "s_load_dword %2, %7, 0x0\n\t"
      "s_load_dwordx4 %3, %8, 0x0\n\t"
      "s_load_dword %4, %8, 0x10\n\t"
      "s_load_dword %5, %9, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(q0), "=&s"(r40), "=&s"(l0), "=&s"(q1), "=&s"(r41), "=&s"(l1)
      : "s"(c.rois + k0 * 5), "s"(roi_level_ptr(c, k0)), "s"(c.rois + k1 * 5), "s"(roi_level_ptr(c, k1))
      : "memory");
  *a = roi_raw(c, q0, r40, l0);
  *b = roi_raw(c, q1, r41, l1);
}

// roi_geom from a fetched RoI
__device__ __forceinline__ RoiGeom roi_geom_raw(const RoiCfg& c, const RoiLevels& lv, const RoiRaw& rr) {
  RoiGeom g;
  g.b = roi_image(lv, rr.r0);
  g.lvl = roi_level(lv, rr.lvl);
  const float sc = lv.scale[g.lvl];
  const float off = c.aligned ? 0.5f : 0.0f;
  float sw = rr.r1 * sc - off, sh = rr.r2 * sc - off;
  float ew = rr.r3 * sc - off, eh = rr.r4 * sc - off;
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

// roi_geom_raw with the level and its scale already picked (same arithmetic)
__device__ __forceinline__ RoiGeom roi_geom_scaled(const RoiCfg& c, const RoiLevels& lv, const RoiRaw& rr, int lvl,
                                                  float sc) {
  RoiGeom g;
  g.b = roi_image(lv, rr.r0);
  g.lvl = lvl;
  const float off = c.aligned ? 0.5f : 0.0f;
  float sw = rr.r1 * sc - off, sh = rr.r2 * sc - off;
  float ew = rr.r3 * sc - off, eh = rr.r4 * sc - off;
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

// a13/a14: FPN level mapping + RoIAlign forward/backward over all levels and
// images in one launch.
// Reference: lib/region.py:243-306 (BasicRoIExtractor: map_rois_to_levels,
// per-level torchvision RoIAlign(output_size, 1/stride, sampling_ratio=2)),
// torchvision legacy (aligned=False) RoIAlign semantics.
//
// Work decomposition: one 256-thread workgroup per (RoI, chunk of 64
// channels).  The bilinear sample grid is separable, so the workgroup first
// tabulates the ph*gh sample rows and pw*gw sample columns (low/high index,
// fractional weights, validity) in LDS once; every output element then only
// multiplies table entries and gathers 4 taps per sample.  Output items are
// mapped channel-major / bin-minor, so a wave writes one contiguous run of
// the [K, C, ph, pw] output and neighbouring lanes read neighbouring x taps
// of the same feature row.  Feature tensors are addressed through explicit
// (batch, channel, y, x) element strides: NCHW, channels_last and strided
// views (FPN P6 = P5[..., ::2, ::2]) all run the same kernel.
#include <math.h>

#include <type_traits>

#include "common.h"

namespace frh {

constexpr int kRoiThreads = 256;
constexpr int kRoiChanChunk = 64;
constexpr int kMaxSamplesPerDim = 1024;

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

// true when the separable tables fit in LDS (always for fixed sampling ratios;
// adaptive grids on huge RoIs fall back to computing taps per sample)
__device__ __forceinline__ bool taps_fit(const RoiGeom& g, const RoiCfg& c) {
  return c.ph * g.gh <= kMaxSamplesPerDim && c.pw * g.gw <= kMaxSamplesPerDim;
}

__device__ __forceinline__ void fill_taps(const RoiGeom& g, const RoiCfg& c, int H, int W, Tap* ty, Tap* tx) {
  if (!taps_fit(g, c)) return;
  const int ny = c.ph * g.gh, nx = c.pw * g.gw;
  for (int e = threadIdx.x; e < ny + nx; e += blockDim.x) {
    if (e < ny) {
      int p = e / g.gh, i = e - p * g.gh;
      ty[e] = make_tap(sample_y(g, p, i), H);
    } else {
      int q = e - ny;
      int p = q / g.gw, i = q - p * g.gw;
      tx[q] = make_tap(sample_x(g, p, i), W);
    }
  }
}

__global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  __shared__ Tap ty[kMaxSamplesPerDim], tx[kMaxSamplesPerDim];
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  fill_taps(g, c, H, W, ty, tx);
  __syncthreads();
  const int nbins = c.ph * c.pw;
  const int nch = min(kRoiChanChunk, c.C - c0);
  const bool tab = taps_fit(g, c);
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  float* o = out + (k * c.C + c0) * nbins;
  for (int item = threadIdx.x; item < nch * nbins; item += blockDim.x) {
    const int cl = item / nbins, bin = item - cl * nbins;
    const int py = bin / c.pw, px = bin - py * c.pw;
    const float* f = base + (int64_t)(c0 + cl) * scs;
    float acc = 0.0f;
    for (int iy = 0; iy < g.gh; ++iy) {
      const Tap a = tab ? ty[py * g.gh + iy] : make_tap(sample_y(g, py, iy), H);
      for (int ix = 0; ix < g.gw; ++ix) {
        const Tap bx = tab ? tx[px * g.gw + ix] : make_tap(sample_x(g, px, ix), W);
        float val = 0.0f;
        if (a.valid && bx.valid) {
          float w1 = a.h * bx.h, w2 = a.h * bx.l, w3 = a.l * bx.h, w4 = a.l * bx.l;
          float v1 = f[a.lo * sy + bx.lo * sx], v2 = f[a.lo * sy + bx.hi * sx];
          float v3 = f[a.hi * sy + bx.lo * sx], v4 = f[a.hi * sy + bx.hi * sx];
          val = ((w1 * v1 + w2 * v2) + w3 * v3) + w4 * v4;
        }
        acc = acc + val;
      }
    }
    o[item] = acc / g.count;
  }
}

// Staged variant (fixed sampling ratio): the RoI's bilinear taps all fall in
// the window [y0, y1] x [x0, x1] of its level (<= ~30x30 cells after FPN level
// mapping).  The workgroup copies that window for as many channels as fit in
// 48 KB of LDS with row-contiguous (coalesced) loads, then evaluates the
// 16 taps of every output element from LDS.  Same arithmetic order as the
// direct kernel, so outputs are identical.
constexpr int kStageTaps = 64;
constexpr int kStageFloats = 12288;

__global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_staged_kernel(RoiLevels lv, RoiCfg c,
                                                                           float* __restrict__ out) {
  __shared__ Tap ty[kStageTaps], tx[kStageTaps];
  __shared__ float win[kStageFloats];
  __shared__ int wb[4];
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int ny = c.ph * g.gh, nx = c.pw * g.gw;
  for (int e = threadIdx.x; e < ny + nx; e += blockDim.x) {
    if (e < ny) {
      int p = e / g.gh, i = e - p * g.gh;
      ty[e] = make_tap(sample_y(g, p, i), H);
    } else {
      int q = e - ny, p = q / g.gw, i = q - p * g.gw;
      tx[q] = make_tap(sample_x(g, p, i), W);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int y0 = 1 << 30, y1 = -1, x0 = 1 << 30, x1 = -1;
    for (int e = 0; e < ny; ++e)
      if (ty[e].valid) {
        y0 = min(y0, ty[e].lo);
        y1 = max(y1, ty[e].hi);
      }
    for (int e = 0; e < nx; ++e)
      if (tx[e].valid) {
        x0 = min(x0, tx[e].lo);
        x1 = max(x1, tx[e].hi);
      }
    wb[0] = y0;
    wb[1] = y1;
    wb[2] = x0;
    wb[3] = x1;
  }
  __syncthreads();
  const int y0 = wb[0], x0 = wb[2];
  const int WH = wb[1] - y0 + 1, WW = wb[3] - x0 + 1;
  const int area = (wb[1] >= 0 && wb[3] >= 0) ? WH * WW : 0;
  const int nbins = c.ph * c.pw;
  const int nch = min(kRoiChanChunk, c.C - c0);
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l];
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  float* o = out + (k * c.C + c0) * nbins;
  int csub = area > 0 ? min(nch, kStageFloats / area) : nch;
  if (csub == 0) {
    // window too large for LDS (only for tiny pooled sizes on huge RoIs): direct gather
    for (int item = threadIdx.x; item < nch * nbins; item += blockDim.x) {
      const int cl = item / nbins, bin = item - cl * nbins;
      const int py = bin / c.pw, px = bin - py * c.pw;
      const float* f = base + (int64_t)(c0 + cl) * scs;
      float acc = 0.0f;
      for (int iy = 0; iy < g.gh; ++iy) {
        const Tap a = ty[py * g.gh + iy];
        for (int ix = 0; ix < g.gw; ++ix) {
          const Tap bx = tx[px * g.gw + ix];
          float val = 0.0f;
          if (a.valid && bx.valid) {
            float w1 = a.h * bx.h, w2 = a.h * bx.l, w3 = a.l * bx.h, w4 = a.l * bx.l;
            val = ((w1 * f[a.lo * sy + bx.lo * sx] + w2 * f[a.lo * sy + bx.hi * sx]) +
                   w3 * f[a.hi * sy + bx.lo * sx]) + w4 * f[a.hi * sy + bx.hi * sx];
          }
          acc = acc + val;
        }
      }
      o[item] = acc / g.count;
    }
    return;
  }
  for (int cc = 0; cc < nch; cc += csub) {
    const int cn = min(csub, nch - cc);
    const int total = cn * area;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
      int ch = e / area, rem = e - ch * area;
      int r = rem / WW, col = rem - r * WW;
      win[e] = base[(int64_t)(c0 + cc + ch) * scs + (int64_t)(y0 + r) * sy + (int64_t)(x0 + col) * sx];
    }
    __syncthreads();
    for (int item = threadIdx.x; item < cn * nbins; item += blockDim.x) {
      const int cl = item / nbins, bin = item - cl * nbins;
      const int py = bin / c.pw, px = bin - py * c.pw;
      const float* w = win + cl * area;
      float acc = 0.0f;
      for (int iy = 0; iy < g.gh; ++iy) {
        const Tap a = ty[py * g.gh + iy];
        for (int ix = 0; ix < g.gw; ++ix) {
          const Tap bx = tx[px * g.gw + ix];
          float val = 0.0f;
          if (a.valid && bx.valid) {
            const int ylo = (a.lo - y0) * WW, yhi = (a.hi - y0) * WW;
            const int xlo = bx.lo - x0, xhi = bx.hi - x0;
            float w1 = a.h * bx.h, w2 = a.h * bx.l, w3 = a.l * bx.h, w4 = a.l * bx.l;
            val = ((w1 * w[ylo + xlo] + w2 * w[ylo + xhi]) + w3 * w[yhi + xlo]) + w4 * w[yhi + xhi];
          }
          acc = acc + val;
        }
      }
      o[(cc + cl) * nbins + bin] = acc / g.count;
    }
    __syncthreads();
  }
}

// Register-tap variant (sampling ratio 2, any pooled size with ph*pw <= 256):
// thread t owns ONE output bin (t % nbins) for a fixed channel residue
// (t / nbins), so its 2x2 sample taps (rows and columns: low/high index +
// weights) are computed once into registers; the thread then walks the
// channels of its chunk with stride (threads / nbins), issuing the 16 tap
// loads of each channel back to back.  No LDS, no per-item division.
template <int SR>
__global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_regtap_kernel(RoiLevels lv, RoiCfg c,
                                                                           float* __restrict__ out) {
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int groups = kRoiThreads / nbins;
  const int t = threadIdx.x;
  if (t >= groups * nbins) return;
  const int bin = t % nbins, cg = t / nbins;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(sample_y(g, py, i), H);
    tx[i] = make_tap(sample_x(g, px, i), W);
  }
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  // per-sample offsets and weights (invalid samples contribute exactly 0)
  int32_t off[SR][SR][4];  // offsets within one channel plane fit in 32 bits
  float wt[SR][SR][4];
  bool ok[SR][SR];
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      ok[iy][ix] = a.valid && b.valid;
      off[iy][ix][0] = (int32_t)(a.lo * sy + b.lo * sx);
      off[iy][ix][1] = (int32_t)(a.lo * sy + b.hi * sx);
      off[iy][ix][2] = (int32_t)(a.hi * sy + b.lo * sx);
      off[iy][ix][3] = (int32_t)(a.hi * sy + b.hi * sx);
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
    }
  const int nch = min(kRoiChanChunk, c.C - c0);
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)c0 * scs;
  float* o = out + (k * c.C + c0) * nbins + bin;
  for (int ch = cg; ch < nch; ch += groups) {
    const float* f = base + (int64_t)ch * scs;
    float v[SR][SR][4];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[iy][ix][q] = f[off[iy][ix][q]];  // invalid taps point at (0,0)
    float acc = 0.0f;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        float val = ((wt[iy][ix][0] * v[iy][ix][0] + wt[iy][ix][1] * v[iy][ix][1]) + wt[iy][ix][2] * v[iy][ix][2]) +
                    wt[iy][ix][3] * v[iy][ix][3];
        acc = acc + (ok[iy][ix] ? val : 0.0f);
      }
    o[(int64_t)ch * nbins] = acc / g.count;
  }
}

__device__ __forceinline__ float pick4(const float4& v, int i) {
  const float a = (i & 1) ? v.y : v.x;
  const float b = (i & 1) ? v.w : v.z;
  return (i & 2) ? b : a;
}

// Row-vector variant (sampling ratio 2, unit x stride, ph*pw <= 256).
// After FPN level mapping a bin spans <= ~4 feature cells, so the x taps of a
// bin's two x-samples (x_lo0 .. x_hi1) fall inside 4 consecutive cells: ONE
// 16-byte load per tap row (rows y_lo/y_hi of the two y-samples) fetches all
// of them -> 4 vector loads per (bin, channel) instead of 16 dword gathers.
// The window start xb = min(x_lo0, W - 4) keeps the load inside the row (the
// KFD runs gfx9+ queues in unaligned mode, so xb need not be 4-aligned).
// Bins whose taps do not fit (huge clamped RoIs, maps narrower than 4) use
// the dword gather.  Arithmetic identical to the reference order.
template <int U>
__global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_vec4_kernel(RoiLevels lv, RoiCfg c,
                                                                         float* __restrict__ out) {
  constexpr int SR = 2;
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int groups = kRoiThreads / nbins;
  const int t = threadIdx.x;
  if (t >= groups * nbins) return;
  const int bin = t % nbins, cg = t / nbins;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(sample_y(g, py, i), H);
    tx[i] = make_tap(sample_x(g, px, i), W);
  }
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  int xmin = 1 << 30, xmax = -1;
#pragma unroll
  for (int i = 0; i < SR; ++i)
    if (tx[i].valid) {
      xmin = min(xmin, tx[i].lo);
      xmax = max(xmax, tx[i].hi);
    }
  const int xb = min(xmin, W - 4);
  const bool fit = sx == 1 && W >= 4 && xmax >= 0 && xmax - xb <= 3;
  int cl[SR], chh[SR], rowo[SR][2];
  bool ok[SR][SR];
  float wt[SR][SR][4];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    cl[i] = tx[i].valid ? tx[i].lo - xb : 0;
    chh[i] = tx[i].valid ? tx[i].hi - xb : 0;
    rowo[i][0] = ty[i].valid ? (int)(ty[i].lo * sy) : 0;
    rowo[i][1] = ty[i].valid ? (int)(ty[i].hi * sy) : 0;
  }
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      ok[iy][ix] = a.valid && b.valid;
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
    }
  const int nch = min(kRoiChanChunk, c.C - c0);
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)c0 * scs;
  float* o = out + (k * c.C + c0) * nbins + bin;
  if (fit) {
    const float* bx = base + xb;
    auto bin_value = [&](const float4 (&rv)[SR][2]) {
      float acc = 0.0f;
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const float v1 = pick4(rv[iy][0], cl[ix]), v2 = pick4(rv[iy][0], chh[ix]);
          const float v3 = pick4(rv[iy][1], cl[ix]), v4 = pick4(rv[iy][1], chh[ix]);
          float val = ((wt[iy][ix][0] * v1 + wt[iy][ix][1] * v2) + wt[iy][ix][2] * v3) + wt[iy][ix][3] * v4;
          acc = acc + (ok[iy][ix] ? val : 0.0f);
        }
      return acc / g.count;
    };
    int ch = cg;
    // U channels per step: all 4U row loads are issued before any is consumed
    for (; ch + (U - 1) * groups < nch; ch += U * groups) {
      float4 rv[U][SR][2];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float* f = bx + (int64_t)(ch + u * groups) * scs;
#pragma unroll
        for (int iy = 0; iy < SR; ++iy) {
          rv[u][iy][0] = *reinterpret_cast<const float4*>(f + rowo[iy][0]);
          rv[u][iy][1] = *reinterpret_cast<const float4*>(f + rowo[iy][1]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) o[(int64_t)(ch + u * groups) * nbins] = bin_value(rv[u]);
    }
    for (; ch < nch; ch += groups) {
      const float* f = bx + (int64_t)ch * scs;
      float4 rv[SR][2];
#pragma unroll
      for (int iy = 0; iy < SR; ++iy) {
        rv[iy][0] = *reinterpret_cast<const float4*>(f + rowo[iy][0]);
        rv[iy][1] = *reinterpret_cast<const float4*>(f + rowo[iy][1]);
      }
      o[(int64_t)ch * nbins] = bin_value(rv);
    }
  } else {
    for (int ch = cg; ch < nch; ch += groups) {
      const float* f = base + (int64_t)ch * scs;
      float acc = 0.0f;
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const int64_t q0 = ok[iy][ix] ? (int64_t)tx[ix].lo * sx : 0, q1 = ok[iy][ix] ? (int64_t)tx[ix].hi * sx : 0;
          const float v1 = f[rowo[iy][0] + q0], v2 = f[rowo[iy][0] + q1];
          const float v3 = f[rowo[iy][1] + q0], v4 = f[rowo[iy][1] + q1];
          float val = ((wt[iy][ix][0] * v1 + wt[iy][ix][1] * v2) + wt[iy][ix][2] * v3) + wt[iy][ix][3] * v4;
          acc = acc + (ok[iy][ix] ? val : 0.0f);
        }
      o[(int64_t)ch * nbins] = acc / g.count;
    }
  }
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, n, 0x00020000);
}

// Buffer-descriptor variant (sampling ratio 2, ph*pw <= 256; the default).
// Lane (bin, channel group cg) keeps its bin's 16 tap offsets in VGPRs as
// 32-bit byte offsets into a descriptor over this (image, level, channel
// chunk) slice; the channel walk moves only the wave-uniform soffset, so the
// loop carries no per-lane address arithmetic.  When every x-sample of the
// wave has x_hi = x_lo + 1 (all but right-border clamped samples) the taps of
// a sample row are one 8-byte load: 8 loads per (bin, channel) instead of 16.
// The 1/count of SR=2 is an exact power of two, so acc * 0.25 == acc / 4.
// Results identical to the direct kernel.
template <int U>
__device__ __forceinline__ void fwd_buf_block(const RoiLevels& lv, const RoiCfg& c, float* __restrict__ out,
                                              int64_t k, int c0, const RoiGeom& g) {
  constexpr int SR = 2;
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int groups = kRoiThreads / nbins;
  const int t = threadIdx.x;
  if (t >= groups * nbins) return;
  const int bin = t % nbins, cg = t / nbins;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(sample_y(g, py, i), H);
    tx[i] = make_tap(sample_x(g, px, i), W);
  }
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l], scs = (int)lv.sc[l];
  const int nch = min(kRoiChanChunk, c.C - c0);
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)c0 * scs;
  const int64_t extent = ((int64_t)(nch - 1) * scs + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(base, extent);
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + c0) * nbins, (int64_t)nch * nbins * 4);
  const int cstep = groups * scs * 4, ostep = groups * nbins * 4;
  bool ok[SR][SR];
  float wt[SR][SR][4];
  int row[SR][2], col[SR][2];
  bool pair = sx == 1;
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    row[i][0] = (cg * scs + (ty[i].valid ? ty[i].lo * sy : 0)) * 4;
    row[i][1] = (cg * scs + (ty[i].valid ? ty[i].hi * sy : 0)) * 4;
    col[i][0] = tx[i].valid ? tx[i].lo * sx * 4 : 0;
    col[i][1] = tx[i].valid ? tx[i].hi * sx * 4 : 0;
    pair = pair && (!tx[i].valid || tx[i].hi == tx[i].lo + 1);
  }
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      ok[iy][ix] = a.valid && b.valid;
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
    }
  auto bin_value = [&](const float (&v)[SR][SR][4]) {
    float acc = 0.0f;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        float val = ((wt[iy][ix][0] * v[iy][ix][0] + wt[iy][ix][1] * v[iy][ix][1]) + wt[iy][ix][2] * v[iy][ix][2]) +
                    wt[iy][ix][3] * v[iy][ix][3];
        acc = acc + (ok[iy][ix] ? val : 0.0f);
      }
    return acc * 0.25f;
  };
  // wave-uniform trip counts (soffset must stay scalar): every lane has a
  // channel in the first nch / groups steps, the tail step is lane-guarded
  const int full = nch / groups, iters = (nch + groups - 1) / groups;
  const bool tail_ok = cg + full * groups < nch;
  if (__all(pair)) {
    int off[SR][2][SR];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) off[iy][r][ix] = row[iy][r] + col[ix][0];
    int it = 0;
    for (; it + U <= full; it += U) {
      u32x2 rv[U][SR][2][SR];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int ix = 0; ix < SR; ++ix)
              rv[u][iy][r][ix] = __builtin_amdgcn_raw_buffer_load_b64(fr, off[iy][r][ix], (it + u) * cstep, 0);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float v[SR][SR][4];
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int ix = 0; ix < SR; ++ix) {
            v[iy][ix][0] = __uint_as_float(rv[u][iy][0][ix].x);
            v[iy][ix][1] = __uint_as_float(rv[u][iy][0][ix].y);
            v[iy][ix][2] = __uint_as_float(rv[u][iy][1][ix].x);
            v[iy][ix][3] = __uint_as_float(rv[u][iy][1][ix].y);
          }
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, t * 4, (it + u) * ostep, 0);
      }
    }
    for (; it < iters; ++it) {
      if (it == full && !tail_ok) break;
      float v[SR][SR][4];
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(fr, off[iy][0][ix], it * cstep, 0);
          const u32x2 b = __builtin_amdgcn_raw_buffer_load_b64(fr, off[iy][1][ix], it * cstep, 0);
          v[iy][ix][0] = __uint_as_float(a.x);
          v[iy][ix][1] = __uint_as_float(a.y);
          v[iy][ix][2] = __uint_as_float(b.x);
          v[iy][ix][3] = __uint_as_float(b.y);
        }
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, t * 4, it * ostep, 0);
    }
  } else {
    for (int it = 0; it < iters; ++it) {
      if (it == full && !tail_ok) break;
      float v[SR][SR][4];
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            v[iy][ix][q] = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(fr, row[iy][q >> 1] + col[ix][q & 1], it * cstep, 0));
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, t * 4, it * ostep, 0);
    }
  }
}

template <int U>
__global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_buf_kernel(RoiLevels lv, RoiCfg c,
                                                                        float* __restrict__ out) {
  const int64_t k = blockIdx.x;
  fwd_buf_block<U>(lv, c, out, k, blockIdx.y * kRoiChanChunk, roi_geom(c, lv, k));
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

// Wave-staged variant (sampling ratio 2, ph*pw <= 64, 2*ph and 2*pw <= 64).
// Every tap of a RoI lies in the window [y0, y1] x [x0, x1] of its level;
// after FPN level mapping that window is a few to ~30 cells per side.  Each
// wave owns 16 channels of the RoI and, per channel, copies the window into
// its own LDS slab with lane-contiguous loads (every feature line fetched
// once per RoI-channel, instead of 8 gathers per bin hitting the same lines),
// then lane = bin reads its 16 taps from LDS.  The loads of channel i+1 are
// in flight while channel i is evaluated.  The slab row has one extra column
// holding a copy of the window's last feature column, so a right-border
// clamped tap (x_lo = x_hi = W-1) reads (x_lo, x_lo + 1) like every other
// sample.  No block barriers: waves are independent.  Windows above
// kWinMax floats take the per-wave gather path.  Results identical to the
// direct kernel.
constexpr int kWinMax = 1024;
constexpr int kWinR = kWinMax / kWave;
constexpr int kWaveChans = kRoiChanChunk / (kRoiThreads / kWave);

// kChunk: channels per workgroup (kChunk / 4 per wave).  kSkip (diagnostics only):
// 1 = skip staged RoIs, 2 = skip gathered ones.
template <int kStageMax, int kSkip = 0, int kChunk = kRoiChanChunk>
__global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_lds_kernel(RoiLevels lv, RoiCfg c,
                                                                        float* __restrict__ out) {
  constexpr int SR = 2;
  __shared__ float slab_all[kRoiThreads / kWave][kWinMax];
  const int64_t k = blockIdx.x;
  // readfirstlane: the wave index is uniform, and the compiler must know it (soffset operands)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
  constexpr int kWC = kChunk / (kRoiThreads / kWave);
  const int cw0 = blockIdx.y * kChunk + wave * kWC;
  const int nch = min(kWC, c.C - cw0);
  float* slab = slab_all[wave];
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int sy = (int)lv.sy[l], sx = (int)lv.sx[l], scs = (int)lv.sc[l];
  // window of the valid taps: lane i evaluates y sample i and x sample i
  int ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
  if (lane < c.ph * SR) {
    const Tap t = make_tap(sample_y(g, lane / SR, lane % SR), H);
    if (t.valid) ylo = t.lo, yhi = t.hi;
  }
  if (lane < c.pw * SR) {
    const Tap t = make_tap(sample_x(g, lane / SR, lane % SR), W);
    if (t.valid) xlo = t.lo, xhi = t.hi;
  }
  const int y0 = __builtin_amdgcn_readfirstlane(wave_min_i32(ylo)), y1 = __builtin_amdgcn_readfirstlane(wave_max_i32(yhi));
  const int x0 = __builtin_amdgcn_readfirstlane(wave_min_i32(xlo)), x1 = __builtin_amdgcn_readfirstlane(wave_max_i32(xhi));
  const bool any = y1 >= y0 && x1 >= x0;
  // odd slab row stride: the 4 tap rows of a wave's bins spread over the LDS banks
  const int ws = (x1 - x0 + 2) | 1, n = any ? (y1 - y0 + 1) * ws : 0;
  if (n > kStageMax) {  // uniform over the block (one RoI): large windows take the block gather path
    if (kSkip != 2)
      for (int cc = 0; cc < kChunk && blockIdx.y * kChunk + cc < c.C; cc += kRoiChanChunk)
        fwd_buf_block<2>(lv, c, out, k, blockIdx.y * kChunk + cc, g);
    return;
  }
  if (kSkip == 1) return;
  if (nch <= 0) return;
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)cw0 * scs;
  const int64_t extent = ((int64_t)(nch - 1) * scs + (int64_t)(H - 1) * sy + (int64_t)(W - 1) * sx + 1) * 4;
  const __amdgpu_buffer_rsrc_t fr = uniform_rsrc(base, extent);
  const __amdgpu_buffer_rsrc_t orr = uniform_rsrc(out + (k * c.C + cw0) * nbins, (int64_t)nch * nbins * 4);
  const int cstep = scs * 4, ostep = nbins * 4;
  // this lane's bin: taps, weights, validity
  const int bin = lane < nbins ? lane : 0;
  const int py = bin / c.pw, px = bin - py * c.pw;
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(sample_y(g, py, i), H);
    tx[i] = make_tap(sample_x(g, px, i), W);
  }
  bool ok[SR][SR];
  float wt[SR][SR][4];
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      ok[iy][ix] = a.valid && b.valid;
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
    }
  auto bin_value = [&](const float (&v)[SR][SR][4]) {
    float acc = 0.0f;
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        float val = ((wt[iy][ix][0] * v[iy][ix][0] + wt[iy][ix][1] * v[iy][ix][1]) + wt[iy][ix][2] * v[iy][ix][2]) +
                    wt[iy][ix][3] * v[iy][ix][3];
        acc = acc + (ok[iy][ix] ? val : 0.0f);
      }
    return acc * 0.25f;
  };
  const bool active = lane < nbins;
  if (n <= kStageMax) {
    // slab addresses of this bin's sample rows (x_lo, x_lo + 1 pairs)
    int sa[SR][2][SR];
#pragma unroll
    for (int iy = 0; iy < SR; ++iy)
#pragma unroll
      for (int ix = 0; ix < SR; ++ix) {
        const bool v = ok[iy][ix];
        sa[iy][0][ix] = v ? (ty[iy].lo - y0) * ws + (tx[ix].lo - x0) : 0;
        sa[iy][1][ix] = v ? (ty[iy].hi - y0) * ws + (tx[ix].lo - x0) : 0;
      }
    // staging: slab element e = lane + 64 j  <-  feature (y0 + e / ws, min(x0 + e % ws, W - 1));
    // the j loop is specialised on RB = 64-element rounds (1, 2, 4, 8, 16) so it unrolls branch-free
    auto run = [&](auto rb) {
      constexpr int RB = decltype(rb)::value, D = kWinR / RB;  // D channel windows per round, 16 loads/lane
      int goff[RB];
#pragma unroll
      for (int j = 0; j < RB; ++j) {
        const int e = lane + j * kWave;
        const int r = e / ws, cc = e - r * ws;
        // lanes past the window re-read its first element: no extra cache line per round
        goff[j] = e < n ? ((y0 + r) * sy + min(x0 + cc, W - 1) * sx) * 4 : (y0 * sy + x0 * sx) * 4;
      }
      float st[D][RB];
      auto issue = [&](int c0r) {
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
          for (int j = 0; j < RB; ++j)
            st[d][j] = __uint_as_float(
                __builtin_amdgcn_raw_buffer_load_b32(fr, goff[j], min(c0r + d, nch - 1) * cstep, 0));
      };
      issue(0);
      for (int i = 0; i < nch; i += D) {
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
          for (int j = 0; j < RB; ++j) slab[(d * RB + j) * kWave + lane] = st[d][j];  // [n, 64 RB) junk, unread
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (i + D < nch) issue(i + D);
        if (active) {
#pragma unroll
          for (int d = 0; d < D; ++d) {
            if (i + d < nch) {
              const float* sl = slab + d * RB * kWave;
              float v[SR][SR][4];
#pragma unroll
              for (int iy = 0; iy < SR; ++iy)
#pragma unroll
                for (int ix = 0; ix < SR; ++ix) {
                  v[iy][ix][0] = sl[sa[iy][0][ix]];
                  v[iy][ix][1] = sl[sa[iy][0][ix] + 1];
                  v[iy][ix][2] = sl[sa[iy][1][ix]];
                  v[iy][ix][3] = sl[sa[iy][1][ix] + 1];
                }
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(bin_value(v)), orr, lane * 4, (i + d) * ostep, 0);
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    };
    const int R = (n + kWave - 1) / kWave;
    if (R <= 1)
      run(std::integral_constant<int, 1>{});
    else if (R <= 2 || kStageMax <= 2 * kWave)
      run(std::integral_constant<int, 2>{});
    else if (R <= 4 || kStageMax <= 4 * kWave)
      run(std::integral_constant<int, 4>{});
    else if (R <= 8 || kStageMax <= 8 * kWave)
      run(std::integral_constant<int, 8>{});
    else
      run(std::integral_constant<int, kWinR>{});
  }
}

// Staged + register-tap variant (sampling ratio SR, ph*pw <= 256).
// After FPN level mapping a RoI covers few feature cells (random-init cfg2:
// median side ~5 cells on P2), so its 16*ph*pw taps per channel hit a small
// window many times over.  Thread (bin, channel group) keeps its bin's tap
// offsets (relative to the window) and weights in registers; the workgroup
// stages the window rows of a channel sub-chunk in LDS with row-contiguous
// loads, then every output element is 16 LDS reads + the reference's
// arithmetic.  Identical results to the direct kernel.
constexpr int kWinFloats = 12288;  // 48 KB window buffer

template <int SR>
__global__ void __launch_bounds__(kRoiThreads) roi_align_fwd_winreg_kernel(RoiLevels lv, RoiCfg c,
                                                                           float* __restrict__ out) {
  __shared__ float win[kWinFloats];
  __shared__ int wb[4];
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  const int nbins = c.ph * c.pw;
  const int groups = kRoiThreads / nbins;
  const int t = threadIdx.x;
  const bool active = t < groups * nbins;
  const int bin = active ? t % nbins : 0, cg = active ? t / nbins : 0;
  const int py = bin / c.pw, px = bin - py * c.pw;
  if (t == 0) {
    wb[0] = 1 << 30;
    wb[1] = -1;
    wb[2] = 1 << 30;
    wb[3] = -1;
  }
  __syncthreads();
  Tap ty[SR], tx[SR];
#pragma unroll
  for (int i = 0; i < SR; ++i) {
    ty[i] = make_tap(sample_y(g, py, i), H);
    tx[i] = make_tap(sample_x(g, px, i), W);
  }
  if (active) {
    int ylo = 1 << 30, yhi = -1, xlo = 1 << 30, xhi = -1;
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      if (ty[i].valid) {
        ylo = min(ylo, ty[i].lo);
        yhi = max(yhi, ty[i].hi);
      }
      if (tx[i].valid) {
        xlo = min(xlo, tx[i].lo);
        xhi = max(xhi, tx[i].hi);
      }
    }
    if (yhi >= 0 && xhi >= 0) {
      atomicMin(&wb[0], ylo);
      atomicMax(&wb[1], yhi);
      atomicMin(&wb[2], xlo);
      atomicMax(&wb[3], xhi);
    }
  }
  __syncthreads();
  const int y0 = wb[0], x0 = wb[2];
  const bool empty = wb[1] < 0;
  const int WH = empty ? 0 : wb[1] - y0 + 1, WW = empty ? 0 : wb[3] - x0 + 1;
  const int area = WH * WW;
  const int nch = min(kRoiChanChunk, c.C - c0);
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  const float* base = lv.feat[l] + (int64_t)g.b * lv.sb[l] + (int64_t)c0 * scs;
  float* o = out + (k * c.C + c0) * nbins + bin;
  int woff[SR][SR][4];
  float wt[SR][SR][4];
  bool ok[SR][SR];
#pragma unroll
  for (int iy = 0; iy < SR; ++iy)
#pragma unroll
    for (int ix = 0; ix < SR; ++ix) {
      const Tap a = ty[iy], b = tx[ix];
      ok[iy][ix] = a.valid && b.valid;
      const int rl = ok[iy][ix] ? (a.lo - y0) * WW : 0, rh = ok[iy][ix] ? (a.hi - y0) * WW : 0;
      const int cl = ok[iy][ix] ? b.lo - x0 : 0, ch = ok[iy][ix] ? b.hi - x0 : 0;
      woff[iy][ix][0] = rl + cl;
      woff[iy][ix][1] = rl + ch;
      woff[iy][ix][2] = rh + cl;
      woff[iy][ix][3] = rh + ch;
      wt[iy][ix][0] = a.h * b.h;
      wt[iy][ix][1] = a.h * b.l;
      wt[iy][ix][2] = a.l * b.h;
      wt[iy][ix][3] = a.l * b.l;
    }
  if (empty) {
    if (active)
      for (int chn = cg; chn < nch; chn += groups) o[(int64_t)chn * nbins] = 0.0f / g.count;
    return;
  }
  const int csub = min(nch, kWinFloats / area);
  if (csub == 0) {
    // window larger than the LDS buffer: gather straight from global memory
    if (!active) return;
    for (int chn = cg; chn < nch; chn += groups) {
      const float* f = base + (int64_t)chn * scs;
      float acc = 0.0f;
#pragma unroll
      for (int iy = 0; iy < SR; ++iy)
#pragma unroll
        for (int ix = 0; ix < SR; ++ix) {
          const Tap a = ty[iy], b = tx[ix];
          const int64_t r0 = (int64_t)a.lo * sy, r1 = (int64_t)a.hi * sy;
          const int64_t q0 = (int64_t)b.lo * sx, q1 = (int64_t)b.hi * sx;
          float val = ((wt[iy][ix][0] * f[r0 + q0] + wt[iy][ix][1] * f[r0 + q1]) + wt[iy][ix][2] * f[r1 + q0]) +
                      wt[iy][ix][3] * f[r1 + q1];
          acc = acc + (ok[iy][ix] ? val : 0.0f);
        }
      o[(int64_t)chn * nbins] = acc / g.count;
    }
    return;
  }
  // staging: the window image [cn][WH][WW] is filled in flat order (lanes
  // along the row), 8 independent loads in flight per lane before the LDS
  // stores, so the copy is bandwidth- not latency-bound.
  constexpr int kUnroll = 8;
  // flat element e = (chn*WH + r)*WW + col advanced by the block size with
  // carries (no per-element integer division)
  const int st_col = kRoiThreads % WW, st_r = (kRoiThreads / WW) % WH, st_ch = kRoiThreads / area;
  const int t_ch = t / area, t_rem = t - t_ch * area, t_r = t_rem / WW, t_col = t_rem - t_r * WW;
  for (int cc = 0; cc < nch; cc += csub) {
    const int cn = min(csub, nch - cc);
    const int total = cn * area;
    int chn = t_ch, r = t_r, col = t_col;
    const float* cbase = base + (int64_t)cc * scs;
    for (int e0 = 0; e0 < total; e0 += kUnroll * kRoiThreads) {
      float v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const bool in = e0 + u * kRoiThreads + t < total;
        const int64_t a = in ? (int64_t)chn * scs + (int64_t)(y0 + r) * sy + (int64_t)(x0 + col) * sx : 0;
        v[u] = cbase[a];
        col += st_col;
        r += st_r;
        chn += st_ch;
        if (col >= WW) {
          col -= WW;
          ++r;
        }
        if (r >= WH) {
          r -= WH;
          ++chn;
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int e = e0 + u * kRoiThreads + t;
        if (e < total) win[e] = v[u];
      }
    }
    __syncthreads();
    if (active) {
      for (int chn = cg; chn < cn; chn += groups) {
        const float* w = win + chn * area;
        float acc = 0.0f;
#pragma unroll
        for (int iy = 0; iy < SR; ++iy)
#pragma unroll
          for (int ix = 0; ix < SR; ++ix) {
            float val = ((wt[iy][ix][0] * w[woff[iy][ix][0]] + wt[iy][ix][1] * w[woff[iy][ix][1]]) +
                         wt[iy][ix][2] * w[woff[iy][ix][2]]) +
                        wt[iy][ix][3] * w[woff[iy][ix][3]];
            acc = acc + (ok[iy][ix] ? val : 0.0f);
          }
        o[(int64_t)(cc + chn) * nbins] = acc / g.count;
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kRoiThreads) roi_align_bwd_kernel(RoiLevels lv, RoiCfg c,
                                                                    const float* __restrict__ gout) {
  __shared__ Tap ty[kMaxSamplesPerDim], tx[kMaxSamplesPerDim];
  const int64_t k = blockIdx.x;
  const int c0 = blockIdx.y * kRoiChanChunk;
  const RoiGeom g = roi_geom(c, lv, k);
  const int l = g.lvl;
  const int H = lv.h[l], W = lv.w[l];
  fill_taps(g, c, H, W, ty, tx);
  __syncthreads();
  const int nbins = c.ph * c.pw;
  const int nch = min(kRoiChanChunk, c.C - c0);
  const bool tab = taps_fit(g, c);
  float* base = lv.grad[l] + (int64_t)g.b * lv.sb[l];
  const int64_t sy = lv.sy[l], sx = lv.sx[l], scs = lv.sc[l];
  const float* go = gout + (k * c.C + c0) * nbins;
  for (int item = threadIdx.x; item < nch * nbins; item += blockDim.x) {
    const int cl = item / nbins, bin = item - cl * nbins;
    const int py = bin / c.pw, px = bin - py * c.pw;
    float* f = base + (int64_t)(c0 + cl) * scs;
    const float gv = go[item];
    for (int iy = 0; iy < g.gh; ++iy) {
      const Tap a = tab ? ty[py * g.gh + iy] : make_tap(sample_y(g, py, iy), H);
      if (!a.valid) continue;
      for (int ix = 0; ix < g.gw; ++ix) {
        const Tap bx = tab ? tx[px * g.gw + ix] : make_tap(sample_x(g, px, ix), W);
        if (!bx.valid) continue;
        float g1 = gv * (a.h * bx.h) / g.count, g2 = gv * (a.h * bx.l) / g.count;
        float g3 = gv * (a.l * bx.h) / g.count, g4 = gv * (a.l * bx.l) / g.count;
        atomicAdd(&f[a.lo * sy + bx.lo * sx], g1);
        atomicAdd(&f[a.lo * sy + bx.hi * sx], g2);
        atomicAdd(&f[a.hi * sy + bx.lo * sx], g3);
        atomicAdd(&f[a.hi * sy + bx.hi * sx], g4);
      }
    }
  }
}

__global__ void roi_level_kernel(const float* rois, int64_t K, float finest, int L, int64_t* levels) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const float* r = rois + k * 5;
  float area = ((r[3] - r[1]) + 1.0f) * ((r[4] - r[2]) + 1.0f);
  float s = sqrtf(area);
  float v = s / finest + 1e-6f;
  // correctly rounded f32 log2, then floor (region.py:262); clamp to [0, L-1]
  float lg = (float)log2((double)v);
  float fl = floorf(lg);
  float hi = (float)(L - 1);
  fl = fl < 0.0f ? 0.0f : (fl > hi ? hi : fl);
  levels[k] = (int64_t)fl;
}

static int32_t make_levels(int32_t L, const float* const* feats, float* const* grads, const int32_t* feat_hw,
                           const int64_t* strides, const float* scales, RoiLevels* lv) {
  FRH_REQUIRE(L >= 1 && L <= FRH_MAX_LEVELS, "num_levels %d out of range", L);
  FRH_REQUIRE(feat_hw && scales && strides, "null pointer argument");
  lv->L = L;
  for (int l = 0; l < L; ++l) {
    lv->feat[l] = feats ? feats[l] : nullptr;
    lv->grad[l] = grads ? grads[l] : nullptr;
    lv->h[l] = feat_hw[2 * l];
    lv->w[l] = feat_hw[2 * l + 1];
    FRH_REQUIRE(lv->h[l] > 0 && lv->w[l] > 0, "level %d has an empty feature map", l);
    lv->sb[l] = strides[4 * l];
    lv->sc[l] = strides[4 * l + 1];
    lv->sy[l] = strides[4 * l + 2];
    lv->sx[l] = strides[4 * l + 3];
    lv->scale[l] = scales[l];
  }
  return FRH_OK;
}

}  // namespace frh

using namespace frh;

extern "C" int32_t frh_roi_level_map(const float* rois, int64_t num_rois, float finest_scale, int32_t num_levels,
                                     int64_t* levels, void* stream) {
  FRH_REQUIRE(num_rois >= 0 && num_levels >= 1, "bad sizes");
  if (num_rois == 0) return FRH_OK;
  FRH_REQUIRE(rois && levels, "null pointer argument");
  hipLaunchKernelGGL(roi_level_kernel, dim3((unsigned)((num_rois + 255) / 256)), dim3(256), 0, as_stream(stream),
                     rois, num_rois, finest_scale, num_levels, levels);
  return check_launch("frh_roi_level_map");
}

static int32_t roi_common_checks(int32_t batch, int32_t channels, int64_t num_rois, int32_t ph, int32_t pw,
                                 const float* rois) {
  FRH_REQUIRE(batch >= 1 && channels >= 1 && num_rois >= 0 && ph >= 1 && pw >= 1, "bad sizes");
  FRH_REQUIRE(num_rois == 0 || rois, "null rois");
  FRH_REQUIRE(num_rois < (int64_t)0x7fffffff, "too many rois");
  return FRH_OK;
}

// variant: 0 = direct gather, 1 = LDS-staged window, -1 = best available.
// Exported for the kernel micro-benchmarks (tools/bench_roi_align.py).
extern "C" int32_t frh_roi_align_fwd_variant(int32_t variant, int32_t num_levels, const float* const* feats,
                                             const int32_t* feat_hw, const int64_t* strides, const float* scales,
                                             int32_t batch, int32_t channels, const float* rois,
                                             const int64_t* roi_levels, int64_t num_rois, int32_t pooled_h,
                                             int32_t pooled_w, int32_t sampling_ratio, int32_t aligned, float* out,
                                             void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  FRH_REQUIRE((feats && out) || num_rois == 0, "null pointer argument");
  RoiLevels lv;
  r = make_levels(num_levels, feats, nullptr, feat_hw, strides, scales, &lv);
  if (r) return r;
  if (num_rois == 0) return FRH_OK;
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  dim3 grid((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk));
  const bool staged_ok = sampling_ratio > 0 && pooled_h * sampling_ratio <= kStageTaps &&
                         pooled_w * sampling_ratio <= kStageTaps;
  const bool regtap_ok = sampling_ratio == 2 && pooled_h * pooled_w <= kRoiThreads;
  // the descriptor variant addresses one (image, level) slice with 32-bit byte offsets
  bool buf_ok = regtap_ok;
  for (int l = 0; l < lv.L; ++l) {
    const int64_t ext = ((int64_t)(channels - 1) * lv.sc[l] + (int64_t)(lv.h[l] - 1) * lv.sy[l] +
                         (int64_t)(lv.w[l] - 1) * lv.sx[l] + 1) * 4;
    buf_ok = buf_ok && lv.sc[l] >= 0 && lv.sy[l] >= 0 && lv.sx[l] >= 0 && ext < ((int64_t)1 << 31);
  }
  const bool lds_ok = buf_ok && pooled_h * pooled_w <= 64 && 2 * pooled_h <= 64 && 2 * pooled_w <= 64;
  if (variant < 0) variant = lds_ok ? 10 : buf_ok ? 8 : 0;
  FRH_REQUIRE(variant == 0 || (variant == 1 && staged_ok) || (variant >= 2 && variant <= 6 && regtap_ok) ||
                  (variant >= 7 && variant <= 8 && buf_ok) || (variant >= 9 && variant <= 16 && lds_ok),
              "roi_align variant %d unsupported here", variant);
  if (variant == 9)
    hipLaunchKernelGGL(roi_align_fwd_lds_kernel<kWinMax>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 10)
    hipLaunchKernelGGL(roi_align_fwd_lds_kernel<256>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 11)
    hipLaunchKernelGGL(roi_align_fwd_lds_kernel<128>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 12)
    hipLaunchKernelGGL(roi_align_fwd_lds_kernel<64>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 13)
    hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, 1>), grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 14)
    hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, 2>), grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 15)
    hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, 0, 256>),
                       dim3((unsigned)num_rois, (unsigned)((channels + 255) / 256)), dim3(kRoiThreads), 0,
                       as_stream(stream), lv, c, out);
  else if (variant == 16)
    hipLaunchKernelGGL((roi_align_fwd_lds_kernel<256, 0, 128>),
                       dim3((unsigned)num_rois, (unsigned)((channels + 127) / 128)), dim3(kRoiThreads), 0,
                       as_stream(stream), lv, c, out);
  else if (variant == 7)
    hipLaunchKernelGGL(roi_align_fwd_buf_kernel<1>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 8)
    hipLaunchKernelGGL(roi_align_fwd_buf_kernel<2>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 4)
    hipLaunchKernelGGL(roi_align_fwd_vec4_kernel<1>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 5)
    hipLaunchKernelGGL(roi_align_fwd_vec4_kernel<2>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 6)
    hipLaunchKernelGGL(roi_align_fwd_vec4_kernel<4>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 3)
    hipLaunchKernelGGL(roi_align_fwd_winreg_kernel<2>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 2)
    hipLaunchKernelGGL(roi_align_fwd_regtap_kernel<2>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else if (variant == 1)
    hipLaunchKernelGGL(roi_align_fwd_staged_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  else
    hipLaunchKernelGGL(roi_align_fwd_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  return check_launch("frh_roi_align_fwd");
}

extern "C" int32_t frh_roi_align_fwd_strided(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                                             const int64_t* strides, const float* scales, int32_t batch,
                                             int32_t channels, const float* rois, const int64_t* roi_levels,
                                             int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                             int32_t sampling_ratio, int32_t aligned, float* out, void* stream) {
  return frh_roi_align_fwd_variant(-1, num_levels, feats, feat_hw, strides, scales, batch, channels, rois,
                                   roi_levels, num_rois, pooled_h, pooled_w, sampling_ratio, aligned, out, stream);
}

extern "C" int32_t frh_roi_align_bwd_strided(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                                             const int64_t* strides, const float* scales, int32_t batch,
                                             int32_t channels, const float* rois, const int64_t* roi_levels,
                                             int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                             int32_t sampling_ratio, int32_t aligned, const float* grad_out,
                                             void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  RoiLevels lv;
  r = make_levels(num_levels, nullptr, grad_feats, feat_hw, strides, scales, &lv);
  if (r) return r;
  if (num_rois == 0) return FRH_OK;
  FRH_REQUIRE(grad_feats && grad_out, "null pointer argument");
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  dim3 grid((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk));
  hipLaunchKernelGGL(roi_align_bwd_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, grad_out);
  return check_launch("frh_roi_align_bwd");
}

// dense-layout convenience entry points (header): layout 0 = NCHW, 1 = NHWC
static void dense_strides(int32_t L, const int32_t* hw, int32_t C, int32_t layout, int64_t* st) {
  for (int l = 0; l < L; ++l) {
    int64_t H = hw[2 * l], W = hw[2 * l + 1];
    if (layout == 0) {
      st[4 * l] = C * H * W;
      st[4 * l + 1] = H * W;
      st[4 * l + 2] = W;
      st[4 * l + 3] = 1;
    } else {
      st[4 * l] = C * H * W;
      st[4 * l + 1] = 1;
      st[4 * l + 2] = W * C;
      st[4 * l + 3] = C;
    }
  }
}

extern "C" int32_t frh_roi_align_fwd(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                                     const float* scales, int32_t batch, int32_t channels, int32_t layout,
                                     const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                     int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                     float* out, void* stream) {
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS && feat_hw, "bad levels");
  FRH_REQUIRE(layout == 0 || layout == 1, "layout must be 0 (NCHW) or 1 (NHWC)");
  int64_t st[4 * FRH_MAX_LEVELS];
  dense_strides(num_levels, feat_hw, channels, layout, st);
  return frh_roi_align_fwd_strided(num_levels, feats, feat_hw, st, scales, batch, channels, rois, roi_levels,
                                   num_rois, pooled_h, pooled_w, sampling_ratio, aligned, out, stream);
}

extern "C" int32_t frh_roi_align_bwd(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                                     const float* scales, int32_t batch, int32_t channels, int32_t layout,
                                     const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                     int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                     const float* grad_out, void* stream) {
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS && feat_hw, "bad levels");
  FRH_REQUIRE(layout == 0 || layout == 1, "layout must be 0 (NCHW) or 1 (NHWC)");
  int64_t st[4 * FRH_MAX_LEVELS];
  dense_strides(num_levels, feat_hw, channels, layout, st);
  return frh_roi_align_bwd_strided(num_levels, grad_feats, feat_hw, st, scales, batch, channels, rois, roi_levels,
                                   num_rois, pooled_h, pooled_w, sampling_ratio, aligned, grad_out, stream);
}

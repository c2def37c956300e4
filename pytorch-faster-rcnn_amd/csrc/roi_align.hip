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

extern "C" int32_t frh_roi_align_fwd_strided(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                                             const int64_t* strides, const float* scales, int32_t batch,
                                             int32_t channels, const float* rois, const int64_t* roi_levels,
                                             int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                             int32_t sampling_ratio, int32_t aligned, float* out, void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  FRH_REQUIRE((feats && out) || num_rois == 0, "null pointer argument");
  RoiLevels lv;
  r = make_levels(num_levels, feats, nullptr, feat_hw, strides, scales, &lv);
  if (r) return r;
  if (num_rois == 0) return FRH_OK;
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  dim3 grid((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk));
  hipLaunchKernelGGL(roi_align_fwd_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, out);
  return check_launch("frh_roi_align_fwd");
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

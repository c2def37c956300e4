// a1/a2: anchor grids for all levels in one launch, inside-image/grid masks.
// Reference: lib/anchor.py:80-129, lib/region.py:10-29, lib/heads/anchor_head.py:89-99.
#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace frh {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int32_t check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return FRH_ELAUNCH;
  }
  return FRH_OK;
}

struct LevelGrid {
  int32_t n;                      // levels
  int32_t A;                      // anchors per location
  int32_t h[FRH_MAX_LEVELS], w[FRH_MAX_LEVELS];
  int32_t in_h[FRH_MAX_LEVELS], in_w[FRH_MAX_LEVELS];
  int64_t off[FRH_MAX_LEVELS + 1];  // first flat index of each level
  float stride[FRH_MAX_LEVELS];
};

// locate level of flat anchor index i (levels are few: linear scan)
__device__ __forceinline__ int level_of(const LevelGrid& g, int64_t i) {
  int l = 0;
  while (l + 1 < g.n && i >= g.off[l + 1]) ++l;
  return l;
}

// Anchor (x1,y1,x2,y2) = centre -/+ size/2 in f32; the centre
// linspace(0, s*g, g+1)[:-1] + s/2 is exact (anchor.py:112-119).
__global__ void anchor_grid_kernel(LevelGrid g, const float* __restrict__ ws,
                                   const float* __restrict__ hs, int center_lt,
                                   float* __restrict__ out, int64_t ld) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.off[g.n]) return;
  int l = level_of(g, i);
  int64_t r = i - g.off[l];
  int64_t hw = (int64_t)g.h[l] * g.w[l];
  int a = (int)(r / hw);
  int64_t p = r - (int64_t)a * hw;
  int y = (int)(p / g.w[l]);
  int x = (int)(p - (int64_t)y * g.w[l]);
  float s = g.stride[l];
  float cx = (float)x * s, cy = (float)y * s;
  if (!center_lt) {
    cx = cx + s / 2.0f;
    cy = cy + s / 2.0f;
  }
  float aw = ws[l * g.A + a], ah = hs[l * g.A + a];
  float hw2 = aw / 2.0f, hh2 = ah / 2.0f;
  out[i] = cx - hw2;
  out[ld + i] = cy - hh2;
  out[2 * ld + i] = cx + hw2;
  out[3 * ld + i] = cy + hh2;
}

__global__ void inside_mask_kernel(LevelGrid g, const float* __restrict__ anc, int64_t ld,
                                   int img_h, int img_w, int border, uint8_t* __restrict__ mask) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.off[g.n]) return;
  int l = level_of(g, i);
  int64_t r = i - g.off[l];
  int64_t hw = (int64_t)g.h[l] * g.w[l];
  int64_t p = r % hw;
  int y = (int)(p / g.w[l]);
  int x = (int)(p - (int64_t)y * g.w[l]);
  bool in_grid = (y < g.in_h[l]) && (x < g.in_w[l]);
  bool in_img = true;
  if (border >= 0) {
    // comparisons of f32 anchors with python ints happen in f32 (region.py:26-29)
    float fb = (float)(-border);
    in_img = (anc[i] >= fb) && (anc[ld + i] >= fb) && (anc[2 * ld + i] < (float)(img_w + border)) &&
             (anc[3 * ld + i] < (float)(img_h + border));
  }
  mask[i] = (in_grid && in_img) ? 1 : 0;
}

static int32_t make_grid(int32_t num_levels, const int32_t* grid_hw, const float* strides,
                         const int32_t* in_hw, int32_t A, LevelGrid* g) {
  FRH_REQUIRE(num_levels >= 1 && num_levels <= FRH_MAX_LEVELS, "num_levels %d out of range", num_levels);
  FRH_REQUIRE(A >= 1, "num_anchors must be >= 1");
  FRH_REQUIRE(grid_hw != nullptr, "grid_hw is null");
  g->n = num_levels;
  g->A = A;
  g->off[0] = 0;
  for (int l = 0; l < num_levels; ++l) {
    g->h[l] = grid_hw[2 * l];
    g->w[l] = grid_hw[2 * l + 1];
    FRH_REQUIRE(g->h[l] > 0 && g->w[l] > 0, "level %d has an empty grid", l);
    g->stride[l] = strides ? strides[l] : 0.f;
    g->in_h[l] = in_hw ? in_hw[2 * l] : g->h[l];
    g->in_w[l] = in_hw ? in_hw[2 * l + 1] : g->w[l];
    g->off[l + 1] = g->off[l] + (int64_t)A * g->h[l] * g->w[l];
  }
  return FRH_OK;
}

}  // namespace frh

using namespace frh;

extern "C" int32_t frh_abi_version(void) { return FRH_ABI_VERSION; }
extern "C" const char* frh_last_error(void) { return frh::g_err; }

extern "C" int32_t frh_anchor_grid(int32_t num_levels, const int32_t* grid_hw, const float* strides,
                                   const float* ws, const float* hs, int32_t num_anchors,
                                   int32_t center_lt, float* out, int64_t ld, void* stream) {
  LevelGrid g;
  int32_t st = make_grid(num_levels, grid_hw, strides, nullptr, num_anchors, &g);
  if (st) return st;
  FRH_REQUIRE(strides && ws && hs && out, "null pointer argument");
  FRH_REQUIRE(ld >= g.off[num_levels], "ld %lld < total anchors %lld", (long long)ld,
              (long long)g.off[num_levels]);
  int64_t n = g.off[num_levels];
  int threads = 256;
  hipLaunchKernelGGL(anchor_grid_kernel, dim3((unsigned)((n + threads - 1) / threads)), dim3(threads),
                     0, as_stream(stream), g, ws, hs, center_lt, out, ld);
  return check_launch("frh_anchor_grid");
}

extern "C" int32_t frh_inside_mask(const float* anchors, int64_t ld, int32_t num_levels,
                                   const int32_t* grid_hw, const int32_t* in_hw, int32_t num_anchors,
                                   int32_t img_h, int32_t img_w, int32_t allowed_border,
                                   uint8_t* mask, void* stream) {
  LevelGrid g;
  int32_t st = make_grid(num_levels, grid_hw, nullptr, in_hw, num_anchors, &g);
  if (st) return st;
  FRH_REQUIRE(anchors && mask && in_hw, "null pointer argument");
  int64_t n = g.off[num_levels];
  int threads = 256;
  hipLaunchKernelGGL(inside_mask_kernel, dim3((unsigned)((n + threads - 1) / threads)), dim3(threads),
                     0, as_stream(stream), g, anchors, ld, img_h, img_w, allowed_border, mask);
  return check_launch("frh_inside_mask");
}

// RoIPool (torchvision.ops.RoIPool semantics) for the C4 config
// (reference configs/faster_rcnn_r50.py:26, registry lib/builder.py:9,22).
// One thread per output element; max over the quantised bin, argmax kept for
// the backward scatter.
#include <math.h>

#include "common.h"

namespace frh {

__global__ void roi_pool_fwd_kernel(const float* __restrict__ feat, int64_t sb, int64_t sc, int64_t sy, int64_t sx,
                                    int H, int W, float scale, const float* __restrict__ rois, int64_t K, int C,
                                    int ph, int pw, float* __restrict__ out, int32_t* __restrict__ argmax) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = K * C * ph * pw;
  if (idx >= total) return;
  int px = (int)(idx % pw);
  int py = (int)((idx / pw) % ph);
  int c = (int)((idx / ((int64_t)pw * ph)) % C);
  int64_t k = idx / ((int64_t)pw * ph * C);
  const float* r = rois + k * 5;
  int b = (int)r[0];
  int rsw = (int)roundf(r[1] * scale), rsh = (int)roundf(r[2] * scale);
  int rew = (int)roundf(r[3] * scale), reh = (int)roundf(r[4] * scale);
  int rw = max(rew - rsw + 1, 1), rh = max(reh - rsh + 1, 1);
  float bh = (float)rh / (float)ph, bw = (float)rw / (float)pw;
  int hs = (int)floorf((float)py * bh), ws = (int)floorf((float)px * bw);
  int he = (int)ceilf((float)(py + 1) * bh), we = (int)ceilf((float)(px + 1) * bw);
  hs = min(max(hs + rsh, 0), H);
  he = min(max(he + rsh, 0), H);
  ws = min(max(ws + rsw, 0), W);
  we = min(max(we + rsw, 0), W);
  bool empty = (he <= hs) || (we <= ws);
  float m = empty ? 0.0f : -3.402823466e+38f;
  int mi = -1;
  const float* f = feat + b * sb + c * sc;
  for (int y = hs; y < he; ++y)
    for (int x = ws; x < we; ++x) {
      float v = f[y * sy + x * sx];
      if (v > m) {
        m = v;
        mi = y * W + x;
      }
    }
  out[idx] = m;
  argmax[idx] = mi;
}

__global__ void roi_pool_bwd_kernel(float* __restrict__ grad, int64_t sb, int64_t sc, int64_t sy, int64_t sx, int W,
                                    const float* __restrict__ rois, int64_t K, int C, int ph, int pw,
                                    const float* __restrict__ gout, const int32_t* __restrict__ argmax) {
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = K * C * ph * pw;
  if (idx >= total) return;
  int mi = argmax[idx];
  if (mi < 0) return;
  int c = (int)((idx / ((int64_t)pw * ph)) % C);
  int64_t k = idx / ((int64_t)pw * ph * C);
  int b = (int)rois[k * 5];
  int y = mi / W, x = mi - (mi / W) * W;
  atomicAdd(&grad[b * sb + c * sc + y * sy + x * sx], gout[idx]);
}

}  // namespace frh

using namespace frh;

extern "C" int32_t frh_roi_pool_fwd(const float* feat, const int64_t* strides, int32_t height, int32_t width,
                                    int32_t channels, float spatial_scale, const float* rois, int64_t num_rois,
                                    int32_t pooled_h, int32_t pooled_w, float* out, int32_t* argmax, void* stream) {
  FRH_REQUIRE(num_rois >= 0 && channels >= 1 && pooled_h >= 1 && pooled_w >= 1 && height > 0 && width > 0,
              "bad sizes");
  if (num_rois == 0) return FRH_OK;
  FRH_REQUIRE(feat && strides && rois && out && argmax, "null pointer argument");
  int64_t total = num_rois * channels * pooled_h * pooled_w;
  hipLaunchKernelGGL(roi_pool_fwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                     feat, strides[0], strides[1], strides[2], strides[3], height, width, spatial_scale, rois,
                     num_rois, channels, pooled_h, pooled_w, out, argmax);
  return check_launch("frh_roi_pool_fwd");
}

extern "C" int32_t frh_roi_pool_bwd(float* grad_feat, const int64_t* strides, int32_t height, int32_t width,
                                    int32_t channels, const float* rois, int64_t num_rois, int32_t pooled_h,
                                    int32_t pooled_w, const float* grad_out, const int32_t* argmax, void* stream) {
  FRH_REQUIRE(num_rois >= 0 && channels >= 1 && pooled_h >= 1 && pooled_w >= 1, "bad sizes");
  if (num_rois == 0) return FRH_OK;
  FRH_REQUIRE(grad_feat && strides && rois && grad_out && argmax, "null pointer argument");
  (void)height;
  int64_t total = num_rois * channels * pooled_h * pooled_w;
  hipLaunchKernelGGL(roi_pool_bwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream),
                     grad_feat, strides[0], strides[1], strides[2], strides[3], width, rois, num_rois, channels,
                     pooled_h, pooled_w, grad_out, argmax);
  return check_launch("frh_roi_pool_bwd");
}

// Backbone epilogue: frozen BatchNorm (+ residual add) (+ ReLU) in one HBM pass.
//   y = act(x * s[c] + b[c] (+ skip)),  s = gamma / sqrt(var + eps),  b = beta - mean * s
// The reference's ResNet keeps every BN in eval mode (lib/backbones.py:69-76, 116-121), so
// each BN is a per-channel affine map of its conv's output; PyTorch runs it as three
// kernels (BN, add, clamp) with a full read + write of the activation each.  Here one
// workgroup row handles one (image, channel) plane: s and b are computed once per block
// from the BN parameters (no host-side folding, so trainable gamma/beta stay live), and
// the plane streams through float4 loads/stores.  In place (y == x) is allowed.
#include <math.h>

#include "common.h"

namespace frh {

constexpr int kBnThreads = 256;
constexpr int kBnVec = 4;  // float4 per thread per block-row step

__global__ void __launch_bounds__(kBnThreads) bn_act_kernel(const float4* x, const float4* skip, float4* y,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ var, float eps, int C,
                                                            int64_t hw4, int tiles, int relu) {
  const int64_t plane = blockIdx.x / tiles;
  const int tile = blockIdx.x - (int)(plane * tiles);
  const int c = (int)(plane % C);
  const float s = (gamma ? gamma[c] : 1.0f) / sqrtf(var[c] + eps);
  const float b = (beta ? beta[c] : 0.0f) - mean[c] * s;
  const int64_t base = plane * hw4;
  for (int64_t i0 = (int64_t)tile * kBnThreads * kBnVec + threadIdx.x; i0 < hw4;
       i0 += (int64_t)tiles * kBnThreads * kBnVec) {
    float4 v[kBnVec], k[kBnVec];
#pragma unroll
    for (int u = 0; u < kBnVec; ++u) {
      const int64_t i = i0 + u * kBnThreads;
      if (i < hw4) {
        v[u] = x[base + i];
        if (skip) k[u] = skip[base + i];
      }
    }
#pragma unroll
    for (int u = 0; u < kBnVec; ++u) {
      const int64_t i = i0 + u * kBnThreads;
      if (i < hw4) {
        float4 r = make_float4(v[u].x * s + b, v[u].y * s + b, v[u].z * s + b, v[u].w * s + b);
        if (skip) r = make_float4(r.x + k[u].x, r.y + k[u].y, r.z + k[u].z, r.w + k[u].w);
        if (relu) r = make_float4(fmaxf(r.x, 0.0f), fmaxf(r.y, 0.0f), fmaxf(r.z, 0.0f), fmaxf(r.w, 0.0f));
        y[base + i] = r;
      }
    }
  }
}

}  // namespace frh

using namespace frh;

extern "C" int32_t frh_bn_act(const float* x, const float* skip, float* y, const float* gamma, const float* beta,
                              const float* mean, const float* var, float eps, int64_t n, int32_t c, int64_t hw,
                              int32_t relu, void* stream) {
  FRH_REQUIRE(n >= 0 && c >= 1 && hw >= 0, "bad sizes");
  if (n == 0 || hw == 0) return FRH_OK;
  FRH_REQUIRE(x && y && mean && var, "null pointer argument");
  FRH_REQUIRE(hw % 4 == 0, "plane size %lld must be a multiple of 4", (long long)hw);
  FRH_REQUIRE(((uintptr_t)x | (uintptr_t)y | (uintptr_t)skip) % 16 == 0, "tensors must be 16-byte aligned");
  const int64_t hw4 = hw / 4;
  const int64_t per_block = (int64_t)kBnThreads * kBnVec;
  const int64_t tiles = (hw4 + per_block - 1) / per_block;
  FRH_REQUIRE(n * (int64_t)c * tiles < ((int64_t)1 << 31), "too many blocks");
  hipLaunchKernelGGL(bn_act_kernel, dim3((unsigned)(n * c * tiles)), dim3(kBnThreads), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(x), reinterpret_cast<const float4*>(skip),
                     reinterpret_cast<float4*>(y), gamma, beta, mean, var, eps, (int)c, hw4, (int)tiles, (int)relu);
  return check_launch("frh_bn_act");
}

// Stem: frozen BN + ReLU + 3x3 / stride-2 / pad-1 max pool (lib/backbones.py: the ResNet
// stem relu(bn1(conv1(x))) -> maxpool) in one pass: the conv1 output is read once and only
// the pooled map is written (PyTorch: BN-act pass + max_pool2d_with_indices, which also
// writes int64 indices).  Thread = four consecutive outputs of one row: input columns
// 8q - 1 .. 8q + 7 of the (up to) three input rows, as two float4 + one scalar each.
// Max over the window's in-bounds elements (the pool's -inf padding); same f32 BN
// arithmetic as bn_act_kernel, so every output equals max_pool2d(bn_act(x)) bit for bit.
namespace frh {

__global__ void __launch_bounds__(kBnThreads) bn_act_maxpool_kernel(const float* __restrict__ x, float4* y,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ beta,
                                                                   const float* __restrict__ mean,
                                                                   const float* __restrict__ var, float eps, int C,
                                                                   int H, int W, int OH, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * kBnThreads + threadIdx.x;
  if (t >= total) return;
  const int OW4 = W / 8;  // (OW = W / 2) / 4 output quads per row
  const int q = (int)(t % OW4);
  const int64_t r = t / OW4;
  const int oy = (int)(r % OH);
  const int64_t plane = r / OH;
  const int c = (int)(plane % C);
  const float s = (gamma ? gamma[c] : 1.0f) / sqrtf(var[c] + eps);
  const float b = (beta ? beta[c] : 0.0f) - mean[c] * s;
  auto act = [&](float v) { return fmaxf(v * s + b, 0.0f); };
  float m0 = -INFINITY, m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY;
  const float* xp = x + plane * (int64_t)H * W;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy) {
    const int iy = 2 * oy + dy;
    if (iy < 0 || iy >= H) continue;
    const float* row = xp + (int64_t)iy * W + 8 * q;
    const float4 a = *reinterpret_cast<const float4*>(row);
    const float4 e = *reinterpret_cast<const float4*>(row + 4);
    const float l = q > 0 ? act(row[-1]) : -INFINITY;
    const float a0 = act(a.x), a1 = act(a.y), a2 = act(a.z), a3 = act(a.w);
    const float e0 = act(e.x), e1 = act(e.y), e2 = act(e.z), e3 = act(e.w);
    m0 = fmaxf(m0, fmaxf(l, fmaxf(a0, a1)));
    m1 = fmaxf(m1, fmaxf(a1, fmaxf(a2, a3)));
    m2 = fmaxf(m2, fmaxf(a3, fmaxf(e0, e1)));
    m3 = fmaxf(m3, fmaxf(e1, fmaxf(e2, e3)));
  }
  y[t] = make_float4(m0, m1, m2, m3);
}

}  // namespace frh

extern "C" int32_t frh_bn_act_maxpool(const float* x, float* y, const float* gamma, const float* beta,
                                      const float* mean, const float* var, float eps, int64_t n, int32_t c, int32_t h,
                                      int32_t w, void* stream) {
  FRH_REQUIRE(n >= 0 && c >= 1 && h >= 1 && w >= 8, "bad sizes");
  if (n == 0) return FRH_OK;
  FRH_REQUIRE(x && y && mean && var, "null pointer argument");
  FRH_REQUIRE(w % 8 == 0, "width %d must be a multiple of 8", w);
  FRH_REQUIRE(((uintptr_t)x | (uintptr_t)y) % 16 == 0, "tensors must be 16-byte aligned");
  const int oh = (h - 1) / 2 + 1;
  const int64_t total = n * (int64_t)c * oh * (w / 8);
  const int64_t blocks = (total + kBnThreads - 1) / kBnThreads;
  FRH_REQUIRE(blocks < ((int64_t)1 << 31), "too many blocks");
  hipLaunchKernelGGL(bn_act_maxpool_kernel, dim3((unsigned)blocks), dim3(kBnThreads), 0, as_stream(stream), x,
                     reinterpret_cast<float4*>(y), gamma, beta, mean, var, eps, (int)c, (int)h, (int)w, oh, total);
  return check_launch("frh_bn_act_maxpool");
}

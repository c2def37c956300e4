// FPN top-down merge, producing channels-last (NHWC) levels.
// Reference: lib/necks.py:72-84 (FPN.forward: lateral 1x1 convs, then
// laterals[i - 1] += F.interpolate(laterals[i], size=laterals[i - 1].shape[2:],
// mode='nearest') from the top level down, then the 3x3 output convs).
//
// out[b, y, x, c] = (lat[b, c, y, x] + bias[c]) + up[b, iy(y), ix(x), c]
// lat: the lateral conv's output (any strides; NCHW from the backbone's NCHW stages),
// without its bias when bias is given (the conv's bias add folded in here: the same f32
// add PyTorch's conv epilogue does, one HBM pass fewer per level).
// up:  the merged coarser level (NHWC, from the previous call), or none for the top level.
// iy / ix: torch's nearest rule, src = min(floor(dst * (float)in / out), in - 1) (exact
// halving when out == 2 * in).  f32 adds in the reference's order: bit-identical to it.
// The transpose runs through a 64 x 64 LDS tile: NCHW rows are read along x, NHWC rows
// written along c, 16 B per lane on both sides when the shapes allow it.  The output
// feeds the 3x3 output convs in channels-last form (MIOpen's faster layout for them,
// DESIGN.md §3) and, through them, the NHWC RoIAlign.  One pass replaces PyTorch's
// upsample (read 1/4, write 1) + add (read 2, write 1) of every level.
#include <algorithm>

#include "common.h"

namespace frh {

constexpr int kFpnTile = 64;
constexpr int kFpnThreads = 256;

__device__ __forceinline__ int nearest_src(int dst, int in, int out) {
  if (out == 2 * in) return dst >> 1;
  if (out == in) return dst;
  const int s = (int)floorf((float)dst * ((float)in / (float)out));
  return s < in - 1 ? s : in - 1;
}

struct FpnMergeArgs {
  const float* lat;
  int64_t lsb, lsc, lsy, lsx;
  const float* bias;  // nullable: [C]
  const float* up;  // nullable: [B, uh, uw, C] contiguous
  int uh, uw;
  float* out;       // [B, H, W, C] contiguous
  int B, C, H, W;
  int vec;          // 16-B paths allowed (x rows and channels multiples of 4, aligned)
};

// grid (ceil(W / 64) * ceil(C / 64), H, B)
__global__ void __launch_bounds__(kFpnThreads) fpn_merge_nhwc_kernel(FpnMergeArgs a) {
  __shared__ float tile[kFpnTile][kFpnTile + 1];  // [c][x]
  const int ntx = (a.W + kFpnTile - 1) / kFpnTile;
  const int x0 = (blockIdx.x % ntx) * kFpnTile, c0 = (blockIdx.x / ntx) * kFpnTile;
  const int y = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const float* lrow = a.lat + (int64_t)b * a.lsb + (int64_t)y * a.lsy;
  // load: 64 channel rows x 64 columns of the lateral map
  if (a.vec) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = r * kFpnThreads + t, c = idx >> 4, xq = (idx & 15) * 4;
      if (c0 + c < a.C && x0 + xq < a.W) {
        const float4 v = *reinterpret_cast<const float4*>(lrow + (int64_t)(c0 + c) * a.lsc + (int64_t)(x0 + xq) * a.lsx);
        tile[c][xq] = v.x, tile[c][xq + 1] = v.y, tile[c][xq + 2] = v.z, tile[c][xq + 3] = v.w;
      }
    }
  } else {
    for (int idx = t; idx < kFpnTile * kFpnTile; idx += kFpnThreads) {
      const int c = idx >> 6, x = idx & 63;
      if (c0 + c < a.C && x0 + x < a.W) tile[c][x] = lrow[(int64_t)(c0 + c) * a.lsc + (int64_t)(x0 + x) * a.lsx];
    }
  }
  __syncthreads();
  const int iy = a.up ? nearest_src(y, a.uh, a.H) : 0;
  float* orow = a.out + ((int64_t)b * a.H + y) * a.W * a.C;
  const float* urow = a.up ? a.up + ((int64_t)b * a.uh + iy) * a.uw * a.C : nullptr;
  if (a.vec) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int idx = r * kFpnThreads + t, x = idx >> 4, cq = (idx & 15) * 4;
      if (x0 + x < a.W && c0 + cq < a.C) {
        float4 v = make_float4(tile[cq][x], tile[cq + 1][x], tile[cq + 2][x], tile[cq + 3][x]);
        if (a.bias) {
          const float4 bb = *reinterpret_cast<const float4*>(a.bias + c0 + cq);
          v = make_float4(v.x + bb.x, v.y + bb.y, v.z + bb.z, v.w + bb.w);
        }
        if (urow) {
          const float4 u = *reinterpret_cast<const float4*>(urow + (int64_t)nearest_src(x0 + x, a.uw, a.W) * a.C + c0 + cq);
          v = make_float4(v.x + u.x, v.y + u.y, v.z + u.z, v.w + u.w);
        }
        *reinterpret_cast<float4*>(orow + (int64_t)(x0 + x) * a.C + c0 + cq) = v;
      }
    }
  } else {
    for (int idx = t; idx < kFpnTile * kFpnTile; idx += kFpnThreads) {
      const int x = idx >> 6, c = idx & 63;
      if (x0 + x < a.W && c0 + c < a.C) {
        float v = tile[c][x];
        if (a.bias) v = v + a.bias[c0 + c];
        if (urow) v = v + urow[(int64_t)nearest_src(x0 + x, a.uw, a.W) * a.C + c0 + c];
        orow[(int64_t)(x0 + x) * a.C + c0 + c] = v;
      }
    }
  }
}

}  // namespace frh

using namespace frh;

extern "C" int32_t frh_fpn_merge_nhwc(const float* lat, const int64_t* lat_strides, const float* bias, const float* up,
                                      int32_t up_h, int32_t up_w, float* out, int32_t batch, int32_t channels,
                                      int32_t height, int32_t width, void* stream) {
  FRH_REQUIRE(batch >= 0 && channels >= 0 && height >= 0 && width >= 0, "bad sizes");
  if ((int64_t)batch * channels * height * width == 0) return FRH_OK;
  FRH_REQUIRE(lat && lat_strides && out, "null pointer argument");
  FRH_REQUIRE(!up || (up_h >= 1 && up_w >= 1), "bad coarser-level size");
  FRH_REQUIRE(height <= 65535 && batch <= 65535, "grid too large");
  FpnMergeArgs a{lat, lat_strides[0], lat_strides[1], lat_strides[2], lat_strides[3], bias, up, up_h, up_w, out,
                 batch, channels, height, width, 0};
  a.vec = lat_strides[3] == 1 && lat_strides[1] % 4 == 0 && lat_strides[2] % 4 == 0 && lat_strides[0] % 4 == 0 &&
          width % 4 == 0 && channels % 4 == 0 &&
          ((uintptr_t)lat | (uintptr_t)up | (uintptr_t)out | (uintptr_t)bias) % 16 == 0;
  const int ntx = (width + kFpnTile - 1) / kFpnTile, ntc = (channels + kFpnTile - 1) / kFpnTile;
  hipLaunchKernelGGL(fpn_merge_nhwc_kernel, dim3((unsigned)(ntx * ntc), (unsigned)height, (unsigned)batch),
                     dim3(kFpnThreads), 0, as_stream(stream), a);
  return check_launch("frh_fpn_merge_nhwc");
}

// ---------------------------------------------------------------- conv bias + ReLU epilogue
// y[r, c] = act(y[r, c] + bias[c]) in place over a channels-last map viewed as [rows, C]
// (rows = B * H * W): the RPN head's 3x3 conv (lib/heads/rpn_head.py: relu(conv(x))) runs
// without its bias in MIOpen's NHWC solver and this one pass replaces PyTorch's bias add +
// ReLU (two read + write passes).  Same f32 add, then max(., 0): bit-identical.
namespace frh {

constexpr int kBiasActThreads = 256;

template <bool kRelu>
__global__ void __launch_bounds__(kBiasActThreads) bias_act_nhwc_kernel(float4* y, const float4* bias, int64_t n4,
                                                                        int c4) {
  const int64_t stride = (int64_t)gridDim.x * kBiasActThreads;
  for (int64_t i = (int64_t)blockIdx.x * kBiasActThreads + threadIdx.x; i < n4; i += stride) {
    const float4 b = bias[i % c4];
    float4 v = y[i];
    v = make_float4(v.x + b.x, v.y + b.y, v.z + b.z, v.w + b.w);
    if (kRelu) v = make_float4(fmaxf(v.x, 0.0f), fmaxf(v.y, 0.0f), fmaxf(v.z, 0.0f), fmaxf(v.w, 0.0f));
    y[i] = v;
  }
}

}  // namespace frh

extern "C" int32_t frh_bias_act_nhwc(float* y, const float* bias, int64_t rows, int32_t channels, int32_t relu,
                                     void* stream) {
  FRH_REQUIRE(rows >= 0 && channels >= 1, "bad sizes");
  if (rows == 0) return FRH_OK;
  FRH_REQUIRE(y && bias, "null pointer argument");
  FRH_REQUIRE(channels % 4 == 0 && ((uintptr_t)y | (uintptr_t)bias) % 16 == 0,
              "channels must be a multiple of 4 and both tensors 16-byte aligned");
  const int64_t n4 = rows * channels / 4;
  const int64_t blocks = std::min<int64_t>((n4 + kBiasActThreads - 1) / kBiasActThreads, 256 * 32);
  auto* y4 = reinterpret_cast<float4*>(y);
  auto* b4 = reinterpret_cast<const float4*>(bias);
  if (relu)
    hipLaunchKernelGGL(bias_act_nhwc_kernel<true>, dim3((unsigned)blocks), dim3(kBiasActThreads), 0, as_stream(stream),
                       y4, b4, n4, channels / 4);
  else
    hipLaunchKernelGGL(bias_act_nhwc_kernel<false>, dim3((unsigned)blocks), dim3(kBiasActThreads), 0,
                       as_stream(stream), y4, b4, n4, channels / 4);
  return check_launch("frh_bias_act_nhwc");
}

// TOOLS-ONLY RoIAlign forward laboratory (see frcnn_tools.h).  Variant 0 is the product's
// instantiation, so A/B runs compare against exactly what ships; 1 is its per-wave stamped
// build.
#include "frcnn_tools.h"
#include "roi_kernels.h"

using namespace frh;

extern "C" size_t frh_roi_align_workspace(int64_t num_rois) { return (size_t)(num_rois > 0 ? num_rois : 1) * 64; }

extern "C" int32_t frh_roi_align_fwd_variant(int32_t variant, int32_t num_levels, const float* const* feats,
                                             const int32_t* feat_hw, const int64_t* strides, const float* scales,
                                             int32_t batch, int32_t channels, const float* rois,
                                             const int64_t* roi_levels, int64_t num_rois, int32_t pooled_h,
                                             int32_t pooled_w, int32_t sampling_ratio, int32_t aligned, float* out,
                                             void* workspace, size_t ws_bytes, void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  FRH_REQUIRE((feats && out) || num_rois == 0, "null pointer argument");
  RoiLevels lv;
  r = make_levels(num_levels, feats, nullptr, feat_hw, strides, scales, &lv);
  if (r) return r;
  if (num_rois == 0) return FRH_OK;
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  const FwdCaps f = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
  FRH_REQUIRE(pair_ok(f, channels, pooled_h, pooled_w), "the pair kernel does not take this shape");
  const int64_t total = num_rois * ((channels + kPairChunk - 1) / kPairChunk);
  FRH_REQUIRE(total <= (int64_t)0x7fffffff - 7, "too many RoIs");
  const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
  hipStream_t st = as_stream(stream);
  if (variant == 0)
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kCpolNT, false>), g1, dim3(kWave), 0, st, lv, c, out);
  else if (variant == 1)
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kCpolNT, true>), g1, dim3(kWave), 0, st, lv, c, out);
  else
    FRH_REQUIRE(false, "roi_align variant %d unknown", variant);
  return check_launch("frh_roi_align_fwd_variant");
}

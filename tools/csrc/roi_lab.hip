// TOOLS-ONLY RoIAlign forward laboratory (see frcnn_tools.h).  Variant 0 is the product's
// instantiation, so A/B runs compare against exactly what ships; 1 is its per-wave stamped
// build.
#include "frcnn_tools.h"
#include "roi_kernels.h"
#include "roi_lab_kernels.h"

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
  lv.B = batch;
  if (num_rois == 0) return FRH_OK;
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  hipStream_t st = as_stream(stream);
  if (variant == 23 || variant == 24) {  // software-pipelined persistent quad kernel (23: 8 waves per CU, 24: 12;
                                        // 2 waves per SIMD by registers: 24 queues its surplus)
    const FwdCaps fq = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
    FRH_REQUIRE(quad_ok(fq, lv, channels, pooled_h, pooled_w), "the quad kernel does not take this shape");
    int dev = 0, ncu = 0;
    FRH_HIP(hipGetDevice(&dev));
    FRH_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int wpc = variant == 23 ? 8 : 12;
    const dim3 gq((unsigned)(8 * ((ncu * wpc + 7) / 8)));
    hipLaunchKernelGGL((roi_align_fwd_quadp_kernel<kCpolNT>), gq, dim3(kWave), 0, st, lv, c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  if (variant >= 28 && variant <= 70) {  // band kernel: 28 product (208 cells), 29 stamped, 30 176 cells,
                                         // 31 256 cells, 32 208 cells at 4 waves per SIMD
    const FwdCaps fq = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
    FRH_REQUIRE(quad_ok(fq, lv, channels, pooled_h, pooled_w) && band_fits(pooled_h, pooled_w, 160),
                "the band kernel does not take this shape");
    const int64_t tq = num_rois * ((channels + 4 * kQuadWave - 1) / (4 * kQuadWave));
    const dim3 gq((unsigned)(8 * ((tq + 7) / 8)));
    if (variant == 28)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 29)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, true, 208>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 30)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 176>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 31)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 256>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 32)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 4>), gq, dim3(kWave), 0, st, lv, c,
                         out);
    else if (variant == 33)  // no quad rotation
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 3, 0>), gq, dim3(kWave), 0, st, lv,
                         c, out);
    else if (variant == 34)  // rotation, per-step stores
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 3, 2>), gq, dim3(kWave), 0, st, lv,
                         c, out);
    else if (variant == 35)  // hybrid: small windows by the quad path
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 3, 1, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 36)  // hybrid, 160-cell slab (10 KB)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 160, false, 3, 1, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 37)  // hybrid, 160-cell slab, 4 waves per SIMD
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 160, false, 4, 1, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 38)  // hybrid, bands without quad rotation
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 3, 0, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 39)  // hybrid, bands without rotation, stamped
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, true, 208, false, 3, 0, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 40)  // hybrid up to the quad path's D = 2 windows (<= 384 cells), bands above
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 3, 0, 2>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 41)  // hybrid (D = 4), 232-cell slab: 8-row bands
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 0, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 42)  // hybrid (D = 2), 232-cell slab
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 0, 2>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 43)  // hybrid (D = 4), 232-cell slab, rotated quads in the bands
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 1, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 44)  // hybrid (D = 4), 256-cell slab
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 256, false, 3, 0, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 46)  // hybrid (D = 4), 232-cell slab, stores after the last band
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    else if (variant == 47)  // product + windows above 464 cells (3+ bands) by the quad stages
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 464>), gq, dim3(kWave), 0,
                         st, lv, c, out);
    else if (variant == 48)  // product + windows above 348 cells by the quad stages
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 348>), gq, dim3(kWave), 0,
                         st, lv, c, out);
    else if (variant == 49)  // product + windows above 696 cells by the quad stages
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 696>), gq, dim3(kWave), 0,
                         st, lv, c, out);
    else if (variant == 50)  // product + two-quad interleaved whole-window stages up to 464 cells
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 0, 2>), gq, dim3(kWave),
                         0, st, lv, c, out);
    else if (variant == 51)  // as 50, windows above 696 cells by the quad stages
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 696, 2>), gq,
                         dim3(kWave), 0, st, lv, c, out);
    else if (variant == 52)  // as 50 plus one [cell][4 quads] stage for windows <= 232 cells
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 0, 3>), gq, dim3(kWave),
                         0, st, lv, c, out);
    else if (variant == 53)  // as 50, the quad D = 4 stage off (bands below 232 cells are unreachable)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 0, 0, 3>), gq, dim3(kWave),
                         0, st, lv, c, out);
    else if (variant == 54)  // the product's paths on a 208-cell slab (13 KB: 12 waves per CU by LDS)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 3, 3, 4, 0, 2>), gq, dim3(kWave),
                         0, st, lv, c, out);
    else if (variant == 55)  // as 54, 4 waves per SIMD requested
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 208, false, 4, 3, 4, 0, 2>), gq, dim3(kWave),
                         0, st, lv, c, out);
    else if (variant == 56)  // the product kernel, stamped (8 int64 per item after the output)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, true, 232, false, 3, 3, 4, 0, 2>), gq, dim3(kWave),
                         0, st, lv, c, out);
    else if (variant == 57 || variant == 58) {  // the product's paths, one wave per (RoI, chunk pair); 58 stamped
      const int64_t tp = num_rois * (((channels + 4 * kQuadWave - 1) / (4 * kQuadWave) + 1) / 2);
      const dim3 gp((unsigned)(8 * ((tp + 7) / 8)));
      if (variant == 57)
        hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 0, 2, 2>), gp,
                           dim3(kWave), 0, st, lv, c, out);
      else
        hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, true, 232, false, 3, 3, 4, 0, 2, 2>), gp,
                           dim3(kWave), 0, st, lv, c, out);
    }
    else if (variant == 59)  // the product kernel with the chunk-major item order (round 4's quad kernel order)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 232, false, 3, 3, 4, 0, 2, 1, 0>), gq,
                         dim3(kWave), 0, st, lv, c, out);
    else if (variant == 62)  // the product's paths on a 240-cell slab (15 KB: the same LDS as the declared 232-cell one)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 240, false, 3, 3, 4, 0, 2>), gq, dim3(kWave),
                         0, st, lv, c, out);
    else if (variant == 63)  // round 6: the product + kFwdTrim (no loads for lanes past the window, no empty rounds)
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 240, false, 3, 3, 4, 0, 2, 1, 1, kFwdTrim>), gq,
                         dim3(kWave), 0, st, lv, c, out);
    else if (variant == 64)  // round 6: the product + the interleaved path's quad rotation
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 240, false, 3, 3, 4, 0, 2, 1, 1, kFwdIlvRot>), gq,
                         dim3(kWave), 0, st, lv, c, out);
    else if (variant == 66) {  // round 6: the product (trim + rotation) on spatially sorted RoI records
      FRH_REQUIRE(workspace && ws_bytes >= (size_t)num_rois * 32, "workspace too small");
      RoiCfg cs = c;
      cs.rec = reinterpret_cast<const int32_t*>(workspace);
      hipLaunchKernelGGL(roi_sort_kernel, dim3(1), dim3(kSortThreads), 0, st, lv, c,
                         reinterpret_cast<int32_t*>(workspace));
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 240, false, 3, 3, 4, 0, 2, 1, 1,
                                                    kFwdTrim | kFwdIlvRot | kFwdSorted>), gq, dim3(kWave), 0, st, lv,
                         cs, out);
    }
    else if (variant == 67) {  // the sort kernel alone (its cost in the variant-66 sum)
      FRH_REQUIRE(workspace && ws_bytes >= (size_t)num_rois * 32, "workspace too small");
      hipLaunchKernelGGL(roi_sort_kernel, dim3(1), dim3(kSortThreads), 0, st, lv, c,
                         reinterpret_cast<int32_t*>(workspace));
    }
    else if (variant == 65)  // round 6: trim + rotation
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, false, 240, false, 3, 3, 4, 0, 2, 1, 1,
                                                    kFwdTrim | kFwdIlvRot>), gq, dim3(kWave), 0, st, lv, c, out);
    else  // 45: hybrid (D = 4), 232-cell slab, stamped
      hipLaunchKernelGGL((roi_align_fwd_band_kernel<kCpolNT, true, 232, false, 3, 0, 4>), gq, dim3(kWave), 0, st,
                         lv, c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  if (variant >= 80 && variant <= 99) {  // round 6: channel-group kernel, one workgroup per (RoI, 64 channels)
    // 80: 4 waves, 144-cell slab (36 KB); 81: 8 waves, 144; 82: 4 waves, 192 cells; 83: 2 waves, 144;
    // 84: 8 waves, 192; 85: 4 waves, 160
    const FwdCaps fq = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
    FRH_REQUIRE(quad_ok(fq, lv, channels, pooled_h, pooled_w) && cg_ok(channels, pooled_h, pooled_w, 112),
                "the channel-group kernel does not take this shape");
    const int64_t tg = num_rois * (channels / kCgChan);
    const dim3 gg((unsigned)(8 * ((tg + 7) / 8)));
    if (variant == 80)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 144>), gg, dim3(4 * kWave), 0, st, lv, c, out);
    else if (variant == 81)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<8, 144>), gg, dim3(8 * kWave), 0, st, lv, c, out);
    else if (variant == 82)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 192>), gg, dim3(4 * kWave), 0, st, lv, c, out);
    else if (variant == 83)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<2, 144>), gg, dim3(2 * kWave), 0, st, lv, c, out);
    else if (variant == 84)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<8, 192>), gg, dim3(8 * kWave), 0, st, lv, c, out);
    else if (variant == 85)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 160>), gg, dim3(4 * kWave), 0, st, lv, c, out);
    else if (variant == 86)  // 120-cell slab (30 KB: 5 workgroups per CU by LDS), <= 96 VGPRs (5 waves per SIMD)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 120, kCpolNT, false, 5>), gg, dim3(4 * kWave), 0, st, lv, c, out);
    else if (variant == 87)  // 120-cell slab, registers as compiled (4 waves per SIMD)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 120>), gg, dim3(4 * kWave), 0, st, lv, c, out);
    else if (variant == 88)  // 112-cell slab (28 KB), 5 waves per SIMD
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 112, kCpolNT, false, 5>), gg, dim3(4 * kWave), 0, st, lv, c, out);
    else if (variant == 89)  // 120 cells, 5 waves per SIMD, one sample row's taps in flight
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 120, kCpolNT, false, 5, false>), gg, dim3(4 * kWave), 0, st, lv,
                         c, out);
    else if (variant == 90)  // 144 cells, one sample row's taps in flight
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 144, kCpolNT, false, 0, false>), gg, dim3(4 * kWave), 0, st, lv,
                         c, out);
    else if (variant == 92)  // as 90, RoI-major item order
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 144, kCpolNT, false, 0, false, 1>), gg, dim3(4 * kWave), 0, st,
                         lv, c, out);
    else if (variant == 93)  // as 90, default store policy
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 144, 0, false, 0, false>), gg, dim3(4 * kWave), 0, st, lv, c, out);
    else if (variant == 94)  // variant 89 (120 cells, 5 waves per SIMD, one sample row in flight), stamped (8 int64 per item after the output)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 120, kCpolNT, false, 5, false, 0, true>), gg, dim3(4 * kWave), 0,
                         st, lv, c, out);
    else if (variant == 95)  // 124 cells (31 KB: 5 workgroups per CU), 5 waves per SIMD, one sample row in flight
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<4, 124, kCpolNT, false, 5, false>), gg, dim3(4 * kWave), 0, st, lv,
                         c, out);
    else if (variant >= 96 && variant <= 99) {  // software-pipelined, kItems items per workgroup:
                                                 // 96 / 97 / 98: 2 / 3 / 4 items at 144 cells; 99: 2 at 116 cells
      const int ki = variant == 96 || variant == 99 ? 2 : variant == 97 ? 3 : 4;
      const int64_t per = (tg + 7) / 8, nwx = (per + ki - 1) / ki;
      const dim3 gp((unsigned)(8 * nwx));
      if (variant == 96)
        hipLaunchKernelGGL((roi_align_fwd_cgp_kernel<4, 144, 2>), gp, dim3(4 * kWave), 0, st, lv, c, out);
      else if (variant == 97)
        hipLaunchKernelGGL((roi_align_fwd_cgp_kernel<4, 144, 3>), gp, dim3(4 * kWave), 0, st, lv, c, out);
      else if (variant == 98)
        hipLaunchKernelGGL((roi_align_fwd_cgp_kernel<4, 144, 4>), gp, dim3(4 * kWave), 0, st, lv, c, out);
      else
        hipLaunchKernelGGL((roi_align_fwd_cgp_kernel<4, 116, 2, kCpolNT, false, 5>), gp, dim3(4 * kWave), 0, st, lv, c,
                           out);
    }
    else  // 91: 8 waves, 144 cells, one sample row's taps in flight, 4 waves per SIMD (2 workgroups per CU)
      hipLaunchKernelGGL((roi_align_fwd_cg_kernel<8, 120, kCpolNT, false, 5, false>), gg, dim3(8 * kWave), 0, st, lv,
                         c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  if (variant == 26 || variant == 27) {  // quad kernel, chunk-pair-major item order (27: + stamps)
    const FwdCaps fq = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
    FRH_REQUIRE(quad_ok(fq, lv, channels, pooled_h, pooled_w), "the quad kernel does not take this shape");
    const int64_t tq = num_rois * ((channels + 4 * kQuadWave - 1) / (4 * kQuadWave));
    const dim3 gq((unsigned)(8 * ((tq + 7) / 8)));
    if (variant == 26)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3, kQuadWave, 0, false, kQuadSlab, 1>), gq,
                         dim3(kWave), 0, st, lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, true, 3, kQuadWave, 0, false, kQuadSlab, 1>), gq,
                         dim3(kWave), 0, st, lv, c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  if (variant == 25) {  // quad kernel with a 16-KB slab (10 waves per CU by LDS; D = 4 up to 256 cells)
    const FwdCaps fq = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
    FRH_REQUIRE(quad_ok(fq, lv, channels, pooled_h, pooled_w, QuadLayout<1, 4096>::kCells),
                "the quad kernel does not take this shape");
    const int64_t tq = num_rois * ((channels + 4 * kQuadWave - 1) / (4 * kQuadWave));
    const dim3 gq((unsigned)(8 * ((tq + 7) / 8)));
    hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3, kQuadWave, 0, false, 4096>), gq, dim3(kWave), 0,
                       st, lv, c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  if (variant == 19 || variant == 20) {  // quad kernel, RoI setup shared by a 4-wave workgroup (20: LDS-staged stores)
    const FwdCaps fq = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
    FRH_REQUIRE(quad_ok(fq, lv, channels, pooled_h, pooled_w), "the quad kernel does not take this shape");
    const int64_t tq = num_rois * ((channels + 16 * kQuadWave - 1) / (16 * kQuadWave));
    const dim3 gq((unsigned)(8 * ((tq + 7) / 8)));
    if (variant == 19)
      hipLaunchKernelGGL((roi_align_fwd_quad4_kernel<kCpolNT, 0>), gq, dim3(4 * kWave), 0, st, lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_quad4_kernel<kCpolNT, 1>), gq, dim3(4 * kWave), 0, st, lv, c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  if (variant >= 8 && variant <= 18) {  // channels-last quad kernel (9: stamped; 10: 3 waves/SIMD; 11: 5;
                                        // 12 / 13 / 14: 32 / 64 / 128 channels per item; 15: 32 stamped)
    const FwdCaps fq = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
    FRH_REQUIRE(quad_ok(fq, lv, channels, pooled_h, pooled_w), "the quad kernel does not take this shape");
    const int qw = variant == 12 || variant == 15 ? 8 : variant == 13 ? 16 : variant == 14 ? 32 : kQuadWave;
    const int64_t tq = num_rois * ((channels + 4 * qw - 1) / (4 * qw));
    const dim3 gq((unsigned)(8 * ((tq + 7) / 8)));
    if (variant == 12)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3, 8>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 13)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3, 16>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 14)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3, 32>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 15)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, true, 3, 8>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 16)  // LDS-staged 16-B output stores
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3, 4, 1>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 17)  // no output stores (diagnostic: the staging + evaluation alone)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3, 4, 2>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 18)  // LDS-staged 16-B stores, default cache policy
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<0, false, 3, 4, 1>), gq, dim3(kWave), 0, st, lv, c, out);
    else
    if (variant == 8)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 9)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, true>), gq, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 10)
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 3>), gq, dim3(kWave), 0, st, lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_quad_kernel<kCpolNT, false, 5>), gq, dim3(kWave), 0, st, lv, c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  if (variant >= 2 && variant <= 7) {  // channels-last kernel: slab cells / outputs in VGPRs or in LDS
    FRH_REQUIRE(nhwc_ok(lv, channels, pooled_h, pooled_w, sampling_ratio), "the nhwc kernel does not take this shape");
    const int64_t tn = num_rois * (channels / kNhwcGroup);
    const dim3 gn((unsigned)(8 * ((tn + 7) / 8)));
    if (variant == 2)
      hipLaunchKernelGGL((roi_align_fwd_nhwc_kernel<7, 7, 56, kCpolNT, true>), gn, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 3)
      hipLaunchKernelGGL((roi_align_fwd_nhwc_kernel<7, 7, 64, kCpolNT, true>), gn, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 4)
      hipLaunchKernelGGL((roi_align_fwd_nhwc_kernel<7, 7, 96, kCpolNT, true>), gn, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 5)
      hipLaunchKernelGGL((roi_align_fwd_nhwc_kernel<7, 7, 56, kCpolNT, false>), gn, dim3(kWave), 0, st, lv, c, out);
    else if (variant == 6)
      hipLaunchKernelGGL((roi_align_fwd_nhwc_kernel<7, 7, 56, kCpolNT, true, true>), gn, dim3(kWave), 0, st, lv, c, out);
    else
      hipLaunchKernelGGL((roi_align_fwd_nhwc_kernel<7, 7, 128, kCpolNT, true>), gn, dim3(kWave), 0, st, lv, c, out);
    return check_launch("frh_roi_align_fwd_variant");
  }
  const FwdCaps f = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
  FRH_REQUIRE(pair_ok(f, channels, pooled_h, pooled_w), "the pair kernel does not take this shape");
  const int64_t total = num_rois * ((channels + kPairChunk - 1) / kPairChunk);
  FRH_REQUIRE(total <= (int64_t)0x7fffffff - 7, "too many RoIs");
  const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
  if (variant == 0)
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kCpolNT, false>), g1, dim3(kWave), 0, st, lv, c, out);
  else if (variant == 1)
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kCpolNT, true>), g1, dim3(kWave), 0, st, lv, c, out);
  else
    FRH_REQUIRE(false, "roi_align variant %d unknown", variant);
  return check_launch("frh_roi_align_fwd_variant");
}

// Round-6 backward A/B (channels-last gradients, sampling 2, 7 x 7 bins): 0 = the product's
// roi_align_bwd_nhwc_kernel (float atomics), 1 = roi_align_bwd_nhwc_reg_kernel (grad_out in
// registers, float atomics), 2 / 3 = the same two in fixed point (absmax pass + conversion, as
// frh_roi_align_bwd_fixed; accs zeroed by the caller).  grads zeroed by the caller for 0 / 1.
extern "C" int32_t frh_roi_align_bwd_variant(int32_t variant, int32_t num_levels, float* const* grad_feats,
                                             int64_t* const* acc_feats, const int32_t* feat_hw, const int64_t* strides,
                                             const float* scales, int32_t batch, int32_t channels, const float* rois,
                                             const int64_t* roi_levels, int64_t num_rois, const float* grad_out,
                                             uint32_t* scale_word, void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, 7, 7, rois);
  if (r) return r;
  const bool fixed = variant == 2 || variant == 3 || variant == 5 || variant == 12;
  RoiLevels lv;
  r = make_levels(num_levels, nullptr, fixed ? reinterpret_cast<float* const*>(acc_feats) : grad_feats, feat_hw,
                  strides, scales, &lv);
  if (r) return r;
  lv.B = batch;
  for (int l = 0; l < lv.L; ++l) FRH_REQUIRE(lv.sc[l] == 1, "channels-last gradients only");
  hipStream_t st = as_stream(stream);
  int hb = 0;
  while (hb < 62 && (int64_t(1) << hb) < num_rois * 49) ++hb;
  RoiCfg c{rois, roi_levels, num_rois, channels, 7, 7, 2, 0, nullptr, scale_word, hb};
  const dim3 grid((unsigned)num_rois, (unsigned)((channels + kWave - 1) / kWave));
  if (fixed) {
    FRH_HIP(hipMemsetAsync(scale_word, 0, 4, st));
    const int64_t ng = num_rois * channels * 49;
    hipLaunchKernelGGL(roi_bwd_absmax_kernel, dim3((unsigned)std::min<int64_t>((ng / 4 + 255) / 256 + 1, kAbsmaxBlocks)),
                       dim3(kAbsmaxThreads), 0, st, grad_out, ng, scale_word);
  }
  if (variant == 0)
    hipLaunchKernelGGL(roi_align_bwd_nhwc_kernel<false>, grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 1)
    hipLaunchKernelGGL(roi_align_bwd_nhwc_reg_kernel<false>, grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 2)
    hipLaunchKernelGGL(roi_align_bwd_nhwc_kernel<true>, grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 3)
    hipLaunchKernelGGL(roi_align_bwd_nhwc_reg_kernel<true>, grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 4)  // round 6: tap lists read by v_readlane, row sums in registers
    hipLaunchKernelGGL(roi_align_bwd_nhwc2_kernel<false>, grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 5)
    hipLaunchKernelGGL(roi_align_bwd_nhwc2_kernel<true>, grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 6)  // diagnostic: variant 4 with plain stores instead of atomics (wrong sums)
    hipLaunchKernelGGL((roi_align_bwd_nhwc2_kernel<false, true>), grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 9 || variant == 10 || variant == 11 || variant == 12) {  // product kernel, kNW waves per RoI
    const dim3 gw((unsigned)num_rois, (unsigned)((channels + kWave - 1) / kWave));
    if (variant == 9)
      hipLaunchKernelGGL((roi_align_bwd_nhwc_kernel<false, 2>), gw, dim3(2 * kWave), 0, st, lv, c, grad_out);
    else if (variant == 10)
      hipLaunchKernelGGL((roi_align_bwd_nhwc_kernel<false, 4>), gw, dim3(4 * kWave), 0, st, lv, c, grad_out);
    else if (variant == 11)
      hipLaunchKernelGGL((roi_align_bwd_nhwc_kernel<false, 8>), gw, dim3(8 * kWave), 0, st, lv, c, grad_out);
    else
      hipLaunchKernelGGL((roi_align_bwd_nhwc_kernel<true, 4>), gw, dim3(4 * kWave), 0, st, lv, c, grad_out);
  }
  else if (variant == 7)  // diagnostic: no column loop (row sums stored)
    hipLaunchKernelGGL((roi_align_bwd_nhwc2_kernel<false, true, 1>), grid, dim3(kWave), 0, st, lv, c, grad_out);
  else if (variant == 8)  // diagnostic: setup only (grad_out staging, tap entries, ranks)
    hipLaunchKernelGGL((roi_align_bwd_nhwc2_kernel<false, true, 2>), grid, dim3(kWave), 0, st, lv, c, grad_out);
  else
    FRH_REQUIRE(false, "backward variant %d unknown", variant);
  if (fixed) {
    for (int l = 0; l < lv.L; ++l) {
      const int64_t n = (int64_t)batch * channels * lv.h[l] * lv.w[l];
      hipLaunchKernelGGL(roi_bwd_fixed_to_f32_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 4096)),
                         dim3(256), 0, st, reinterpret_cast<const long long*>(acc_feats[l]), grad_feats[l], n,
                         scale_word, hb);
    }
  }
  return check_launch("frh_roi_align_bwd_variant");
}

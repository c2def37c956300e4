// a13/a14: FPN level mapping + RoIAlign forward/backward over all levels and
// images.
// Reference: lib/region.py:243-306 (BasicRoIExtractor: map_rois_to_levels,
// per-level torchvision RoIAlign(output_size, 1/stride, sampling_ratio=2)),
// torchvision legacy (aligned=False) RoIAlign semantics.
//
// Forward (all bit-identical: -ffp-contract=off, reference op order; kernels in
// roi_kernels.h):
//  * roi_align_fwd_cg_kernel -- channels-last features with C % 64 == 0 (the product trunk's
//    FPN levels): one 4-wave workgroup per (RoI, 64 channels), the tap window staged once as
//    [cell][64 channels] (256-B requests), lane = (bin, channel quad): bank-conflict-free
//    ds_read_b128 taps; windows above the 30-KB slab in bands of bin rows.
//  * roi_align_fwd_band_kernel -- channels-last features (unit channel stride, C % 4
//    == 0, sampling 2, 7x7 bins and smaller): small windows as the quad kernel (16-B
//    LDS-DMA staging, lane = cell, one ds_read_b128 per tap for 4 channels), larger ones
//    in row bands of [cell][16 channels] with one 64-B request per cell (roi_kernels.h).
//  * roi_align_fwd_quad_kernel -- the quad path alone, for channels-last shapes the band
//    kernel does not take.
//  * roi_align_fwd_pair_kernel -- the default (sampling 2, up to 8x8 bins, even C):
//    one wave per (RoI, 16 channels); the RoI's tap window staged by LDS-DMA with
//    channel pairs interleaved into one slab buffer per wave, packed-f32 bilinear sums.
//  * roi_align_fwd_lds_kernel -- odd channel counts: per-(RoI, 64 channels)
//    workgroup, windows <= 256 floats staged in LDS, larger ones gathered.
//  * roi_align_fwd_kernel -- direct gather, any pooled size / sampling ratio.
// Backward: roi_align_bwd_sep_kernel (sampling 2, up to 8x8 bins: separable
// row-run sums, one atomic per run) / roi_align_bwd_lds_kernel (up to 64 bins) /
// roi_align_bwd_kernel (per-tap atomics, any shape).
// Feature tensors are addressed through explicit (batch, channel, y, x) element
// strides: NCHW, channels_last and strided views (FPN P6 = P5[..., ::2, ::2]) all
// run.  The forward laboratory (stamped builds, candidate kernels) is the tools-only
// library (tools/csrc/roi_lab.hip).
#include <hip/hip_ext.h>
#include "roi_kernels.h"

namespace frh {

// The band kernel's slab: 240 cells x 16 channels = 15 KB (10 waves per CU by LDS, 3 per
// SIMD by registers): 8-row bands of the widest (29-column) windows, i.e. two bin rows of a
// tap-list window per band; whole 1-KB LDS-DMA rounds (2 x 240 cells x 32 B of the interleaved
// path and 15 rounds of 16 band cells both fill exactly 15 KB).  Windows of <= 192 cells take
// the quad path (kHybrid = 4), <= 480 cells the two interleaved stages, larger ones the bands.
// The bands' results are stored after the last band (kRot 3: whole channel rows per store).
// Measured (tools/bench_roi_sets.py, MI355X, µs per launch, bench / VOC / train-step RoIs):
// this form 40.9 / 76.2 / 65.2 (stores per band: 40.9-42.9 / 77.2-79.0 / 67.2-69.3); bands
// only 44.1-47.3 / 76-78 / 66-70; quad kernel (13 KB slab, pair order) 37.7-39.1 / 103-106 /
// 96-98; round 4's 37.1-39.5 / 142 / 150.
constexpr int kBandCells = 240;  // 15 KB: whole 1-KB DMA rounds, 10 workgroups per CU by LDS
// The channel-group kernel's slab (round 6): 120 cells x 64 channels = 30 KB + the sample tables,
// 5 workgroups of 4 waves per CU (by LDS, and by its 82 VGPRs at waves_per_eu 5: one sample row's
// 8 tap reads in flight at a time).  Measured (tools/bench_roi_sets.py, lab variants 80-99, µs per
// launch, bench / VOC / train RoIs, bit-identical): this form (variant 89) 32.5-34.3 / 56.6-58.5 /
// 50.4-52.5; 144 cells at 4 per CU with both rows' reads in flight (variant 80, the first product
// form) 33.5-35.5 / 58.9-61.5 / 53.3-55.2; the round-5 band kernel 38.7-42.1 / 67.4-72.7 /
// 58.2-61.4.  120 cells hold the 4 tap-list rows of a 28-column window (cg_ok: 7 x 7 bins at most).
constexpr int kCgCells = 120;
static_assert(2 * kBandCells * 32 <= kBandCells * 64 && (kBandCells + 15) / 16 * 1024 <= kBandCells * 64,
              "the interleaved stages and the band DMA rounds must fit the slab");

// region.py:256-264: floor(log2(sqrt(area) / finest + 1e-6)) clamped to [0, L-1]
__device__ __forceinline__ int64_t roi_level_of(float x1, float y1, float x2, float y2, float finest, int L) {
  float area = ((x2 - x1) + 1.0f) * ((y2 - y1) + 1.0f);
  float s = sqrtf(area);
  float v = s / finest + 1e-6f;
  // correctly rounded f32 log2, then floor (region.py:262); clamp to [0, L-1]
  float lg = (float)log2((double)v);
  float fl = floorf(lg);
  float hi = (float)(L - 1);
  fl = !(fl >= 0.0f) ? 0.0f : (fl > hi ? hi : fl);  // NaN (NaN coordinates): level 0
  return (int64_t)fl;
}

__global__ void roi_level_kernel(const float* rois, int64_t K, float finest, int L, int64_t* levels) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const float* r = rois + k * 5;
  levels[k] = roi_level_of(r[1], r[2], r[3], r[4], finest, L);
}

constexpr int kRowSegs = 64;

struct RowsArgs {
  const float* boxes;
  int64_t ld, seg_stride;
  int32_t S, flat, L;
  float finest;
  int64_t K;
  float* rois;
  int64_t* levels;
  int64_t offs[kRowSegs + 1];
  const int32_t* dev_counts;  // nullable: per-image row counts on the device (flat rows, capacity K)
};

// RoI rows [K, 5] = (image, x1, y1, x2, y2) of the images' boxes, concatenated in image
// order, and (L > 1) their FPN levels: the reference's batch-index column
// (_attach_idx_to_rois_, region.py:266-269) and map_rois_to_levels (:256-264) in one pass.
__global__ void roi_rows_kernel(RowsArgs a) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= a.K) return;
  int b = 0;
  if (a.dev_counts) {  // rows past the images' total are padding rows: image 0
    int64_t end = a.dev_counts[0];
    while (b + 1 < a.S && k >= end) end += a.dev_counts[++b];
    if (k >= end) b = 0;
  } else {
    while (b + 1 < a.S && k >= a.offs[b + 1]) ++b;
  }
  const int64_t col = a.flat ? k : k - a.offs[b];
  const float* p = a.boxes + (int64_t)b * a.seg_stride + col;
  const float x1 = p[0], y1 = p[a.ld], x2 = p[2 * a.ld], y2 = p[3 * a.ld];
  float* r = a.rois + k * 5;
  r[0] = (float)b;
  r[1] = x1;
  r[2] = y1;
  r[3] = x2;
  r[4] = y2;
  if (a.levels) a.levels[k] = roi_level_of(x1, y1, x2, y2, a.finest, a.L);
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

extern "C" int32_t frh_roi_rows(int32_t num_segs, const float* boxes, int64_t box_ld, int64_t box_seg_stride,
                                int32_t flat, const int64_t* seg_offsets, float finest_scale, int32_t num_levels,
                                float* rois, int64_t* levels, void* stream) {
  FRH_REQUIRE(num_segs >= 1 && num_segs <= kRowSegs, "num_segs must be in [1, %d]", kRowSegs);
  FRH_REQUIRE(seg_offsets && num_levels >= 1, "bad arguments");
  RowsArgs a{boxes, box_ld, box_seg_stride, num_segs, flat ? 1 : 0, num_levels, finest_scale, 0, rois,
             num_levels > 1 ? levels : nullptr, {}, nullptr};
  for (int b = 0; b <= num_segs; ++b) {
    a.offs[b] = seg_offsets[b];
    FRH_REQUIRE(b == 0 ? a.offs[0] == 0 : a.offs[b] >= a.offs[b - 1], "seg_offsets must start at 0 and not decrease");
  }
  a.K = a.offs[num_segs];
  if (a.K == 0) return FRH_OK;
  FRH_REQUIRE(boxes && rois && (num_levels == 1 || levels), "null pointer argument");
  hipLaunchKernelGGL(roi_rows_kernel, dim3((unsigned)((a.K + 255) / 256)), dim3(256), 0, as_stream(stream), a);
  return check_launch("frh_roi_rows");
}

extern "C" int32_t frh_roi_rows_dev(int32_t num_segs, const float* boxes, int64_t box_ld, int64_t num_rows,
                                    const int32_t* seg_counts, float finest_scale, int32_t num_levels, float* rois,
                                    int64_t* levels, void* stream) {
  FRH_REQUIRE(num_segs >= 1 && num_segs <= kRowSegs, "num_segs must be in [1, %d]", kRowSegs);
  FRH_REQUIRE(seg_counts && num_levels >= 1 && num_rows >= 0, "bad arguments");
  if (num_rows == 0) return FRH_OK;
  FRH_REQUIRE(boxes && rois && (num_levels == 1 || levels), "null pointer argument");
  RowsArgs a{boxes, box_ld, 0, num_segs, 1, num_levels, finest_scale, num_rows, rois,
             num_levels > 1 ? levels : nullptr, {}, seg_counts};
  hipLaunchKernelGGL(roi_rows_kernel, dim3((unsigned)((num_rows + 255) / 256)), dim3(256), 0, as_stream(stream), a);
  return check_launch("frh_roi_rows_dev");
}

static int32_t roi_fwd(int32_t num_levels, const float* const* feats, const int32_t* feat_hw, const int64_t* strides,
                       const float* scales, int32_t batch, int32_t channels, const float* rois,
                       const int64_t* roi_levels, int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                       int32_t sampling_ratio, int32_t aligned, float* out, hipStream_t st, hipEvent_t e0,
                       hipEvent_t e1, unsigned long long* span = nullptr) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  FRH_REQUIRE((feats && out) || num_rois == 0, "null pointer argument");
  RoiLevels lv;
  r = make_levels(num_levels, feats, nullptr, feat_hw, strides, scales, &lv);
  if (r) return r;
  lv.B = batch;
  if (num_rois == 0) return FRH_OK;
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned, span};
  const FwdCaps f = fwd_caps(lv, channels, pooled_h, pooled_w, sampling_ratio);
  // e0 / e1 (measurement entry): the kernel's own start / end timestamps (hipExtLaunchKernel
  // binds them to the dispatch; no extra packets in the stream)
  auto go = [&](auto kern, dim3 grid, dim3 block) {
    if (e0 || e1)
      hipExtLaunchKernelGGL(kern, grid, block, 0, st, e0, e1, 0, lv, c, out);
    else
      hipLaunchKernelGGL(kern, grid, block, 0, st, lv, c, out);
  };
  if (quad_ok(f, lv, channels, pooled_h, pooled_w) && cg_ok(channels, pooled_h, pooled_w, kCgCells)) {
    // channels-last features, C % 64 == 0 (the FPN's NHWC levels, round 6): one 4-wave workgroup
    // per (RoI, 64 channels), the window staged once as [cell][64 channels], conflict-free taps
    const int64_t total = num_rois * (channels / kCgChan);
    FRH_REQUIRE(total <= (int64_t)0x7fffffff - 7, "too many RoIs");
    const dim3 grid((unsigned)(8 * ((total + 7) / 8)));
    if (span)
      go(roi_align_fwd_cg_kernel<4, kCgCells, kCpolNT, true, 5, false>, grid, dim3(4 * kWave));
    else
      go(roi_align_fwd_cg_kernel<4, kCgCells, kCpolNT, false, 5, false>, grid, dim3(4 * kWave));
  } else if (quad_ok(f, lv, channels, pooled_h, pooled_w) && band_fits(pooled_h, pooled_w, kBandCells)) {
    // channels-last features (the FPN's NHWC levels): one wave per (RoI, 16 channels); tap
    // windows of <= 192 cells staged whole, 4 quads at a time ([quad][cell]); <= 480 cells
    // whole in two stages of [cell][2 quads] (32 B per cell and request); larger in row bands
    // of [cell][16 channels], 64 B per cell and request
    const int64_t total = num_rois * ((channels + kQuadChunk - 1) / kQuadChunk);
    FRH_REQUIRE(total <= (int64_t)0x7fffffff - 7, "too many RoIs");
    const dim3 grid((unsigned)(8 * ((total + 7) / 8)));
    // kFwdTrim | kFwdIlvRot (round 6): no loads for lanes past the window and no empty DMA rounds;
    // the interleaved path's two lanes of a cell read different quads at each step
    constexpr int kOpt = kFwdTrim | kFwdIlvRot;
    if (span)
      go(roi_align_fwd_band_kernel<kCpolNT, false, kBandCells, true, 3, 3, 4, 0, 2, 1, 1, kOpt>, grid, dim3(kWave));
    else
      go(roi_align_fwd_band_kernel<kCpolNT, false, kBandCells, false, 3, 3, 4, 0, 2, 1, 1, kOpt>, grid, dim3(kWave));
  } else if (quad_ok(f, lv, channels, pooled_h, pooled_w)) {
    // channels-last, shapes the band kernel does not take: one quad per 16-B DMA lane
    const int64_t total = num_rois * ((channels + kQuadChunk - 1) / kQuadChunk);
    FRH_REQUIRE(total <= (int64_t)0x7fffffff - 7, "too many RoIs");
    const dim3 grid((unsigned)(8 * ((total + 7) / 8)));
    go(roi_align_fwd_quad_kernel<kCpolNT, false, 3>, grid, dim3(kWave));
  } else if (pair_ok(f, channels, pooled_h, pooled_w)) {
    // chunk-major XCD order, nt output stores, one 6.5 KB slab per wave, lean tap state
    const int64_t total = num_rois * ((channels + kPairChunk - 1) / kPairChunk);
    FRH_REQUIRE(total <= (int64_t)0x7fffffff - 7, "too many RoIs");
    const dim3 grid((unsigned)(8 * ((total + 7) / 8)));
    if (span)
      go(roi_align_fwd_pair_kernel<kCpolNT, false, true>, grid, dim3(kWave));
    else
      go(roi_align_fwd_pair_kernel<kCpolNT, false>, grid, dim3(kWave));
  } else if (f.lds) {
    go(roi_align_fwd_lds_kernel<256>, dim3((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk)),
       dim3(kRoiThreads));
  } else {
    go(roi_align_fwd_kernel, dim3((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk)),
       dim3(kRoiThreads));
  }
  return check_launch("frh_roi_align_fwd");
}

extern "C" int32_t frh_roi_align_fwd_strided(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                                             const int64_t* strides, const float* scales, int32_t batch,
                                             int32_t channels, const float* rois, const int64_t* roi_levels,
                                             int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                             int32_t sampling_ratio, int32_t aligned, float* out, void* stream) {
  return roi_fwd(num_levels, feats, feat_hw, strides, scales, batch, channels, rois, roi_levels, num_rois, pooled_h,
                 pooled_w, sampling_ratio, aligned, out, as_stream(stream), nullptr, nullptr);
}

extern "C" int32_t frh_roi_align_fwd_strided_timed(int32_t num_levels, const float* const* feats,
                                                   const int32_t* feat_hw, const int64_t* strides,
                                                   const float* scales, int32_t batch, int32_t channels,
                                                   const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                                   int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio,
                                                   int32_t aligned, float* out, void* start_event, void* stop_event,
                                                   uint64_t* span, void* stream) {
  FRH_REQUIRE(start_event && stop_event, "null event");
  return roi_fwd(num_levels, feats, feat_hw, strides, scales, batch, channels, rois, roi_levels, num_rois, pooled_h,
                 pooled_w, sampling_ratio, aligned, out, as_stream(stream), static_cast<hipEvent_t>(start_event),
                 static_cast<hipEvent_t>(stop_event), reinterpret_cast<unsigned long long*>(span));
}

// The channels-last backward: 4 waves per (RoI, 64 channels), the RoI's tap rows split between
// them (round 6; tools/bench_roi_bwd.py variants 9-12, µs per call incl. the clear, bench / voc /
// train RoIs: one wave 236 / 500 / 400, 2 waves 177 / 438 / 365, 4 waves 153 / 401 / 338, 8 waves
// 148 / 408 / 337; fixed point 390 -> 321 / 799 -> 721 / 702 -> 637)
constexpr int kBwdWaves = 4;

// channels-last gradient levels (unit channel stride), sampling 2, up to 8 x 8 bins: lane = channel
static bool bwd_nhwc_ok(const RoiLevels& lv, int32_t sampling_ratio, int32_t ph, int32_t pw) {
  if (sampling_ratio != 2 || ph > 8 || pw > 8 || 4 * ph > kSepEnt || 4 * pw > kSepEnt) return false;
  for (int l = 0; l < lv.L; ++l)
    if (lv.sc[l] != 1) return false;
  return true;
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
  lv.B = batch;
  if (num_rois == 0) return FRH_OK;
  FRH_REQUIRE(grad_feats && grad_out, "null pointer argument");
  RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned};
  dim3 grid((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk));
  if (bwd_nhwc_ok(lv, sampling_ratio, pooled_h, pooled_w))
    hipLaunchKernelGGL((roi_align_bwd_nhwc_kernel<false, kBwdWaves>),
                       dim3((unsigned)num_rois, (unsigned)((channels + kWave - 1) / kWave)), dim3(kBwdWaves * kWave), 0,
                       as_stream(stream), lv, c, grad_out);
  else if (sampling_ratio == 2 && 4 * pooled_h <= kSepEnt && 4 * pooled_w <= kSepEnt)
    hipLaunchKernelGGL(roi_align_bwd_sep_kernel<false>, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c,
                       grad_out);
  else if (sampling_ratio == 2 && pooled_h * pooled_w <= 64)
    hipLaunchKernelGGL(roi_align_bwd_lds_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, grad_out);
  else
    hipLaunchKernelGGL(roi_align_bwd_kernel, grid, dim3(kRoiThreads), 0, as_stream(stream), lv, c, grad_out);
  return check_launch("frh_roi_align_bwd");
}

extern "C" int32_t frh_roi_align_bwd_fixed(int32_t num_levels, float* const* grad_feats, int64_t* const* acc_feats,
                                           const int32_t* feat_hw, const int64_t* strides, const float* scales,
                                           int32_t batch, int32_t channels, const float* rois,
                                           const int64_t* roi_levels, int64_t num_rois, int32_t pooled_h,
                                           int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                           const float* grad_out, uint32_t* scale_word, void* stream) {
  int32_t r = roi_common_checks(batch, channels, num_rois, pooled_h, pooled_w, rois);
  if (r) return r;
  FRH_REQUIRE(grad_feats && acc_feats && scale_word, "null pointer argument");
  FRH_REQUIRE(sampling_ratio == 2 && 4 * pooled_h <= kSepEnt && 4 * pooled_w <= kSepEnt,
              "the deterministic backward takes sampling_ratio 2 and up to %d x %d bins", kSepEnt / 4, kSepEnt / 4);
  RoiLevels lv;
  // the kernel adds into the accumulators through lv.grad (same element strides)
  r = make_levels(num_levels, nullptr, reinterpret_cast<float* const*>(acc_feats), feat_hw, strides, scales, &lv);
  if (r) return r;
  lv.B = batch;
  hipStream_t st = as_stream(stream);
  int64_t numel[FRH_MAX_LEVELS];
  for (int l = 0; l < num_levels; ++l) {
    FRH_REQUIRE(grad_feats[l] && acc_feats[l], "null level buffer");
    const int64_t n = (int64_t)batch * channels * lv.h[l] * lv.w[l];
    const int64_t last = (int64_t)(batch - 1) * lv.sb[l] + (int64_t)(channels - 1) * lv.sc[l] +
                         (int64_t)(lv.h[l] - 1) * lv.sy[l] + (int64_t)(lv.w[l] - 1) * lv.sx[l];
    FRH_REQUIRE(lv.sb[l] > 0 && lv.sc[l] > 0 && lv.sy[l] > 0 && lv.sx[l] > 0 && last == n - 1,
                "level %d: the deterministic backward needs dense gradient buffers", l);
    numel[l] = n;
  }
  // the call's fixed-point unit: max|grad_out| (one streaming pass), headroom for K * bins
  int hb = 0;
  while (hb < 62 && (int64_t(1) << hb) < num_rois * pooled_h * pooled_w) ++hb;
  FRH_REQUIRE(hb <= 40, "too many RoIs x bins for the fixed-point backward");
  if (hipMemsetAsync(scale_word, 0, sizeof(uint32_t), st) != hipSuccess) return check_launch("frh_roi_align_bwd_fixed");
  if (num_rois > 0) {
    FRH_REQUIRE(grad_out, "null grad_out");
    const int64_t ng = num_rois * channels * pooled_h * pooled_w;
    const int64_t mb = std::min<int64_t>((ng / 4 + kAbsmaxThreads - 1) / kAbsmaxThreads + 1, kAbsmaxBlocks);
    hipLaunchKernelGGL(roi_bwd_absmax_kernel, dim3((unsigned)mb), dim3(kAbsmaxThreads), 0, st, grad_out, ng,
                       scale_word);
    RoiCfg c{rois, roi_levels, num_rois, channels, pooled_h, pooled_w, sampling_ratio, aligned, nullptr, scale_word, hb};
    if (bwd_nhwc_ok(lv, sampling_ratio, pooled_h, pooled_w)) {
      hipLaunchKernelGGL((roi_align_bwd_nhwc_kernel<true, kBwdWaves>),
                         dim3((unsigned)num_rois, (unsigned)((channels + kWave - 1) / kWave)), dim3(kBwdWaves * kWave),
                         0, st, lv, c, grad_out);
    } else {
      dim3 grid((unsigned)num_rois, (unsigned)((channels + kRoiChanChunk - 1) / kRoiChanChunk));
      hipLaunchKernelGGL(roi_align_bwd_sep_kernel<true>, grid, dim3(kRoiThreads), 0, st, lv, c, grad_out);
    }
  }
  for (int l = 0; l < num_levels; ++l) {
    const int64_t blocks = std::min<int64_t>((numel[l] + 255) / 256, 4096);
    hipLaunchKernelGGL(roi_bwd_fixed_to_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                       reinterpret_cast<const long long*>(acc_feats[l]), grad_feats[l], numel[l], scale_word, hb);
  }
  return check_launch("frh_roi_align_bwd_fixed");
}

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

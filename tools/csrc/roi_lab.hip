// TOOLS-ONLY RoIAlign forward laboratory (see frcnn_tools.h).  Variant 0 is the
// product default instantiation, so A/B runs compare against exactly what ships.
#include "frcnn_tools.h"
#include "roi_kernels.h"

using namespace frh;

namespace {

// The product pair kernel with kWPG independent waves per workgroup (one item each): a CU
// admits at most 16 workgroups, so single-wave workgroups cap residency at 16 waves per CU
// whatever the register count allows.  XCD x (= workgroup id % 8) walks the x-th eighth of
// the chunk-major item list, kWPG consecutive items per workgroup.
template <int kWPG, int kMinW, bool kStamp, bool kDynR = false, bool kWideSt = false>
__global__ void __launch_bounds__(kWave * kWPG, kMinW) pair_mw_kernel(RoiLevels lv, RoiCfg c, float* __restrict__ out) {
  const int64_t t_start = kStamp ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  constexpr int kOut = kWideSt ? 2 * kPairWave * kWave + kWave : 0;  // [channel][bin] output staging + idle lanes
  __shared__ __attribute__((aligned(16))) float slab[kWPG][kPairHalf + kOut];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)slab[wave]);
  const uint32_t G = (uint32_t)(c.C + kPairChunk - 1) / (uint32_t)kPairChunk, K32 = (uint32_t)c.K;
  const uint32_t total = K32 * G, per = (total + 7u) / 8u;
  const uint32_t w = (blockIdx.x & 7u) * per + (blockIdx.x >> 3) * (uint32_t)kWPG + (uint32_t)wave;
  const uint32_t wend = min((blockIdx.x & 7u) * per + per, total);
  if (w >= wend) return;
  const int ch0 = (int)(w / K32);
  const int64_t k0 = (int64_t)(w - (uint32_t)ch0 * K32);
  pair_item<kPairWave, kPairHalf, kCpolNT, 0, kStamp, true, true, true, kDynR, kWideSt>(
      lv, c, out, k0, ch0, w, roi_fetch(c, k0), sbase, t_start, threadIdx.x & (kWave - 1), sbase + 4u * kPairHalf);
}

template <int kWPG, int kMinW = 1, bool kStamp = false, bool kDynR = false, bool kWideSt = false>
void launch_mw(const RoiLevels& lv, const RoiCfg& c, float* out, int64_t total, hipStream_t st) {
  const int64_t per = (total + 7) / 8;
  const int64_t wgs = 8 * ((per + kWPG - 1) / kWPG);
  hipLaunchKernelGGL((pair_mw_kernel<kWPG, kMinW, kStamp, kDynR, kWideSt>), dim3((unsigned)wgs), dim3(kWave * kWPG), 0,
                     st, lv, c, out);
}

}  // namespace

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
  const bool pok = pair_ok(f, channels, pooled_h, pooled_w);
  const int64_t total = num_rois * ((channels + kPairChunk - 1) / kPairChunk);
  FRH_REQUIRE(total <= (int64_t)0x7fffffff - 7, "too many RoIs");
  const dim3 g1((unsigned)(8 * ((total + 7) / 8)));
  if (variant == 0) {
    FRH_REQUIRE(pok, "the pair kernel does not take this shape");
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1, kCpolNT, 0, false, true, 1, true, 1, true>),
                       g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant == 1) {
    FRH_REQUIRE(pok, "the pair kernel does not take this shape");
    hipLaunchKernelGGL((roi_align_fwd_pair_kernel<kPairWave, kPairHalf, 1, kCpolNT, 0, true, true, 1, true, 1, true>),
                       g1, dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else if (variant >= 10 && variant <= 16) {
    FRH_REQUIRE(pok, "the pair kernel does not take this shape");
    hipStream_t st = as_stream(stream);
    if (variant == 10) launch_mw<2>(lv, c, out, total, st);
    else if (variant == 11) launch_mw<4>(lv, c, out, total, st);
    else if (variant == 12) launch_mw<2, 5>(lv, c, out, total, st);  // registers for 5 waves per SIMD
    else if (variant == 13) launch_mw<4, 5>(lv, c, out, total, st);
    else if (variant == 14) launch_mw<2, 1, true>(lv, c, out, total, st);  // 10, stamped
    else if (variant == 15) launch_mw<8>(lv, c, out, total, st);
    else launch_mw<4, 5, true>(lv, c, out, total, st);  // 13, stamped
  } else if (variant >= 20 && variant <= 27) {
    FRH_REQUIRE(pok, "the pair kernel does not take this shape");
    hipStream_t st = as_stream(stream);
    if (variant == 20) launch_mw<1, 1, false, true, false>(lv, c, out, total, st);       // dynamic DMA rounds
    else if (variant == 21) launch_mw<1, 1, false, true, true>(lv, c, out, total, st);   // + wide stores
    else if (variant == 22) launch_mw<2, 1, false, true, true>(lv, c, out, total, st);   // 21, 2 waves per WG
    else if (variant == 23) launch_mw<1, 1, true, true, true>(lv, c, out, total, st);    // 21 stamped
    else if (variant == 24) launch_mw<1, 1, false, false, true>(lv, c, out, total, st);  // wide stores only
    else if (variant == 25) launch_mw<2, 5, false, true, true>(lv, c, out, total, st);
    else if (variant == 26) launch_mw<2, 1, false, true, false>(lv, c, out, total, st);  // 20, 2 waves per WG
    else if (variant == 27) launch_mw<4, 1, false, true, false>(lv, c, out, total, st);  // 20, 4 waves per WG
    else FRH_REQUIRE(false, "roi_align variant %d unknown", variant);
  } else if (variant >= 30 && variant <= 33) {  // persistent pipelined waves: Q per XCD
    FRH_REQUIRE(pok, "the pair kernel does not take this shape");
    const unsigned q = variant == 30 ? 384 : variant == 31 ? 256 : variant == 32 ? 320 : 448;
    hipLaunchKernelGGL((roi_align_fwd_pipe_kernel<>), dim3(8 * q), dim3(kWave), 0, as_stream(stream), lv, c, out);
  } else {
    FRH_REQUIRE(false, "roi_align variant %d unknown", variant);
  }
  return check_launch("frh_roi_align_fwd_variant");
}

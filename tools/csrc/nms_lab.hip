// TOOLS-ONLY: the product NMS (mask + scan) with the scan's per-block timestamps.
#include "frcnn_tools.h"
#include "common.h"

namespace frh {
int32_t launch_nms_sorted(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                          double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                          uint64_t* mask, const int64_t* seg_base, hipStream_t st, int64_t* stamps);
}  // namespace frh

extern "C" int32_t frh_nms_sorted_stamped(int32_t num_segs, const float* boxes, int64_t seg_stride,
                                          const int32_t* counts, int32_t n_max, double iou_thr, int32_t max_keep,
                                          int32_t* keep, int64_t keep_seg_stride, int32_t* keep_counts,
                                          void* workspace, size_t ws_bytes, int64_t* stamps, void* stream) {
  FRH_REQUIRE(num_segs > 0 && n_max > 0 && stamps, "bad arguments");
  FRH_REQUIRE(workspace && ws_bytes >= frh_nms_workspace(num_segs, n_max), "workspace too small");
  return frh::launch_nms_sorted(num_segs, boxes, seg_stride, counts, n_max, iou_thr, max_keep, keep, keep_seg_stride,
                                keep_counts, static_cast<uint64_t*>(workspace), nullptr, frh::as_stream(stream),
                                stamps);
}

namespace frh {
bool nms_fused_fits(int32_t S, int32_t n_max);
size_t nms_fused_flag_bytes(int32_t S, int32_t n_max);
int32_t launch_nms_fused(int32_t S, const float* boxes, int64_t seg_stride, const int32_t* counts, int32_t n_max,
                         double thr, int32_t max_keep, int32_t* keep, int64_t kstride, int32_t* kcounts,
                         uint64_t* mask, uint32_t* flags, int32_t* status, hipStream_t st, int64_t* stamps,
                         const float* row_scores = nullptr, uint32_t* kscore = nullptr);
}  // namespace frh

// The RPN's one-launch NMS (nms_fused_kernel) on pre-sorted segments, tiles at s * tri(nbw):
// workspace = frh_nms_workspace bytes of mask + frh_nms_fused_flag_bytes of flags (zeroed
// here); stamps (or null): the kernel's timing build, S * nbw * 8 + S * tri(nbw) int64.
extern "C" size_t frh_nms_fused_flag_bytes(int32_t num_segs, int32_t n_max) {
  return frh::nms_fused_flag_bytes(num_segs, n_max);
}

extern "C" int32_t frh_nms_fused_stamped(int32_t num_segs, const float* boxes, int64_t seg_stride,
                                         const int32_t* counts, int32_t n_max, double iou_thr, int32_t max_keep,
                                         int32_t* keep, int64_t keep_seg_stride, int32_t* keep_counts,
                                         int32_t* status, void* workspace, size_t ws_bytes, int64_t* stamps,
                                         void* stream) {
  const size_t mb = frh_nms_workspace(num_segs, n_max), fb = frh::nms_fused_flag_bytes(num_segs, n_max);
  FRH_REQUIRE(workspace && ws_bytes >= mb + fb, "workspace too small");
  uint32_t* flags = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + mb);
  FRH_HIP(hipMemsetAsync(flags, 0, fb, frh::as_stream(stream)));
  return frh::launch_nms_fused(num_segs, boxes, seg_stride, counts, n_max, iou_thr, max_keep, keep, keep_seg_stride,
                               keep_counts, static_cast<uint64_t*>(workspace), flags, status, frh::as_stream(stream),
                               stamps);
}

// TOOLS-ONLY: the multi-launch forms of the one-launch kernels, for A/B timing and the
// equality tests (tests/test_gpu_fused.py): frh_rpn_proposals_strided with the four-launch
// selection (keys / refine / collect / rank) instead of rpn_select_kernel, or with the
// two-launch NMS (mask, scan) instead of nms_fused_kernel, and frh_sample_random with the
// keys + collect launches instead of sampler_fused_kernel.
#include "frcnn_tools.h"
#include "common.h"

namespace frh {
int32_t rpn_proposals_impl(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                           const float* const* reg_ptrs, const int64_t* cls_strides, const int64_t* reg_strides,
                           const int32_t* grid_hw, int32_t num_anchors, int32_t cls_channels, const float* anchors,
                           int64_t anchor_ld, const float* means, const float* stds, const float* img_hw,
                           const float* min_size, int32_t pre_nms, int32_t post_nms, int32_t max_num, double nms_iou,
                           float* out_boxes, float* out_scores, int32_t* out_counts, int32_t* status,
                           void* workspace, size_t ws_bytes, void* stream, bool select_launches,
                           int64_t* select_stamps = nullptr, bool nms_launches = false,
                           bool merge_launch = false, int64_t* nms_stamps = nullptr);
int32_t sample_random_impl(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                           const int32_t* num_boxes, int64_t max_boxes, int32_t max_num, int32_t pos_num,
                           uint64_t seed, int64_t* labels_out, int32_t* sel, int32_t* sel_counts, int32_t* status,
                           void* workspace, size_t ws_bytes, void* stream, bool two_launches,
                           int64_t* stamps = nullptr);
}  // namespace frh

extern "C" int32_t frh_rpn_proposals_launches(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                              const float* const* reg_ptrs, const int64_t* cls_strides,
                                              const int64_t* reg_strides, const int32_t* grid_hw,
                                              int32_t num_anchors, int32_t cls_channels, const float* anchors,
                                              int64_t anchor_ld, const float* means, const float* stds,
                                              const float* img_hw, const float* min_size, int32_t pre_nms,
                                              int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                              float* out_scores, int32_t* out_counts, int32_t* status, void* workspace,
                                              size_t ws_bytes, void* stream) {
  return frh::rpn_proposals_impl(num_imgs, num_levels, cls_ptrs, reg_ptrs, cls_strides, reg_strides, grid_hw,
                                 num_anchors, cls_channels, anchors, anchor_ld, means, stds, img_hw, min_size, pre_nms,
                                 post_nms, max_num, nms_iou, out_boxes, out_scores, out_counts, status, workspace, ws_bytes,
                                 stream, true);
}

extern "C" int32_t frh_rpn_proposals_nms2(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                          const float* const* reg_ptrs, const int64_t* cls_strides,
                                          const int64_t* reg_strides, const int32_t* grid_hw, int32_t num_anchors,
                                          int32_t cls_channels, const float* anchors, int64_t anchor_ld,
                                          const float* means, const float* stds, const float* img_hw,
                                          const float* min_size, int32_t pre_nms, int32_t post_nms, int32_t max_num,
                                          double nms_iou, float* out_boxes, float* out_scores, int32_t* out_counts,
                                          int32_t* status, void* workspace, size_t ws_bytes, void* stream) {
  return frh::rpn_proposals_impl(num_imgs, num_levels, cls_ptrs, reg_ptrs, cls_strides, reg_strides, grid_hw,
                                 num_anchors, cls_channels, anchors, anchor_ld, means, stds, img_hw, min_size, pre_nms,
                                 post_nms, max_num, nms_iou, out_boxes, out_scores, out_counts, status, workspace, ws_bytes,
                                 stream, false, nullptr, true);
}

// the round-4 merge (rpn_merge_lds_kernel) after the one-launch NMS instead of rpn_merge_wide_kernel
extern "C" int32_t frh_rpn_proposals_merge_launch(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                                  const float* const* reg_ptrs, const int64_t* cls_strides,
                                                  const int64_t* reg_strides, const int32_t* grid_hw,
                                                  int32_t num_anchors, int32_t cls_channels, const float* anchors,
                                                  int64_t anchor_ld, const float* means, const float* stds,
                                                  const float* img_hw, const float* min_size, int32_t pre_nms,
                                                  int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                                  float* out_scores, int32_t* out_counts, int32_t* status,
                                                  void* workspace, size_t ws_bytes, void* stream) {
  return frh::rpn_proposals_impl(num_imgs, num_levels, cls_ptrs, reg_ptrs, cls_strides, reg_strides, grid_hw,
                                 num_anchors, cls_channels, anchors, anchor_ld, means, stds, img_hw, min_size, pre_nms,
                                 post_nms, max_num, nms_iou, out_boxes, out_scores, out_counts, status, workspace, ws_bytes,
                                 stream, false, nullptr, false, true);
}

// the one-launch NMS with its stamps (nms_fused_kernel<true>: S * nbw * 8 per-block + S * tri
// per-tile int64, stamps zeroed by the caller)
extern "C" int32_t frh_rpn_proposals_nms_stamped(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                                 const float* const* reg_ptrs, const int64_t* cls_strides,
                                                 const int64_t* reg_strides, const int32_t* grid_hw,
                                                 int32_t num_anchors, int32_t cls_channels, const float* anchors,
                                                 int64_t anchor_ld, const float* means, const float* stds,
                                                 const float* img_hw, const float* min_size, int32_t pre_nms,
                                                 int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                                 float* out_scores, int32_t* out_counts, int32_t* status,
                                                 void* workspace, size_t ws_bytes, int64_t* stamps, void* stream) {
  return frh::rpn_proposals_impl(num_imgs, num_levels, cls_ptrs, reg_ptrs, cls_strides, reg_strides, grid_hw,
                                 num_anchors, cls_channels, anchors, anchor_ld, means, stds, img_hw, min_size, pre_nms,
                                 post_nms, max_num, nms_iou, out_boxes, out_scores, out_counts, status, workspace, ws_bytes,
                                 stream, false, nullptr, false, false, stamps);
}

extern "C" int32_t frh_sample_random_launches(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                                              const int32_t* num_boxes, int64_t max_boxes, int32_t max_num,
                                              int32_t pos_num, uint64_t seed, int64_t* labels_out, int32_t* sel,
                                              int32_t* sel_counts, int32_t* status, void* workspace, size_t ws_bytes,
                                              void* stream) {
  return frh::sample_random_impl(num_segs, labels_in, label_seg_stride, num_boxes, max_boxes, max_num, pos_num, seed,
                                 labels_out, sel, sel_counts, status, workspace, ws_bytes, stream, true);
}

// the one-launch kernels with per-workgroup phase stamps (16 int64 per workgroup of the grid,
// s_memrealtime): rpn_select_kernel [S][grid x][16], sampler_fused_kernel [images][chunks][16]
extern "C" int32_t frh_rpn_proposals_stamped(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                             const float* const* reg_ptrs, const int64_t* cls_strides,
                                             const int64_t* reg_strides, const int32_t* grid_hw,
                                             int32_t num_anchors, int32_t cls_channels, const float* anchors,
                                             int64_t anchor_ld, const float* means, const float* stds,
                                             const float* img_hw, const float* min_size, int32_t pre_nms,
                                             int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                             float* out_scores, int32_t* out_counts, int32_t* status, void* workspace,
                                             size_t ws_bytes, int64_t* stamps, void* stream) {
  return frh::rpn_proposals_impl(num_imgs, num_levels, cls_ptrs, reg_ptrs, cls_strides, reg_strides, grid_hw,
                                 num_anchors, cls_channels, anchors, anchor_ld, means, stds, img_hw, min_size, pre_nms,
                                 post_nms, max_num, nms_iou, out_boxes, out_scores, out_counts, status, workspace, ws_bytes,
                                 stream, false, stamps);
}

extern "C" int32_t frh_sample_random_stamped(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                                             const int32_t* num_boxes, int64_t max_boxes, int32_t max_num,
                                             int32_t pos_num, uint64_t seed, int64_t* labels_out, int32_t* sel,
                                             int32_t* sel_counts, int32_t* status, void* workspace, size_t ws_bytes, int64_t* stamps,
                                             void* stream) {
  return frh::sample_random_impl(num_segs, labels_in, label_seg_stride, num_boxes, max_boxes, max_num, pos_num, seed,
                                 labels_out, sel, sel_counts, status, workspace, ws_bytes, stream, false, stamps);
}

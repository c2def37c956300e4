// TOOLS-ONLY entry points (tools/lib/libfrcnn_tools.so; never linked into the product
// library).  RoIAlign forward laboratory: the product's forward kernel and a per-wave
// timestamped build of it (tools/bench_roi_align.py); the NMS scan's stamped build
// (tools/bench_nms.py).
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* variant 0: frh_roi_align_fwd_strided's pair kernel; 1: the same with per-item stamps (8
 * int64 per item after the output).  Arguments as frh_roi_align_fwd_strided, plus a
 * workspace of frh_roi_align_workspace bytes (unused by these two). */
/* round-6 backward A/B: 0 nhwc float, 1 register-resident float, 2 / 3 the same in fixed point */
int32_t frh_roi_align_bwd_variant(int32_t variant, int32_t num_levels, float* const* grad_feats,
                                  int64_t* const* acc_feats, const int32_t* feat_hw, const int64_t* strides,
                                  const float* scales, int32_t batch, int32_t channels, const float* rois,
                                  const int64_t* roi_levels, int64_t num_rois, const float* grad_out,
                                  uint32_t* scale_word, void* stream);
int32_t frh_roi_align_fwd_variant(int32_t variant, int32_t num_levels, const float* const* feats,
                                  const int32_t* feat_hw, const int64_t* strides, const float* scales,
                                  int32_t batch, int32_t channels, const float* rois, const int64_t* roi_levels,
                                  int64_t num_rois, int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio,
                                  int32_t aligned, float* out, void* workspace, size_t ws_bytes, void* stream);
/* workspace bytes of frh_roi_align_fwd_variant for num_rois RoIs */
size_t frh_roi_align_workspace(int64_t num_rois);

/* frh_nms_sorted with the stamped scan build: per (segment, column block) 8 int64 of
 * s_memrealtime (100 MHz) at stamps + (s * ceil(n_max / 64) + b) * 8 -- resolver starts
 * waiting, block ready seen, block resolved, loader fold published, loader copies issued. */
int32_t frh_nms_sorted_stamped(int32_t num_segs, const float* boxes, int64_t seg_stride, const int32_t* counts,
                               int32_t n_max, double iou_thr, int32_t max_keep, int32_t* keep,
                               int64_t keep_seg_stride, int32_t* keep_counts, void* workspace, size_t ws_bytes,
                               int64_t* stamps, void* stream);

/* The RPN's one-launch NMS (nms_fused_kernel) on pre-sorted segments: workspace = the
 * frh_nms_workspace mask bytes followed by frh_nms_fused_flag_bytes flag bytes (zeroed by the
 * call); stamps null (plain build) or num_segs * ceil(n_max / 64) * 8 + num_segs * tri int64
 * (timing build). */
size_t frh_nms_fused_flag_bytes(int32_t num_segs, int32_t n_max);
int32_t frh_nms_fused_stamped(int32_t num_segs, const float* boxes, int64_t seg_stride, const int32_t* counts,
                              int32_t n_max, double iou_thr, int32_t max_keep, int32_t* keep, int64_t keep_seg_stride,
                              int32_t* keep_counts, int32_t* status, void* workspace, size_t ws_bytes, int64_t* stamps,
                              void* stream);

/* frh_rpn_proposals_strided with the four-launch selection (keys, refine, collect, rank)
 * instead of the one-launch rpn_select_kernel; same arguments and outputs. */
int32_t frh_rpn_proposals_launches(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                   const float* const* reg_ptrs, const int64_t* cls_strides,
                                   const int64_t* reg_strides, const int32_t* grid_hw, int32_t num_anchors,
                                   int32_t cls_channels, const float* anchors, int64_t anchor_ld, const float* means,
                                   const float* stds, const float* img_hw, const float* min_size, int32_t pre_nms,
                                   int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                   float* out_scores, int32_t* out_counts, int32_t* status, void* workspace, size_t ws_bytes,
                                   void* stream);

/* frh_rpn_proposals_strided with the two-launch NMS (mask, scan) instead of the one-launch
 * nms_fused_kernel; same arguments and outputs. */
int32_t frh_rpn_proposals_nms2(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                               const float* const* reg_ptrs, const int64_t* cls_strides, const int64_t* reg_strides,
                               const int32_t* grid_hw, int32_t num_anchors, int32_t cls_channels, const float* anchors,
                               int64_t anchor_ld, const float* means, const float* stds, const float* img_hw,
                               const float* min_size, int32_t pre_nms, int32_t post_nms, int32_t max_num,
                               double nms_iou, float* out_boxes, float* out_scores, int32_t* out_counts,
                               int32_t* status, void* workspace, size_t ws_bytes, void* stream);

/* frh_rpn_proposals_strided with the round-4 cross-level merge (rpn_merge_lds_kernel: one
 * workgroup per level and image, keep-index indirection) instead of rpn_merge_wide_kernel. */
int32_t frh_rpn_proposals_merge_launch(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                       const float* const* reg_ptrs, const int64_t* cls_strides,
                                       const int64_t* reg_strides, const int32_t* grid_hw, int32_t num_anchors,
                                       int32_t cls_channels, const float* anchors, int64_t anchor_ld,
                                       const float* means, const float* stds, const float* img_hw,
                                       const float* min_size, int32_t pre_nms, int32_t post_nms, int32_t max_num,
                                       double nms_iou, float* out_boxes, float* out_scores, int32_t* out_counts,
                                       int32_t* status, void* workspace, size_t ws_bytes, void* stream);

/* frh_sample_random with the keys + collect launches instead of the one-launch sampler. */
int32_t frh_sample_random_launches(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                                   const int32_t* num_boxes, int64_t max_boxes, int32_t max_num, int32_t pos_num,
                                   uint64_t seed, int64_t* labels_out, int32_t* sel, int32_t* sel_counts,
                                   int32_t* status, void* workspace, size_t ws_bytes, void* stream);

/* the one-launch selection kernels with per-workgroup phase stamps (16 int64 of s_memrealtime
 * per workgroup of the grid): rpn_select_kernel [S][grid x][16] (frh_rpn_proposals_strided's
 * arguments + stamps), sampler_fused_kernel [images][chunks][16] (frh_sample_random's + stamps) */
int32_t frh_rpn_proposals_stamped(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                  const float* const* reg_ptrs, const int64_t* cls_strides,
                                  const int64_t* reg_strides, const int32_t* grid_hw, int32_t num_anchors,
                                  int32_t cls_channels, const float* anchors, int64_t anchor_ld, const float* means,
                                  const float* stds, const float* img_hw, const float* min_size, int32_t pre_nms,
                                  int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                  float* out_scores, int32_t* out_counts, int32_t* status, void* workspace, size_t ws_bytes,
                                  int64_t* stamps, void* stream);

/* the one-launch NMS timing build inside the proposals: stamps = S*nbw*8 per-block + S*tri
 * per-tile int64 (nms_fused_kernel<true>), zeroed by the caller. */
int32_t frh_rpn_proposals_nms_stamped(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                  const float* const* reg_ptrs, const int64_t* cls_strides,
                                  const int64_t* reg_strides, const int32_t* grid_hw, int32_t num_anchors,
                                  int32_t cls_channels, const float* anchors, int64_t anchor_ld, const float* means,
                                  const float* stds, const float* img_hw, const float* min_size, int32_t pre_nms,
                                  int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                  float* out_scores, int32_t* out_counts, int32_t* status, void* workspace, size_t ws_bytes,
                                  int64_t* stamps, void* stream);
int32_t frh_sample_random_stamped(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                                  const int32_t* num_boxes, int64_t max_boxes, int32_t max_num, int32_t pos_num,
                                  uint64_t seed, int64_t* labels_out, int32_t* sel, int32_t* sel_counts,
                                  int32_t* status, void* workspace, size_t ws_bytes, int64_t* stamps, void* stream);

#ifdef __cplusplus
}
#endif

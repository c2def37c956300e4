/* TOOLS ONLY: entry points of tools/lib/libfrcnn_tools.so (tools/csrc/*.hip),
 * the RoIAlign variants measured on the way to the product kernels.
 * Not part of the product ABI (include/frcnn_amd.h); the product library does
 * not export these.  Same conventions as include/frcnn_amd.h. */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Plane-sweep forward (measured slower than the product kernel: 104 vs 45 us on cfg2;
 * sampling_ratio 2, even C, unit x
 * stride, W_l <= 256): one workgroup per (level, image, channel pair) streams
 * that plane pair through an LDS row ring exactly once and evaluates every
 * (RoI, bin row) as soon as its rows have landed; a small plan launch first
 * writes each bin row's y taps and each (RoI, px)'s x taps into the workspace
 * (frh_roi_align_sweep_workspace bytes).  Bit-identical to
 * frh_roi_align_fwd_strided, which it falls back to for any other shape or a
 * missing / short workspace. */
size_t frh_roi_align_sweep_workspace(int64_t num_rois, int32_t pooled_h, int32_t pooled_w);
int32_t frh_roi_align_fwd_sweep(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                                const int64_t* strides, const float* scales, int32_t batch, int32_t channels,
                                const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                float* out, void* workspace, size_t ws_bytes, void* stream);
/* Plane-sweep backward: the same sweep accumulates each (image, channel pair)'s
 * gradient rows in LDS and writes every element of grad_feats exactly once
 * (no clearing, no global atomics).  Returns FRH_EUNSUPPORTED (nothing
 * launched) outside the sweep's shapes or without the workspace
 * (frh_roi_align_sweep_workspace bytes): the caller then clears the gradient
 * and uses frh_roi_align_bwd_strided.  Float atomics in LDS: the summation
 * order, and the last bits, vary from run to run (as torchvision's CUDA). */
int32_t frh_roi_align_bwd_sweep(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                                const int64_t* strides, const float* scales, int32_t batch, int32_t channels,
                                const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                const float* grad_out, void* workspace, size_t ws_bytes, void* stream);
/* The grouped forward (opt-in): a one-workgroup planning launch sorts the
 * RoIs into spatial groups of 8 (same image and level); the main launch
 * stages the union of each group's tap rows per channel into LDS by LDS-DMA
 * and evaluates every RoI of the group from it, so a line shared by several
 * RoIs is fetched once.  Bit-identical to frh_roi_align_fwd_strided, which it
 * falls back to when the workspace is absent / short, K > 8192, or the shape
 * is outside (sampling 2, ph*pw <= 64).  workspace: frh_roi_align_workspace(K)
 * bytes.  Currently slower than the default on cfg2. */
size_t frh_roi_align_workspace(int64_t num_rois);
int32_t frh_roi_align_fwd_ws(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                             const int64_t* strides, const float* scales, int32_t batch, int32_t channels,
                             const float* rois, const int64_t* roi_levels, int64_t num_rois,
                             int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                             float* out, void* workspace, size_t ws_bytes, void* stream);
/* A named forward kernel (0 direct gather, 10 per-RoI LDS windows, 20 channel pairs
 * = the product default, 25 persistent, 30 wide-staged, 50 grouped, 51 grouped with
 * timing stamps written past the results; -1 = default, -2 = grouped if possible;
 * list in tools/csrc/roi_variants.hip). */
int32_t frh_roi_align_fwd_variant(int32_t variant, int32_t num_levels, const float* const* feats,
                                  const int32_t* feat_hw, const int64_t* strides, const float* scales,
                                  int32_t batch, int32_t channels, const float* rois,
                                  const int64_t* roi_levels, int64_t num_rois, int32_t pooled_h,
                                  int32_t pooled_w, int32_t sampling_ratio, int32_t aligned, float* out,
                                  void* workspace, size_t ws_bytes, void* stream);
/* Tiled gather backward (sampling_ratio 2, pooled_h * pooled_w <= 64): the same
 * gradient as frh_roi_align_bwd_strided without global atomics.  OVERWRITES every
 * cell of grad_feats (no need to clear it first).  Workspace: caller-allocated,
 * frh_roi_align_bwd_workspace bytes (tile lists over 16x16-cell tiles). */
size_t frh_roi_align_bwd_workspace(int32_t num_levels, const int32_t* feat_hw, int32_t batch,
                                   int64_t num_rois);
int32_t frh_roi_align_bwd_tiled(int32_t num_levels, float* const* grad_feats,
                                const int32_t* feat_hw, const int64_t* strides,
                                const float* scales, int32_t batch, int32_t channels,
                                const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio,
                                int32_t aligned, const float* grad_out, void* workspace,
                                size_t ws_bytes, void* stream);

/* Backward into a channels-last gradient (unit channel stride, C % 16 == 0):
 * 64-B atomic segments per 16 channels (measured slower than the product's). */
int32_t frh_roi_align_bwd_cl(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                             const int64_t* strides, const float* scales, int32_t batch, int32_t channels,
                             const float* rois, const int64_t* roi_levels, int64_t num_rois,
                             int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                             const float* grad_out, void* stream);

/* The product NMS rebuilt with per-block resolver timestamps (tools/csrc/nms_timeline.hip):
 * same arguments as frh_nms_workspace / frh_nms_sorted; frh_tl_nms_timeline sets the
 * stamp buffer (uint64 [S][256][8] wall_clock64 ticks, nullptr = off). */
size_t frh_tl_nms_workspace(int32_t num_segs, int32_t n_max);
int32_t frh_tl_nms_sorted(int32_t num_segs, const float* boxes, int64_t seg_stride, const int32_t* counts,
                          int32_t n_max, double iou_thr, int32_t max_keep, int32_t* keep, int64_t keep_seg_stride,
                          int32_t* keep_counts, void* workspace, size_t ws_bytes, void* stream);
int32_t frh_tl_nms_timeline(void* stamps);

/* tools/csrc/nms_exact.hip: the exact-test mask NMS (A/B of the float-filtered mask) */
size_t frh_ex_nms_workspace(int32_t num_segs, int32_t n_max);
int32_t frh_ex_nms_sorted(int32_t num_segs, const float* boxes, int64_t seg_stride, const int32_t* counts,
                          int32_t n_max, double iou_thr, int32_t max_keep, int32_t* keep, int64_t keep_seg_stride,
                          int32_t* keep_counts, void* workspace, size_t ws_bytes, void* stream);

/* The product RPN proposals rebuilt with segment-0 top-k timestamps
 * (tools/csrc/topk_timeline.hip): same arguments as frh_rpn_proposals_workspace /
 * frh_rpn_proposals / frh_rpn_proposals_nms_view; frh_tl_topk_timeline sets the stamp
 * buffer (uint64 [2048] wall_clock64 ticks: [4 g + 0..2] per collect workgroup g,
 * [1024 + 0..7] the last workgroup; nullptr = off). */
size_t frh_tl_rpn_proposals_workspace(int32_t num_imgs, int32_t num_levels, const int32_t* grid_hw,
                                      int32_t num_anchors, int32_t pre_nms);
int32_t frh_tl_rpn_proposals(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                             const float* const* reg_ptrs, const int32_t* grid_hw, int32_t num_anchors,
                             int32_t cls_channels, const float* anchors, int64_t anchor_ld, const float* means,
                             const float* stds, const float* img_hw, const float* min_size, int32_t pre_nms,
                             int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                             float* out_scores, int32_t* out_counts, void* workspace, size_t ws_bytes,
                             void* stream);
int32_t frh_tl_rpn_proposals_nms_view(int32_t num_imgs, int32_t num_levels, const int32_t* grid_hw,
                                      int32_t num_anchors, int32_t pre_nms, int64_t* out);
int32_t frh_tl_topk_timeline(void* stamps);

#ifdef __cplusplus
}
#endif

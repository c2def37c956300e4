/*
 * frcnn_amd.h — C-ABI of the MI355X (gfx950) Faster R-CNN detection hot path.
 *
 * Every entry point replaces one function/type of the reference
 * (pengfeidip/pytorch-faster-rcnn, cited as path:line) or of the third-party
 * torchvision kernels the reference calls.  Conventions:
 *   - plain device pointers + sizes; no framework types.  Boxes are
 *     coordinate-major "[4, n]" float32 (row k = coordinate k, row stride `ld`
 *     elements), exactly the reference's channel-first layout, unless a
 *     parameter says "[n,4]" (row-major xyxy, torchvision layout).
 *   - `stream` is a hipStream_t; every call is asynchronous on it and never
 *     synchronises, allocates or frees (capturable into a hipGraph).
 *   - scratch memory comes from the caller through (workspace, ws_bytes);
 *     each op has a *_workspace() size query.  The library keeps no global
 *     mutable state: reentrant and thread-safe per stream.
 *   - variable-size results are written into caller-sized maxima plus a
 *     device-side int32 count.
 *   - return 0 on success, a negative FRH_E* code otherwise;
 *     frh_last_error() gives a thread-local message.
 */
#ifndef FRCNN_AMD_H
#define FRCNN_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRH_ABI_VERSION 3

#define FRH_OK 0
#define FRH_EINVAL (-1)
#define FRH_EUNSUPPORTED (-2)
#define FRH_ELAUNCH (-3)

#define FRH_MAX_LEVELS 8

int32_t frh_abi_version(void);
const char* frh_last_error(void);

/* Device status word (ABI 2).  The one-launch kernels of frh_rpn_proposals* and
 * frh_sample_random hand data between the workgroups of ONE launch through bounded
 * in-launch waits, sized to the device's resident capacity (CU count x occupancy, queried
 * per device).  A wait that runs out -- a workgroup it needs was never scheduled, e.g. beside
 * other kernels or on a partitioned GPU -- ORs one of these bits into the caller's device
 * int32 `status` word and ends that workgroup's work: the call's outputs are then undefined
 * and the workspace's zero region may be left dirty (re-zero it).  The library never reads
 * the word except (ABI 3) the loss entries, which write NaN losses while it is nonzero, and
 * frh_sample_random's one-launch form, which does nothing while it is nonzero (its zero region
 * may be dirty): the step's own loss read carries a failure, and the caller checks the word
 * where it synchronises anyway (frcnn_amd: every training step before the optimizer update,
 * the numpy sampler's count read, or after every call with FRCNN_AMD_DEBUG=1) and clears it. */
#define FRH_DEVERR_SELECT_BARRIER 1   /* rpn_select_kernel: a segment barrier timed out */
#define FRH_DEVERR_NMS_COLUMN 2       /* nms_fused_kernel: a mask column never completed */
#define FRH_DEVERR_SAMPLER_BARRIER 4  /* sampler_fused_kernel: an image barrier timed out */

/* ---- a1: AnchorCreator.__call__ over all FPN levels in one launch ------------
 * Replaces lib/anchor.py:107-129 (called per level from
 * lib/heads/anchor_head.py:66-67).  Level l has grid (grid_hw[2l], grid_hw[2l+1]),
 * stride strides[l] and per-anchor sizes ws/hs[l*num_anchors + a] (the f32
 * casts of the reference's float64 base*s*sqrt(ar), anchor.py:92-97).
 * Output: [4, ld] with level l occupying columns [off_l, off_l + A*H*W) in
 * the reference's [4, A, H, W].view(4,-1) order, off_l = sum of earlier levels. */
int32_t frh_anchor_grid(int32_t num_levels, const int32_t* grid_hw, const float* strides,
                        const float* ws, const float* hs, int32_t num_anchors,
                        int32_t center_lt, float* out, int64_t ld, void* stream);

/* ---- a2: inside_anchor_mask & inside_grid_mask --------------------------------
 * Replaces lib/region.py:10-29 as combined in lib/heads/anchor_head.py:93-99.
 * in_hw[2l..] = min(grid, int(img/stride)+1) computed by the caller in double
 * exactly as region.py:12-13.  allowed_border < 0 disables the image test. */
int32_t frh_inside_mask(const float* anchors, int64_t ld, int32_t num_levels,
                        const int32_t* grid_hw, const int32_t* in_hw, int32_t num_anchors,
                        int32_t img_h, int32_t img_w, int32_t allowed_border,
                        uint8_t* mask, void* stream);

/* ---- a3: calc_iou / elem_iou ----------------------------------------------------
 * calc_iou: lib/utils.py:151-172 -> out[n, k] (row-major), bit-exact.
 * elem_iou: lib/utils.py:174-182 (no +1) -> out[n]. */
int32_t frh_iou_table(const float* a, int64_t lda, int64_t n, const float* b, int64_t ldb,
                      int64_t k, float* out, void* stream);
int32_t frh_elem_iou(const float* a, int64_t lda, const float* b, int64_t ldb, int64_t n,
                     float* out, void* stream);

/* ---- a4: MaxIoUAssigner.__call__, batched over segments (images) -------------
 * Replaces lib/region.py:60-107.  Segment s: boxes at boxes + s*box_seg_stride
 * ([4, box_ld]), count num_boxes[s] (device), optional validity mask
 * valid + s*valid_seg_stride (nullptr = all valid; invalid boxes get label -1
 * and take no part in the per-gt maxima), gts at gts + s*gt_seg_stride
 * ([4, gt_ld]), count num_gts[s] (device).  Labels are int64:
 * -1 ignore, 0 negative, g+1 positive for gt g; max_iou f32.  Thresholds are
 * compared in f32 like the reference (`f32 tensor < python float`).  Rows in
 * [num_boxes[s], max_boxes) are padding: label -1, max_iou 0.
 * max_boxes / max_gts bound the launch (host-known maxima of the counts).  One launch: the
 * last workgroup of each segment labels the boxes tied at a gt's maximum (hand-off inside
 * the launch).  Workspace: frh_maxiou_assign_workspace bytes whose leading
 * frh_maxiou_assign_zero_bytes(num_segs, max_gts) bytes are zero before the call; every call
 * leaves them zero, so a caller zero-fills them once per (num_segs, max_gts) layout and reuses
 * the buffer for calls ordered on one stream. */
size_t frh_maxiou_assign_zero_bytes(int32_t num_segs, int32_t max_gts);
size_t frh_maxiou_assign_workspace(int32_t num_segs, int32_t max_gts, int64_t max_boxes);
int32_t frh_maxiou_assign(int32_t num_segs, const float* boxes, int64_t box_ld,
                          int64_t box_seg_stride, const int32_t* num_boxes,
                          const uint8_t* valid, int64_t valid_seg_stride,
                          const float* gts, int64_t gt_ld, int64_t gt_seg_stride,
                          const int32_t* num_gts, float pos_iou, float neg_iou,
                          float min_pos_iou, int64_t* labels, int64_t label_seg_stride,
                          float* max_iou, int64_t iou_seg_stride, int64_t max_boxes,
                          int32_t max_gts, void* workspace, size_t ws_bytes, void* stream);

/* ---- a5: RandomSampler / random_sample_label ----------------------------------
 * Replaces lib/region.py:43-57,112-126.  Two modes:
 *  (1) reference-RNG parity: frh_sample_candidates lists, per segment and in
 *      ascending box order, the positive (label>0) and negative (label==0)
 *      boxes plus their counts ([S,2] device int32).  The host draws the
 *      reference's numpy permutation, then frh_sample_apply keeps the chosen
 *      list positions (keep_pos/keep_neg [S, keep_ld] device, counts in
 *      keep_counts [S,2]) and writes labels_out (-1 for everything else).
 *  (2) device RNG: frh_sample_random keeps min(npos,pos_num) positives and
 *      min(nneg, max_num-kept_pos) negatives, each chosen uniformly without
 *      replacement by the smallest 32-bit hash(seed, seg, box) keys.  Outputs
 *      (either or both): labels_out (the sampled labels, -1 elsewhere) and / or
 *      sel [S][2][max_num] (the kept positives / negatives, in no order) with
 *      sel_counts [S][2] -- the form frh_anchor_target / frh_bbox_target take
 *      without a compaction pass over every box. */
size_t frh_sample_workspace(int32_t num_segs, int64_t max_boxes);
/* frh_sample_random's workspace contract: its leading frh_sample_zero_bytes(num_segs) bytes
 * (the same for every num_segs <= 64: nothing else is placed there) are zero before the call
 * and every completed call leaves them zero (images above 16 384 boxes take a one-launch
 * sampler whose per-image counters and histograms live there and are reset by the launch's
 * last workgroup), so a caller zero-fills the buffer once and reuses it for calls ordered on
 * one stream, whatever their num_segs.  After FRH_DEVERR_SAMPLER_BARRIER, re-zero it.
 * num_segs <= 64. */
size_t frh_sample_zero_bytes(int32_t num_segs);
int32_t frh_sample_candidates(int32_t num_segs, const int64_t* labels, int64_t label_seg_stride,
                              const int32_t* num_boxes, int64_t max_boxes, int32_t* pos_list,
                              int32_t* neg_list, int64_t list_seg_stride, int32_t* counts,
                              void* workspace, size_t ws_bytes, void* stream);
int32_t frh_sample_apply(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                         const int32_t* num_boxes, int64_t max_boxes, const int32_t* pos_list,
                         const int32_t* neg_list, int64_t list_seg_stride,
                         const int32_t* keep_pos, const int32_t* keep_neg, int64_t keep_ld,
                         const int32_t* keep_counts, int64_t* labels_out, void* stream);
int32_t frh_sample_random(int32_t num_segs, const int64_t* labels_in, int64_t label_seg_stride,
                          const int32_t* num_boxes, int64_t max_boxes, int32_t max_num,
                          int32_t pos_num, uint64_t seed, int64_t* labels_out, int32_t* sel,
                          int32_t* sel_counts, int32_t* status, void* workspace, size_t ws_bytes,
                          void* stream);

/* ---- a6: anchor_target (lib/anchor.py:11-76) after assign+sample -------------
 * Chosen = boxes with sampled label >= 0, ascending.  Segment outputs are
 * concatenated in segment order (the reference's per-image results followed
 * by torch.cat in anchor_head.py:189-192); out_counts[s] = chosen count of s,
 * out_counts[num_segs] = total.  Outputs (column j of the concatenation):
 *   chosen_idx[j] (int64, index into the per-segment box space),
 *   seg_of[j] (int32), tar_labels[j] (int64: gt_label[g] or 0 for negatives;
 *   gt_label == nullptr => 1/0), tar_anchors/tar_bbox/tar_param [4, out_ld].
 * tar_param = (bbox2param(anchor, gt) - means) / stds (anchor.py:69-73).
 * sel / sel_counts (nullable; frh_sample_random's lists, max_num = max_out_per_seg
 * <= 8192): the chosen boxes are those lists (ranked into ascending box order in
 * the gather itself) and `labels` are the assignment labels before sampling; no
 * workspace is needed.  With sel, columns [total, num_segs*max_out_per_seg) are padding
 * (seg_of -1, tar_labels -1, zero boxes), so a caller may consume the whole capacity
 * against the device total instead of reading it back. */
int32_t frh_anchor_target(int32_t num_segs, const int64_t* labels, int64_t label_seg_stride,
                          const int32_t* num_boxes, int64_t max_boxes, const float* anchors,
                          int64_t anchor_ld, int64_t anchor_seg_stride, const float* gts,
                          int64_t gt_ld, int64_t gt_seg_stride, const int64_t* gt_labels,
                          int64_t gt_label_seg_stride, const float* means, const float* stds,
                          int64_t max_out_per_seg, const int32_t* sel, const int32_t* sel_counts,
                          int64_t* chosen_idx, int32_t* seg_of,
                          int64_t* tar_labels, float* tar_anchors, float* tar_bbox,
                          float* tar_param, int64_t out_ld, int32_t* out_counts,
                          void* workspace, size_t ws_bytes, void* stream);
size_t frh_anchor_target_workspace(int32_t num_segs, int64_t max_boxes);

/* gather of per-level head outputs at chosen anchors (anchor.py:51-56) and its
 * adjoint (autograd backward).  Level l tensor: [B, C*A, H, W] contiguous
 * viewed per image as [C, A*H*W] (anchor_head.py:82); level_off[l] = first
 * flat index of the level.  out: [C, out_ld].  A column with seg_of < 0 (padding) gathers
 * zeros and scatters nothing. */
int32_t frh_gather_level_outputs(int32_t num_levels, const float* const* level_ptrs,
                                 const int64_t* level_off, const int64_t* level_hw_a,
                                 int32_t channels, int64_t total, const int64_t* chosen_idx,
                                 const int32_t* seg_of, float* out, int64_t out_ld,
                                 void* stream);
int32_t frh_scatter_level_grads(int32_t num_levels, float* const* level_grads,
                                const int64_t* level_off, const int64_t* level_hw_a,
                                int32_t channels, int64_t total, const int64_t* chosen_idx,
                                const int32_t* seg_of, const float* grad, int64_t grad_ld,
                                void* stream);
/* The same for head outputs of any layout (NCHW or channels-last): level l is
 * [B, C*A, H_l, W_l] with element strides level_strides[4l..4l+3] = (b, c, y, x),
 * level_hw[2l..2l+1] = (H_l, W_l), A = num_anchors; anchor index a*H*W + y*W + x of the
 * reference's [C, A*H*W] view reads tensor channel c*A + a. */
int32_t frh_gather_level_outputs_strided(int32_t num_levels, const float* const* level_ptrs,
                                         const int64_t* level_off, const int32_t* level_hw,
                                         const int64_t* level_strides, int32_t num_anchors,
                                         int32_t channels, int64_t total, const int64_t* chosen_idx,
                                         const int32_t* seg_of, float* out, int64_t out_ld,
                                         void* stream);
int32_t frh_scatter_level_grads_strided(int32_t num_levels, float* const* level_grads,
                                        const int64_t* level_off, const int32_t* level_hw,
                                        const int64_t* level_strides, int32_t num_anchors,
                                        int32_t channels, int64_t total, const int64_t* chosen_idx,
                                        const int32_t* seg_of, const float* grad, int64_t grad_ld,
                                        void* stream);

/* ---- a12: bbox_target (lib/bbox.py:6-82) ------------------------------------
 * frh_prepend_gt_labels builds the reference's candidate list
 * [gts ; proposals] (bbox.py:27-29): rows_out[s, j] = j+1 for j < G_s, else
 * prop_labels[s, j-G_s]; num_rows[s] = G_s + n_s; rows in [G_s + n_s, max_rows) are
 * padding, label -1.  After sampling those rows,
 * frh_bbox_target (labels = the sampled rows, num_rows from the prepend)
 * gathers the chosen rows (ascending) into concatenated
 * outputs: tar_props/tar_bbox/tar_param [4, out_ld], tar_label (int64, gt
 * class or 0), tar_is_gt (int64 0/1), out_counts[S+1] as in frh_anchor_target;
 * sel / sel_counts as in frh_anchor_target (labels = the prepended rows; padding columns
 * past the total: tar_label -1, tar_is_gt 0, zero boxes). */
int32_t frh_prepend_gt_labels(int32_t num_segs, const int64_t* prop_labels,
                              int64_t prop_label_seg_stride, const int32_t* num_props,
                              const int32_t* num_gts, int64_t max_rows, int64_t* rows_out,
                              int64_t rows_seg_stride, int32_t* num_rows, void* stream);
size_t frh_bbox_target_workspace(int32_t num_segs, int64_t max_rows);
int32_t frh_bbox_target(int32_t num_segs, const int64_t* labels, int64_t label_seg_stride,
                        const int32_t* num_rows, const int32_t* num_gts, int64_t max_rows,
                        const float* props, int64_t prop_ld, int64_t prop_seg_stride,
                        const float* gts, int64_t gt_ld, int64_t gt_seg_stride,
                        const int64_t* gt_labels, int64_t gt_label_seg_stride,
                        const float* means, const float* stds, int64_t max_out_per_seg,
                        const int32_t* sel, const int32_t* sel_counts,
                        float* tar_props, float* tar_bbox, int64_t* tar_label,
                        float* tar_param, int64_t* tar_is_gt, int64_t out_ld,
                        int32_t* out_counts, void* workspace, size_t ws_bytes, void* stream);

/* ---- a7/a8: bbox2param / param2bbox (+clamp_bbox) ----------------------------
 * lib/utils.py:47-70 and 83-144.  param2bbox handles the batched
 * [4*ncls, n] layout of batched_param2bbox (utils.py:96-106): class c of
 * coordinate k is row k*ncls + c, output in the same layout.  clamp != 0
 * clamps x to [0, img_w-1] and y to [0, img_h-1] (utils.py:109-120). */
int32_t frh_bbox2param(const float* base, int64_t ldb, const float* bbox, int64_t ldx,
                       int64_t n, const float* means, const float* stds, float* out,
                       int64_t ldo, void* stream);
int32_t frh_param2bbox(const float* base, int64_t ldb, const float* param, int64_t ldp,
                       int64_t n, int32_t ncls, const float* means, const float* stds,
                       int32_t clamp, float img_h, float img_w, float* out, int64_t ldo,
                       void* stream);

/* ---- a9/a10: RPNHead.predict_single_image, all images x levels ----------------
 * lib/heads/rpn_head.py:68-120 with torchvision.ops.nms semantics.  Per
 * (image, level): score = sigmoid(cls) (use_sigmoid) or softmax(cls)[1];
 * top pre_nms by (score desc, index asc); decode+clamp (param2bbox); drop
 * boxes with w+1 < min_size or h+1 < min_size when min_size > 0; greedy NMS
 * (IoU > nms_iou in double); first post_nms.  Then per image the levels are
 * concatenated and, if more than max_num survive, the max_num best are kept
 * in (score desc, concat order) order.  cls level l: [B, C*A, H_l, W_l],
 * reg level l: [B, 4*A, H_l, W_l]; anchors [4, anchor_ld] from
 * frh_anchor_grid.  img_hw / min_size are host arrays [B*2] / [B].
 * Outputs: boxes [B, 4, max_num], scores [B, max_num], counts [B] (device).
 * status: the device status word (FRH_DEVERR_SELECT_BARRIER, FRH_DEVERR_NMS_COLUMN). */
size_t frh_rpn_proposals_workspace(int32_t num_imgs, int32_t num_levels,
                                   const int32_t* grid_hw, int32_t num_anchors,
                                   int32_t pre_nms);
int32_t frh_rpn_proposals(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                          const float* const* reg_ptrs, const int32_t* grid_hw,
                          int32_t num_anchors, int32_t cls_channels, const float* anchors,
                          int64_t anchor_ld, const float* means, const float* stds,
                          const float* img_hw, const float* min_size, int32_t pre_nms,
                          int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                          float* out_scores, int32_t* out_counts, int32_t* status, void* workspace,
                          size_t ws_bytes, void* stream);

/* The same for head outputs of any layout (NCHW or the channels-last outputs of an NHWC
 * RPN head): cls_strides / reg_strides [L][4] element strides (b, c, y, x) of each level;
 * anchor a*H*W + y*W + x reads channel c*A + a (cls) / coord*A + a (reg), as the
 * reference's views (anchor_head.py:82, rpn_head.py:72). */
int32_t frh_rpn_proposals_strided(int32_t num_imgs, int32_t num_levels, const float* const* cls_ptrs,
                                  const float* const* reg_ptrs, const int64_t* cls_strides,
                                  const int64_t* reg_strides, const int32_t* grid_hw,
                                  int32_t num_anchors, int32_t cls_channels, const float* anchors,
                                  int64_t anchor_ld, const float* means, const float* stds,
                                  const float* img_hw, const float* min_size, int32_t pre_nms,
                                  int32_t post_nms, int32_t max_num, double nms_iou, float* out_boxes,
                                  float* out_scores, int32_t* out_counts, int32_t* status,
                                  void* workspace, size_t ws_bytes, void* stream);

/* Measurement hook: byte offsets in the frh_rpn_proposals workspace of its per-level
 * NMS input (out[0] boxes [S, P, 4] in descending-score order, out[1] counts [S]
 * int32), out[2] = P, out[3] = S = num_imgs * num_levels.  bench.py replays that
 * NMS alone for its roofline line. */
int32_t frh_rpn_proposals_nms_view(int32_t num_imgs, int32_t num_levels, const int32_t* grid_hw,
                                   int32_t num_anchors, int32_t pre_nms, int64_t* out);

/* ---- a10: torchvision.ops.nms on pre-sorted segments --------------------------
 * boxes [S, n_max, 4] row-major xyxy, already in descending-score order
 * (stable); count[s] valid rows, n_max <= 184320 (the offset-trick batched_nms of
 * lib/utils.py:211-221 runs one NMS over up to 1000 proposals x 20 classes).
 * keep[s, :] = kept row positions (ascending = score order), keep_counts[s].
 * max_keep >= 0 stops after that many.  Workspace: one upper-triangle suppression
 * mask of ceil(n_max / 64) column blocks per segment (512 B per 64x64 tile). */
size_t frh_nms_workspace(int32_t num_segs, int32_t n_max);
int32_t frh_nms_sorted(int32_t num_segs, const float* boxes, int64_t seg_stride,
                       const int32_t* counts, int32_t n_max, double iou_thr, int32_t max_keep,
                       int32_t* keep, int64_t keep_seg_stride, int32_t* keep_counts,
                       void* workspace, size_t ws_bytes, void* stream);

/* ---- a11: class-wise batched multiclass NMS ------------------------------------
 * Replaces utils.multiclass_nms + batched_nms (lib/utils.py:211-269), called per
 * image by anchor_head.py:207-262, fcos_head.py:566-627, bbox_head.py:122-146 --
 * here for B images at once, one NMS segment per (image, class).  Per image b:
 * boxes [n_max][4] (box_per_class = 0) or [n_max][4 * C] viewed (n, 4, C), scores
 * [n_max][C], optional score_factor [n_max] (or [n_max][C] with sf_per_class, official
 * mode) and row_valid [n_max] (0 = a row the reference removed before the call), rows
 * < num_rows[b] (device int32).
 * channel_mask [C] (device uint8) = the nms_channel set; mode 0 official (every
 * (row, class) pair), 1 strict (argmax class per row); pairs need score >=
 * min_score; the score is multiplied by score_factor after that test.
 * by_class = 1: one segment per (image, class); 0: one per image (the reference's
 * single pass; needed when a candidate coordinate is < 0).  Two calls, neither of
 * which allocates or synchronises: prepare (candidates + per-segment NMS mask
 * offsets) writes the device int32 info[4]: info[0] = the largest segment (limit
 * 65536), info[1] = 1 if a candidate coordinate is < 0 (with by_class = 1 the caller
 * then redoes prepare with by_class = 0), info[2] | info[3] << 32 = the NMS mask
 * tiles.  The caller copies info to the host, then calls finish (same mode /
 * by_class; scores needed in strict mode) with max_count = info[0], mask_tiles =
 * info[2..3] and an NMS workspace of frh_mcnms_nms_workspace(..., max_count,
 * mask_tiles) bytes: per-segment sort (score desc, candidate asc), torchvision nms per
 * segment, the keeps of all classes merged in (score desc, candidate asc) order, the
 * first max_num (<= 0: all) written to out_boxes [B][out_cap][4], out_scores
 * [B][out_cap], out_labels [B][out_cap] (the class index), out_counts [B] (device). */
size_t frh_mcnms_workspace(int32_t num_imgs, int32_t num_classes, int64_t n_max);
int32_t frh_mcnms_prepare(int32_t num_imgs, int32_t num_classes, int64_t n_max, const int32_t* num_rows,
                          const float* boxes, int64_t box_img_stride, int32_t box_per_class,
                          const float* scores, int64_t score_img_stride, const float* score_factor,
                          int64_t sf_img_stride, int32_t sf_per_class, const uint8_t* row_valid,
                          int64_t valid_img_stride, const uint8_t* channel_mask, int32_t mode,
                          int32_t by_class, float min_score, void* workspace, size_t ws_bytes,
                          int32_t* info, void* stream);
size_t frh_mcnms_nms_workspace(int32_t num_imgs, int32_t num_classes, int32_t max_count, int64_t mask_tiles);
int32_t frh_mcnms_finish(int32_t num_imgs, int32_t num_classes, int64_t n_max, int32_t max_count,
                         int64_t mask_tiles, const float* boxes, int64_t box_img_stride, int32_t box_per_class,
                         const float* scores, int64_t score_img_stride, int32_t mode, int32_t by_class,
                         double nms_iou, int32_t max_num, float* out_boxes, float* out_scores,
                         int64_t* out_labels, int32_t* out_counts, int64_t out_cap, void* workspace,
                         size_t ws_bytes, void* nms_ws, size_t nms_ws_bytes, void* stream);

/* ---- a13/a14: BasicRoIExtractor.map_rois_to_levels + RoIAlign ----------------
 * level = clamp(floor(log2(sqrt((x2-x1+1)(y2-y1+1))/finest_scale + 1e-6)),
 * 0, L-1) (lib/region.py:256-264).  rois [K,5] = (batch_idx, x1, y1, x2, y2)
 * (torchvision convention).  roi_levels == nullptr => every roi on level 0.
 * RoIAlign = torchvision legacy aligned=False semantics (lib/builder.py:9,
 * used at lib/region.py:250-276); feats[l] is [B, C, H_l, W_l] NCHW
 * (layout 0) or NHWC (layout 1, i.e. channels_last strides); out [K, C, ph, pw]. */
int32_t frh_roi_level_map(const float* rois, int64_t num_rois, float finest_scale,
                          int32_t num_levels, int64_t* levels, void* stream);
/* The RoI rows the extractor feeds RoIAlign: rois [K, 5] = (image b, x1, y1, x2, y2) for the
 * boxes of num_segs images (<= 64) concatenated in image order (the reference attaches the
 * index per image, region.py:266-269, in its per-image forward, :303-306), and with
 * num_levels > 1 their levels as frh_roi_level_map computes them (region.py:256-264).  seg_offsets: HOST array [num_segs + 1] of row offsets
 * (0, n_0, n_0 + n_1, ...).  Boxes are [4, box_ld] coordinate-major: image b's box j at column
 * j of boxes + b * box_seg_stride, or (flat != 0) at column offsets[b] + j of boxes. */
int32_t frh_roi_rows(int32_t num_segs, const float* boxes, int64_t box_ld, int64_t box_seg_stride,
                     int32_t flat, const int64_t* seg_offsets, float finest_scale, int32_t num_levels,
                     float* rois, int64_t* levels, void* stream);
/* frh_roi_rows for rows of a fixed capacity whose per-image counts stay on the device
 * (seg_counts[b], image b's rows back to back from column 0 of boxes, images in order; rows
 * past their total are padding rows of image 0): the RCNN targets' buffer consumed without a
 * host synchronisation on its size (num_rows = the capacity). */
int32_t frh_roi_rows_dev(int32_t num_segs, const float* boxes, int64_t box_ld, int64_t num_rows,
                         const int32_t* seg_counts, float finest_scale, int32_t num_levels,
                         float* rois, int64_t* levels, void* stream);
int32_t frh_roi_align_fwd(int32_t num_levels, const float* const* feats, const int32_t* feat_hw,
                          const float* scales, int32_t batch, int32_t channels, int32_t layout,
                          const float* rois, const int64_t* roi_levels, int64_t num_rois,
                          int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio,
                          int32_t aligned, float* out, void* stream);
int32_t frh_roi_align_bwd(int32_t num_levels, float* const* grad_feats, const int32_t* feat_hw,
                          const float* scales, int32_t batch, int32_t channels, int32_t layout,
                          const float* rois, const int64_t* roi_levels, int64_t num_rois,
                          int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio,
                          int32_t aligned, const float* grad_out, void* stream);
/* Same ops with explicit per-level element strides strides[4l..4l+3] =
 * (batch, channel, y, x): any dense or strided feature view (NCHW,
 * channels_last, the FPN's P5[..., ::2, ::2] extra level). */
int32_t frh_roi_align_fwd_strided(int32_t num_levels, const float* const* feats,
                                  const int32_t* feat_hw, const int64_t* strides,
                                  const float* scales, int32_t batch, int32_t channels,
                                  const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                  int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio,
                                  int32_t aligned, float* out, void* stream);
/* Measurement entry (bench.py's roofline line): frh_roi_align_fwd_strided with the forward
 * kernel launched through hipExtLaunchKernel, which binds the two caller-created hipEvent_t
 * to the dispatch's own start and end timestamps (no extra stream packets).  span (nullable,
 * device, FRH_SPAN_SHARDS x FRH_SPAN_STRIDE u64, shard k's words {0, 1} initialised to
 * {UINT64_MAX, 0}): the kernel's own span on the GPU's 100 MHz s_memrealtime clock -- the
 * earliest wave start (min over shards of word 0) and the latest wave end (max of word 1);
 * one lane per wave records both with memory-side atomic min / max on its workgroup's shard. */
#define FRH_SPAN_SHARDS 256
#define FRH_SPAN_STRIDE 16
int32_t frh_roi_align_fwd_strided_timed(int32_t num_levels, const float* const* feats,
                                        const int32_t* feat_hw, const int64_t* strides,
                                        const float* scales, int32_t batch, int32_t channels,
                                        const float* rois, const int64_t* roi_levels,
                                        int64_t num_rois, int32_t pooled_h, int32_t pooled_w,
                                        int32_t sampling_ratio, int32_t aligned, float* out,
                                        void* start_event, void* stop_event, uint64_t* span,
                                        void* stream);
/* Backward of the strided forward: grad_feats (same strides) must be cleared by the
 * caller; contributions are added with float atomics (sampling 2, up to 8x8 bins:
 * one atomic per row run of a RoI's taps), so the summation order -- and the last
 * bits -- vary from run to run, as in torchvision's CUDA backward. */
int32_t frh_roi_align_bwd_strided(int32_t num_levels, float* const* grad_feats,
                                  const int32_t* feat_hw, const int64_t* strides,
                                  const float* scales, int32_t batch, int32_t channels,
                                  const float* rois, const int64_t* roi_levels, int64_t num_rois,
                                  int32_t pooled_h, int32_t pooled_w, int32_t sampling_ratio,
                                  int32_t aligned, const float* grad_out, void* stream);

/* Deterministic backward (parity runs; SURVEY §5 race detection): the gradient of
 * frh_roi_align_bwd_strided, accumulated in fixed point -- int64, each (RoI, row, column)
 * partial sum rounded once and added with integer atomics, which are associative -- so the
 * result is bit-identical across runs whatever order the RoIs are scheduled in (float atomics
 * reorder sums).  The unit is set per call from the gradient's own magnitude (ABI 3; was a
 * fixed 2^-40): 2^-(62 - hb - E) with max|grad_out| < 2^E and hb = ceil(log2(num_rois *
 * pooled_h * pooled_w)) -- the most any cell can receive is max|grad_out| * num_rois * bins, so
 * no accumulator can overflow, and the resolution is ~2^-(62 - hb) of the largest gradient
 * element (about 2^-46 at cfg2) whatever its scale.  A non-finite grad_out makes every
 * gradient element NaN.  acc_feats: per level an int64 buffer with the element strides of
 * grad_feats, zeroed by the caller; grad_feats (dense: every element is written) = acc * unit
 * rounded to f32.  scale_word: 4 bytes of caller-owned device memory (the call writes it: the
 * bits of max|grad_out|).  sampling_ratio 2 and up to 8 x 8 bins (the reference configs' 7 x 7). */
int32_t frh_roi_align_bwd_fixed(int32_t num_levels, float* const* grad_feats, int64_t* const* acc_feats,
                                const int32_t* feat_hw, const int64_t* strides, const float* scales,
                                int32_t batch, int32_t channels, const float* rois,
                                const int64_t* roi_levels, int64_t num_rois, int32_t pooled_h,
                                int32_t pooled_w, int32_t sampling_ratio, int32_t aligned,
                                const float* grad_out, uint32_t* scale_word, void* stream);

/* ---- RoIPool (torchvision.ops.RoIPool; C4 config configs/faster_rcnn_r50.py:26) --
 * feat [B, C, H, W] with element strides strides[0..3] = (b, c, y, x); rois
 * [K, 5]; out [K, C, ph, pw] + int32 argmax (flat y*W+x, -1 for empty bins). */
int32_t frh_roi_pool_fwd(const float* feat, const int64_t* strides, int32_t height, int32_t width,
                         int32_t channels, float spatial_scale, const float* rois, int64_t num_rois,
                         int32_t pooled_h, int32_t pooled_w, float* out, int32_t* argmax,
                         void* stream);
int32_t frh_roi_pool_bwd(float* grad_feat, const int64_t* strides, int32_t height, int32_t width,
                         int32_t channels, const float* rois, int64_t num_rois, int32_t pooled_h,
                         int32_t pooled_w, const float* grad_out, const int32_t* argmax, void* stream);

/* ---------------------------------------------------------------- a16 ATSS / LTRB targets
 * Replaces FCOSHead.single_image_targets_atss (lib/heads/fcos_head.py:283-368) with
 * topk_by_center (:106-116, row index by floor division), bbox2ltrb (:78-87),
 * positive_ltrb (:51-53), centerness (:56-59) and paint_value (:90-94), for all
 * images of a batch.  Levels: grid_hw[2l..2l+1] = (H_l, W_l), strides[l] (host arrays);
 * anchors [4, anchor_ld] f32 = one anchor per cell, levels concatenated (AnchorCreator
 * scale atss_cfg.scale, ratio 1).  gts [B][4][max_gts] f32 (segment stride gt_seg_stride),
 * num_gts [B] (device), gt_labels [B][max_gts] i64, img_hw [B][2] (device, img_shape h, w).
 * Outputs over the N level-concatenated cells: cls [B][N] i64 (-1 outside the painted
 * image, 0 background, label), reg [B][N][4] f32 ltrb (-1 when not positive),
 * ctr [B][N] f32 (-1 / 0 / centerness).  topk <= 16, num_levels <= 16.  Top-k ties
 * break by ascending cell index; the per-gt IoU mean / unbiased std use double sums. */
size_t frh_atss_workspace(int32_t batch, int32_t max_gts, int32_t num_levels, int32_t topk,
                          int64_t num_cells);
int32_t frh_atss_assign(int32_t batch, int32_t num_levels, const int32_t* grid_hw,
                        const float* strides, const float* anchors, int64_t anchor_ld,
                        const float* gts, int64_t gt_seg_stride, const int32_t* num_gts,
                        const int64_t* gt_labels, int32_t max_gts, const int32_t* img_hw,
                        int32_t topk, int64_t* cls, float* reg, float* ctr, void* workspace,
                        size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- backbone epilogue
 * Frozen BatchNorm (+ residual) (+ ReLU) of the reference ResNet's bottlenecks
 * (lib/backbones.py:69-76 keeps every BN in eval mode; torchvision Bottleneck.forward):
 * y = act(x * s + b (+ skip)), s = gamma / sqrt(var + eps), b = beta - mean * s, per
 * channel; x / skip / y contiguous NCHW f32 [n, c, hw], 16-byte aligned, hw % 4 == 0;
 * gamma / beta may be NULL (1 / 0); y may alias x. */
int32_t frh_bn_act(const float* x, const float* skip, float* y, const float* gamma,
                   const float* beta, const float* mean, const float* var, float eps,
                   int64_t n, int32_t c, int64_t hw, int32_t relu, void* stream);

/* The ResNet stem's frozen BN + ReLU + max_pool2d(kernel 3, stride 2, padding 1)
 * (lib/backbones.py, ResNet stem) in one pass: y [n, c, (h - 1) / 2 + 1, w / 2] =
 * maxpool(act(x * s + b)); x contiguous NCHW f32 [n, c, h, w], w % 8 == 0, x / y 16-byte
 * aligned.  Equal to frh_bn_act followed by the max pool, bit for bit. */
int32_t frh_bn_act_maxpool(const float* x, float* y, const float* gamma, const float* beta, const float* mean,
                           const float* var, float eps, int64_t n, int32_t c, int32_t h, int32_t w, void* stream);

/* FPN top-down merge into channels-last levels (lib/necks.py:72-84):
 * out[b, y, x, c] = (lat[b, c, y, x] + bias[c]) + up[b, iy, ix, c] with torch's nearest rule
 * (iy = min(floor(y * (float)up_h / height), up_h - 1); y / 2 when height == 2 * up_h);
 * lat: any strides (lat_strides = element strides b, c, y, x) -- the lateral conv's output
 * without its bias when bias ([channels]) is given, with it when bias is NULL; up: NHWC
 * contiguous [batch, up_h, up_w, channels] or NULL (the top level: a transpose); out: NHWC
 * contiguous [batch, height, width, channels].  f32 adds in that order (bit-identical to
 * the conv's bias add followed by the reference's upsample add). */
int32_t frh_fpn_merge_nhwc(const float* lat, const int64_t* lat_strides, const float* bias, const float* up,
                           int32_t up_h, int32_t up_w, float* out, int32_t batch, int32_t channels, int32_t height,
                           int32_t width, void* stream);

/* Conv epilogue on a channels-last map viewed as [rows, channels] (rows = batch * H * W):
 * y = relu ? max(y + bias[c], 0) : y + bias[c], in place -- the RPN head's
 * relu(conv(x)) (lib/heads/rpn_head.py, RPNHead.forward) after a bias-free NHWC conv, one
 * pass for PyTorch's bias add + ReLU.  channels % 4 == 0, y and bias 16-byte aligned. */
int32_t frh_bias_act_nhwc(float* y, const float* bias, int64_t rows, int32_t channels, int32_t relu, void* stream);

/* ---------------------------------------------------------------- f1: fused losses
 * Classification losses of lib/losses.py on the head outputs, summed (the reference's
 * reductions): kind 0 = sigmoid_focal_loss (losses.py:33-61, one-hot[:, 1:] targets),
 * 1 = CrossEntropyLoss(use_sigmoid=True) (losses.py:139-150; C == 1 takes the target
 * value itself, int64 or, with target_is_float, f32), 2 = CrossEntropyLoss softmax
 * (losses.py:151-153, labels in [0, C)).  Logit (i, k) is x[i*sr + k*sc] (any strides,
 * so AnchorHead's [C, S] targets need no transpose copy); out is one f32 on the device.
 * status (nullable, ABI 3): the device status word; while it is nonzero the forward writes NaN.
 * Backward writes grad_x (i, k) at grad_x[i*gsr + k*gsc] = grad_out[0] * dL/dx.  Rows with an
 * int64 label < 0 (padding rows of a fixed-capacity target buffer) add nothing, gradient 0.
 * Callers: AnchorHead.calc_loss (anchor_head.py:113-139), BBoxHead.calc_loss
 * (bbox_head.py:56-87), FCOSHead losses (fcos_head.py:418-534). */
/* Forward workspace: frh_loss_workspace() bytes whose first 256 bytes (the arrival counter of
 * the in-launch finalisation) are zero before the first call; every call leaves them zero, so
 * a caller zero-fills the buffer once and reuses it for calls ordered on one stream. */
size_t frh_loss_workspace(void);
int32_t frh_cls_loss_fwd(int32_t kind, const float* x, int64_t n, int64_t c, int64_t sr,
                         int64_t sc, const void* target, int32_t target_is_float, float alpha,
                         float gamma, const int32_t* status, float* out, void* workspace,
                         size_t ws_bytes, void* stream);
int32_t frh_cls_loss_bwd(int32_t kind, const float* x, int64_t n, int64_t c, int64_t sr,
                         int64_t sc, const void* target, int32_t target_is_float, float alpha,
                         float gamma, const float* grad_out, float* grad_x, int64_t gsr,
                         int64_t gsc, void* stream);
/* smooth_l1_loss_v2 (losses.py:77-83) summed over rows i < n, columns j < m of
 * x(i, j) = x[i*xs_i + j*xs_j + label[i]*xs_l] against y[i*ys_i + j*ys_j].  label (optional)
 * masks rows with label <= 0 -- the reference's positive-row selection
 * (anchor_head.py:126-128, bbox_head.py:71-76) -- and, with xs_l != 0, picks the labelled
 * class's deltas (reg_out.view(-1, 4, C)[arange, :, label], bbox_head.py:70-72); labels
 * >= n_sel make the sum NaN.  Backward writes only the selected unmasked elements of
 * grad_x (zero-filled by the caller). */
int32_t frh_smooth_l1_fwd(const float* x, int64_t xs_i, int64_t xs_j, int64_t xs_l,
                          const float* y, int64_t ys_i, int64_t ys_j, const int64_t* label,
                          int64_t n, int64_t m, int64_t n_sel, float beta, const int32_t* status,
                          float* out, void* workspace, size_t ws_bytes, void* stream);
int32_t frh_smooth_l1_bwd(const float* x, int64_t xs_i, int64_t xs_j, int64_t xs_l,
                          const float* y, int64_t ys_i, int64_t ys_j, const int64_t* label,
                          int64_t n, int64_t m, int64_t n_sel, float beta,
                          const float* grad_out, float* grad_x, int64_t gs_i, int64_t gs_j,
                          int64_t gs_l, void* stream);
/* One head's two losses in ONE launch, scaled as the heads scale them: out[0] =
 * (cls_sum * cls_weight) / cls_div, out[1] = (reg_sum * reg_weight) / reg_div (f32), cls_sum
 * as frh_cls_loss_fwd, reg_sum as frh_smooth_l1_fwd (both sums bit-identical to theirs).
 * Replaces `loss_cls(...) / avg_factor` and `loss_bbox.masked / class_selected(...) /
 * avg_factor` of AnchorHead.calc_loss (anchor_head.py:113-139) and BBoxHead.calc_loss
 * (bbox_head.py:56-87) with a sampler (avg_factor = the sample count, a host value).
 * Workspace as frh_cls_loss_fwd.  Backward: frh_cls_loss_bwd / frh_smooth_l1_bwd.
 * div_count (nullable): both divisors are this device int32 count instead (a fixed-capacity
 * target buffer consumed without a host sync; 0 gives zero losses, as the heads return). */
int32_t frh_det_loss_fwd(int32_t kind, const float* x, int64_t n, int64_t c, int64_t sr, int64_t sc,
                         const void* target, int32_t target_is_float, float alpha, float gamma,
                         float cls_weight, float cls_div, const float* rx, int64_t xs_i,
                         int64_t xs_j, int64_t xs_l, const float* ry, int64_t ys_i, int64_t ys_j,
                         const int64_t* label, int64_t rn, int64_t rm, int64_t n_sel, float beta,
                         float reg_weight, float reg_div, const int32_t* div_count,
                         const int32_t* status, float* out, void* workspace, size_t ws_bytes,
                         void* stream);

/* ---------------------------------------------------------------- f4: image pipeline
 * The train/test pipelines of configs/faster_rcnn_r50_fpn.py:120-139 (mmdet v1: Resize
 * keep_ratio -> RandomFlip -> Normalize -> Pad(size_divisor) -> DefaultFormatBundle ->
 * collate), fused: src holds uint8 HWC 3-channel images (image b at byte offset
 * src_offsets[b], size src_hw[2b..2b+1] = h, w; host arrays); each is resized to
 * dst_hw[b] with cv2.resize INTER_LINEAR's fixed-point arithmetic (exact 2x downscale:
 * INTER_AREA), flipped horizontally when flip[b] (may be NULL), normalised
 * (v - mean[c]) / std[c] in f32 (channels reversed first when to_rgb), and written to
 * dst [batch][3][out_h][out_w] f32 with zeros outside [0, dst_h) x [0, dst_w).  The host
 * side (lib-mirror frcnn_amd.datasets) computes the sizes, scale factors, box transforms
 * and img_meta exactly as mmcv/mmdet do. */
int32_t frh_image_preprocess(const uint8_t* src, int32_t batch, const int64_t* src_offsets,
                             const int32_t* src_hw, const int32_t* dst_hw, const int32_t* flip,
                             const float* mean, const float* std, int32_t to_rgb, float* dst,
                             int32_t out_h, int32_t out_w, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FRCNN_AMD_H */

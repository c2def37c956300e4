"""RCNN-stage proposal targets (reference lib/bbox.py:6-82) on the HIP kernels.

`bbox_targets_batched` runs every image at once: MaxIoU assignment of the
proposals, the reference's "prepend the gts as candidates" step
(bbox.py:27-29), sampling and the gather/encode of the chosen rows.
Per-image results come back as column slices of concatenated buffers, in
the reference's per-image row order.
"""
import torch

from . import ops


class PropBatch(list):
    """Per-image proposal views [4, n_i] that also expose the batched buffer
    [B, 4, cap] and the device counts they were cut from (RPN output), or the flat
    [4, sum n_i] buffer they are consecutive column slices of (RCNN targets)."""
    buffer = None
    counts_dev = None
    flat_buffer = None


class FlatList(list):
    """Per-image views that are consecutive slices (last dimension) of `flat`."""

    def __init__(self, flat):
        super().__init__()
        self.flat = flat


def _as_batch(props_list, dev):
    if isinstance(props_list, PropBatch) and props_list.buffer is not None:
        buf = props_list.buffer
        return buf, buf.stride(0), props_list.counts_dev, buf.shape[2]
    buf, counts, nmax = ops.pack_boxes([p.float() for p in props_list], dev)
    return buf, buf.stride(0), counts, nmax


def bbox_targets_batched(props_list, gt_bboxes, gt_labels, assigner, sampler, target_means=None,
                         target_stds=None, sync=True):
    """sync=False (device sampler mode): the flat full-capacity buffers of
    ops.bbox_target_batched(sync=False) -- padding columns past the device total, no
    per-image split -- with no host synchronisation on their size."""
    from .builder import build_module
    if isinstance(assigner, dict):
        assigner = build_module(assigner)
    if isinstance(sampler, dict):
        sampler = build_module(sampler)
    dev = gt_bboxes[0].device
    S = len(gt_bboxes)
    props, pstride, pcount, pmax = _as_batch(props_list, dev)
    gts, gcnt, gmax = ops.pack_boxes([g.float() for g in gt_bboxes], dev)
    glab = ops.pack_labels(gt_labels, gmax, dev)
    labels, _ = ops.maxiou_assign(props, pstride, pcount, pmax, gts, gcnt, gmax, assigner.pos_iou, assigner.neg_iou,
                                  assigner.min_pos_iou, num_segs=S)
    max_rows = gmax + pmax
    rows, num_rows = ops.prepend_gt_labels(labels, pcount, gcnt, max_rows)
    rows = ops.sample_labels(rows, num_rows, max_rows, sampler.max_num, sampler.pos_num,
                             lists=ops.sampler_mode() == 'device')
    r = ops.bbox_target_batched(rows, num_rows, gcnt, max_rows, props, pstride, gts, glab,
                                target_means, target_stds, sampler.max_num, sync=sync)
    if not sync:
        return r
    out = {k: FlatList(r[k]) for k in ('tar_bbox', 'tar_label', 'tar_param', 'tar_is_gt')}
    out['tar_props'] = PropBatch()
    out['tar_props'].flat_buffer = r['tar_props']  # [4, n]: the images' rows back to back
    off = 0
    for c in r['counts']:
        for k in out:
            v = r[k]
            out[k].append(v[..., off:off + c])
        off += c
    out['flat'] = r
    return out


def bbox_target(props, gt_bbox, gt_label, assigner, sampler, target_means=None, target_stds=None):
    """Single image, reference signature: (tar_props, tar_bbox, tar_label, tar_param, tar_is_gt)."""
    with torch.no_grad():
        r = bbox_targets_batched([props], [gt_bbox], [gt_label], assigner, sampler, target_means, target_stds)
    return (r['tar_props'][0], r['tar_bbox'][0], r['tar_label'][0], r['tar_param'][0], r['tar_is_gt'][0])

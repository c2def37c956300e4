"""Anchors and anchor targets (reference lib/anchor.py), on the HIP kernels.

`AnchorCreator` keeps the reference constructor/call contract
(`anchor.py:80-129`): anchor sizes are the f32 casts of float64
`base*s*sqrt(ar)`, the grid is generated on device by `frh_anchor_grid`.
`anchor_target` keeps the single-image contract of `anchor.py:11-76`; the
heads use the batched form (`anchor_targets_batched`) that runs every image
of the batch in one set of launches.
"""
import numpy as np
import torch

from . import ops


def anchor_sizes(base, scales, aspect_ratios):
    """(ws, hs) exactly as anchor.py:91-97 computes them (float64, then f32)."""
    ws, hs = [], []
    for s in scales:
        for ar in aspect_ratios:
            ws.append(base * s * np.sqrt(ar))
            hs.append(base * s / np.sqrt(ar))
    return (np.asarray(ws, dtype=np.float64).astype(np.float32).tolist(),
            np.asarray(hs, dtype=np.float64).astype(np.float32).tolist())


class AnchorCreator(object):
    def __init__(self, base=16, scales=(8, 16, 32), aspect_ratios=(0.5, 1.0, 2.0), center_lt=False,
                 device=torch.device('cpu')):
        self.device = torch.device(device)
        self.center_lt = center_lt
        self.base = base
        self.scales = list(scales)
        self.aspect_ratios = list(aspect_ratios)
        self.num_anchors = len(self.scales) * len(self.aspect_ratios)
        self.ws, self.hs = anchor_sizes(base, self.scales, self.aspect_ratios)
        self.anchor_ws = torch.tensor(self.ws, dtype=torch.float32)
        self.anchor_hs = torch.tensor(self.hs, dtype=torch.float32)

    def to(self, device):
        device = torch.device(device)
        if self.device == device:
            return True
        self.device = device
        self.anchor_ws = self.anchor_ws.to(device)
        self.anchor_hs = self.anchor_hs.to(device)

    def __call__(self, stride, grid):
        gh, gw = int(grid[0]), int(grid[1])
        dev = self.device if self.device.type == 'cuda' else torch.device('cuda', torch.cuda.current_device())
        flat = ops.anchor_grid([(gh, gw)], [float(stride)], self.ws, self.hs, self.num_anchors, self.center_lt, dev)
        return flat.reshape(4, self.num_anchors, gh, gw)


def in_grid_sizes(img_size, grid_sizes, strides):
    """inside_grid_mask's visible grid per level, in Python double (region.py:11-13)."""
    out = []
    for (gh, gw), s in zip(grid_sizes, strides):
        r = 1.0 / s
        out.append((min(int(gh), int(img_size[0] * r) + 1), min(int(gw), int(img_size[1] * r) + 1)))
    return out


def anchor_targets_batched(labels, num_boxes, max_boxes, anchors, gts, gt_labels, sampler, means, stds, sync=True):
    """Sample (optional) + gather/encode for all images: the per-image anchor_target
    results concatenated in image order (anchor_head.py:177-192)."""
    if sampler is not None:  # device mode: the sampler's lists feed the gather (no compaction pass)
        labels = ops.sample_labels(labels, num_boxes, max_boxes, sampler.max_num, sampler.pos_num,
                                   lists=ops.sampler_mode() == 'device')
        cap = sampler.max_num
    else:
        cap = max_boxes
    return ops.anchor_target_batched(labels, num_boxes, max_boxes, anchors, gts, gt_labels, means, stds, cap,
                                     sync=sync)


def anchor_target(cls_out, reg_out, cls_channels, in_anchors, in_mask, gt_bbox, gt_label=None, assigner=None,
                  sampler=None, target_means=None, target_stds=None):
    """Single-image anchor_target with the reference signature (anchor.py:11-76)."""
    if assigner is None:
        raise AssertionError('assigner is required')
    from .builder import build_module
    if isinstance(assigner, dict):
        assigner = build_module(assigner)
    if isinstance(sampler, dict):
        sampler = build_module(sampler)
    dev = in_anchors.device
    in_anchors = in_anchors.float().contiguous()
    gts, gcnt, gmax = ops.pack_boxes([gt_bbox.float()], dev)
    n = in_anchors.shape[1]
    num = torch.tensor([n], dtype=torch.int32, device=dev)
    labels, _ = ops.maxiou_assign(in_anchors, 0, num, n, gts, gcnt, gmax, assigner.pos_iou, assigner.neg_iou,
                                  assigner.min_pos_iou)
    gl = ops.pack_labels([gt_label], gmax, dev) if gt_label is not None else None
    r = anchor_targets_batched(labels, num, n, in_anchors, gts, gl, sampler, target_means, target_stds)
    full_idx = torch.nonzero(in_mask.view(-1)).view(-1)[r['chosen_idx']]
    cls_out_ = cls_out.view(cls_channels, -1)
    reg_out_ = reg_out.view(4, -1)
    return (cls_out_[:, full_idx], reg_out_[:, full_idx], r['tar_labels'], r['tar_anchors'], r['tar_bbox'],
            r['tar_param'])

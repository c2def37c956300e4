"""Masks, MaxIoU assignment, random sampling and the FPN RoI extractor
(reference lib/region.py) on the HIP kernels."""
import torch
from torch import nn

from . import ops
from .utils import to_pair


def inside_grid_mask(num_anchors, img_size, grid_size, stride, device=None):
    """region.py:10-16: float [A*H*W] flags of the grid cells inside the image."""
    gh, gw = int(grid_size[0]), int(grid_size[1])
    r = 1.0 / stride
    ih, iw = min(gh, int(img_size[0] * r) + 1), min(gw, int(img_size[1] * r) + 1)
    dev = device if device is not None and torch.device(device).type == 'cuda' else torch.device('cuda')
    dummy = torch.empty(4, 1, dtype=torch.float32, device=dev)
    m = ops.inside_mask(dummy, [(gh, gw)], [(ih, iw)], num_anchors, 0, 0, -1)
    return m.float()


def inside_anchor_mask(anchors, img_size, allowed_border=0):
    """region.py:19-29: bool [n], anchors fully inside the image (+border)."""
    n = anchors.shape[1]
    if allowed_border < 0:
        return torch.ones(n, dtype=torch.bool, device=anchors.device)
    a = anchors.float()
    if a.stride(1) != 1:
        a = a.contiguous()
    m = ops.inside_mask(a, [(1, n)], [(1, n)], 1, img_size[0], img_size[1], allowed_border)
    return m.bool()


class MaxIoUAssigner(object):
    """region.py:60-107.  labels: -1 ignore, 0 negative, g+1 positive; plus max IoU."""

    def __init__(self, pos_iou, neg_iou, min_pos_iou):
        self.pos_iou = pos_iou
        self.neg_iou = neg_iou
        self.min_pos_iou = min_pos_iou

    def __call__(self, bboxes, gt_bboxes):
        if bboxes.shape[0] != 4 or gt_bboxes.shape[0] != 4:
            raise AssertionError('boxes must be [4, n]')
        if gt_bboxes.shape[1] == 0:
            # torch.max over an empty dim raises in the reference (region.py:86)
            raise RuntimeError('MaxIoUAssigner: no gt boxes')
        dev = bboxes.device
        b = bboxes.float()
        if b.stride(1) != 1:
            b = b.contiguous()
        n = b.shape[1]
        gts, gcnt, gmax = ops.pack_boxes([gt_bboxes.float()], dev)
        num = torch.tensor([n], dtype=torch.int32, device=dev)
        labels, max_iou = ops.maxiou_assign(b, 0, num, n, gts, gcnt, gmax, self.pos_iou, self.neg_iou,
                                            self.min_pos_iou)
        return labels[0, :n], max_iou[0, :n]


def random_sample_label(labels, pos_num, tot_num):
    """region.py:43-57 (labels of 1/0/-1, sampled in place as in the reference)."""
    if pos_num > tot_num:
        raise AssertionError('pos_num > tot_num')
    n = labels.numel()
    num = torch.tensor([n], dtype=torch.int32, device=labels.device)
    out = ops.sample_labels(labels.view(1, n).long(), num, n, tot_num, pos_num)
    labels.copy_(out.view(-1).to(labels.dtype))
    return labels


class RandomSampler(object):
    """region.py:112-126: keep <= pos_num positives, fill to max_num with negatives."""

    def __init__(self, max_num, pos_num):
        if pos_num > max_num:
            raise AssertionError('pos_num > max_num')
        self.max_num = max_num
        self.pos_num = pos_num

    def __call__(self, labels, overlaps_iou=None, props_bbox=None, gt_bbox=None):
        n = labels.numel()
        num = torch.tensor([n], dtype=torch.int32, device=labels.device)
        out = ops.sample_labels(labels.view(1, n).long(), num, n, self.max_num, self.pos_num)
        return out.view(-1).to(labels.dtype)


class RoiBatch(list):
    """Per-image RoI feature list that also carries the contiguous [sum K, C, ph, pw]
    tensor the views come from (lets the RCNN head skip a torch.cat)."""
    flat = None


class BasicRoIExtractor(nn.Module):
    """region.py:243-306: FPN level mapping + RoIAlign, all images and levels in one launch."""

    def __init__(self, roi_layers, output_size=(7, 7), finest_scale=56):
        super().__init__()
        if not isinstance(roi_layers, list):
            raise AssertionError('roi_layers must be a list')
        from .builder import build_module
        self.output_size = to_pair(output_size)
        self.finest_scale = finest_scale
        layers = []
        for cfg in roi_layers:
            cfg = dict(cfg)
            cfg['output_size'] = output_size
            layers.append(build_module(cfg))
        self.roi_layers = layers

    def map_rois_to_levels(self, rois, num_lvls):
        """rois [4, K] -> level per roi (region.py:256-264)."""
        r5 = torch.cat([rois.new_zeros(1, rois.shape[1]), rois.float()], 0).t().contiguous()
        return ops.roi_level_map(r5, self.finest_scale, num_lvls)

    def _fusable(self):
        from .ops import RoIAlign
        first = self.roi_layers[0]
        return all(isinstance(l, RoIAlign) and l.sampling_ratio == first.sampling_ratio and
                   l.aligned == first.aligned and l.output_size == first.output_size for l in self.roi_layers)

    def forward(self, level_feats, rois_list):
        n_lvls = len(self.roi_layers)
        if not (0 < n_lvls <= len(level_feats)):
            raise AssertionError('not enough feature levels')
        counts = [int(r.shape[1]) for r in rois_list]
        dev = level_feats[0].device
        if self._fusable():
            rois, levels = self._rows(rois_list, counts, n_lvls, dev)
            first = self.roi_layers[0]
            out = ops.roi_align_multilevel(list(level_feats[:n_lvls]), rois, levels,
                                           [l.spatial_scale for l in self.roi_layers], first.output_size,
                                           first.sampling_ratio, first.aligned)
        else:
            out = self._forward_per_level(level_feats, rois_list, counts)
        res = RoiBatch()
        off = 0
        for c in counts:
            res.append(out[off:off + c])
            off += c
        res.flat = out
        return res

    def forward_flat(self, level_feats, boxes, counts_dev):
        """forward over a fixed-capacity flat box buffer [4, K] whose per-image counts stay
        on the device (the sync-free RCNN targets): [K, C, ph, pw] for all K rows, the rows
        past the total being padding (image 0, zero box)."""
        n_lvls = len(self.roi_layers)
        if not (0 < n_lvls <= len(level_feats)) or not self._fusable():
            raise AssertionError('forward_flat needs RoIAlign layers of one configuration')
        if not 0 < counts_dev.numel() <= 64:
            raise AssertionError('forward_flat takes 1..64 images')
        rois, levels = ops.roi_rows_dev(boxes, counts_dev, self.finest_scale, n_lvls)
        first = self.roi_layers[0]
        return ops.roi_align_multilevel(list(level_feats[:n_lvls]), rois, levels,
                                        [l.spatial_scale for l in self.roi_layers], first.output_size,
                                        first.sampling_ratio, first.aligned)

    def _rows(self, rois_list, counts, n_lvls, dev):
        """(image, box) rows + levels in one kernel (frh_roi_rows), reading the RCNN targets'
        flat buffer or the RPN's batched proposal buffer in place when the list carries one."""
        if not 0 < len(counts) <= 64:
            boxes = torch.cat([r.float() for r in rois_list], 1) if rois_list else torch.zeros(4, 0, device=dev)
            bidx = torch.repeat_interleave(torch.arange(len(counts), device=dev, dtype=torch.float32),
                                           ops.device_ints(counts, dev, torch.int64), output_size=sum(counts))
            rois = torch.cat([bidx.view(1, -1), boxes], 0).t().contiguous()
            return rois, (ops.roi_level_map(rois, self.finest_scale, n_lvls) if n_lvls > 1 else None)
        flat = getattr(rois_list, 'flat_buffer', None)
        if flat is not None and flat.dtype == torch.float32:
            return ops.roi_rows(flat, counts, self.finest_scale, n_lvls)
        buf = getattr(rois_list, 'buffer', None)
        if buf is not None and buf.dtype == torch.float32 and buf.dim() == 3:
            return ops.roi_rows(buf, counts, self.finest_scale, n_lvls, seg_stride=buf.stride(0), flat=False)
        return ops.roi_rows(torch.cat([r.float() for r in rois_list], 1), counts, self.finest_scale, n_lvls)

    def _forward_per_level(self, level_feats, rois_list, counts):
        # generic path for non-RoIAlign layers (e.g. RoIPool): per level, all images at once
        n_lvls = len(self.roi_layers)
        dev = level_feats[0].device
        boxes = torch.cat([r.float() for r in rois_list], 1)
        bidx = torch.repeat_interleave(torch.arange(len(counts), device=dev, dtype=torch.float32),
                                       ops.device_ints(counts, dev, torch.int64), output_size=sum(counts))
        rois = torch.cat([bidx.view(1, -1), boxes], 0).t().contiguous()
        C = level_feats[0].shape[1]
        out = level_feats[0].new_zeros((rois.shape[0], C) + tuple(self.output_size))
        lv = ops.roi_level_map(rois, self.finest_scale, n_lvls) if n_lvls > 1 else None
        for i in range(n_lvls):
            sel = (lv == i).nonzero().view(-1) if lv is not None else torch.arange(rois.shape[0], device=dev)
            if sel.numel():
                out[sel] = self.roi_layers[i](level_feats[i], rois[sel])
        return out

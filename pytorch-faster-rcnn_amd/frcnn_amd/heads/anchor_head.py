"""AnchorHead (reference lib/heads/anchor_head.py) with a batched target path.

The reference loops over images in Python (anchor_head.py:177-187) and over
levels inside each image; here one set of launches covers the whole batch:
cached all-level anchors [4, N], cached inside masks [B, N], one fused
MaxIoU assignment over (images x anchors), one sampling launch (or the
numpy-parity host round trip), one gather/encode launch, then the per-level
head outputs are gathered at the chosen anchors by an autograd-aware HIP
gather.  Results equal the reference's per-image targets concatenated in
image order.
"""
import logging
from collections import OrderedDict

import torch
from torch import nn

from .. import ops, utils, losses
from ..utils import ChannelsLastConvs
from ..anchor import AnchorCreator, in_grid_sizes, anchor_targets_batched
from ..region import MaxIoUAssigner


class AnchorHead(ChannelsLastConvs):
    def __init__(self, num_classes, anchor_scales=(8,), anchor_ratios=(0.5, 1.0, 2.0),
                 anchor_strides=(4, 8, 16, 32, 64), anchor_center_lt=False, target_means=(0.0, 0.0, 0.0, 0.0),
                 target_stds=(1.0, 1.0, 1.0, 1.0), loss_cls=None, loss_bbox=None):
        super().__init__()
        from ..builder import build_module
        self.num_classes = num_classes
        self.anchor_scales = list(anchor_scales)
        self.anchor_ratios = list(anchor_ratios)
        self.anchor_strides = list(anchor_strides)
        self.anchor_base_sizes = list(anchor_strides)
        self.anchor_center_lt = anchor_center_lt
        self.anchor_creators = [AnchorCreator(base=b, scales=self.anchor_scales, aspect_ratios=self.anchor_ratios,
                                              center_lt=anchor_center_lt) for b in self.anchor_strides]
        self.num_anchors = len(self.anchor_scales) * len(self.anchor_ratios)
        self.target_means = list(target_means)
        self.target_stds = list(target_stds)
        self.loss_cls = build_module(loss_cls) if isinstance(loss_cls, dict) else loss_cls
        self.loss_bbox = build_module(loss_bbox) if isinstance(loss_bbox, dict) else loss_bbox
        self.use_sigmoid = self.loss_cls.use_sigmoid
        self.cls_channels = num_classes - 1 if self.use_sigmoid else num_classes
        self._anchor_cache = {}
        self._mask_cache = OrderedDict()  # LRU: keep-ratio resizing makes many image shapes
        self.allow_sync_free = True  # False: keep the synced (read-back) targets even with the device sampler

    # ------------------------------------------------------------ anchors
    def _flat_anchors(self, grid_sizes, device):
        key = (tuple((int(h), int(w)) for h, w in grid_sizes), str(device))
        a = self._anchor_cache.get(key)
        if a is None:
            ws = [v for c in self.anchor_creators for v in c.ws]
            hs = [v for c in self.anchor_creators for v in c.hs]
            a = ops.anchor_grid(key[0], [float(s) for s in self.anchor_strides], ws, hs, self.num_anchors,
                                self.anchor_center_lt, device)
            self._anchor_cache[key] = a
        return a

    def create_anchors(self, grid_sizes):
        """Per-level [4, A, H, W] anchors (anchor_head.py:66-67), views of the cached flat grid."""
        flat = self._flat_anchors(grid_sizes, torch.device('cuda', torch.cuda.current_device()))
        out, off = [], 0
        for h, w in grid_sizes:
            n = self.num_anchors * int(h) * int(w)
            out.append(flat[:, off:off + n].reshape(4, self.num_anchors, int(h), int(w)))
            off += n
        return out

    MASK_CACHE_MAX = 64  # per-image masks, batch stacks and count tensors (LRU)

    def _cached(self, key, make):
        c = self._mask_cache
        v = c.get(key)
        if v is None:
            v = c[key] = make()
            while len(c) > self.MASK_CACHE_MAX:
                c.popitem(last=False)
        else:
            c.move_to_end(key)
        return v

    def _valid_masks(self, anchors, grid_sizes, img_metas, allowed_border):
        grids = tuple((int(h), int(w)) for h, w in grid_sizes)
        masks = []
        for m in img_metas:
            img = tuple(int(v) for v in m['img_shape'][:2])
            key = (grids, img, int(allowed_border), anchors.data_ptr())
            masks.append((key, self._cached(key, lambda: ops.inside_mask(
                anchors, grid_sizes, in_grid_sizes(img, grid_sizes, self.anchor_strides), self.num_anchors, img[0],
                img[1], allowed_border))))
        # the [B, N] stack of the batch's image shapes (cached too: a fixed-shape batch repeats it)
        return self._cached(('batch',) + tuple(k for k, _ in masks), lambda: torch.stack([v for _, v in masks]))

    # ------------------------------------------------------------ targets
    def targets_batched(self, cls_outs, reg_outs, gt_bboxes, gt_labels, img_metas, train_cfg):
        """(tar_cls_out [C, T], tar_reg_out [4, T], tar_labels [T], tar_param [4, T]) for the batch."""
        return self._targets(cls_outs, reg_outs, gt_bboxes, gt_labels, img_metas, train_cfg)[:4]

    def sync_free(self, train_cfg, device):
        """Whether the loss can consume the targets without reading their size back to the
        host: the device sampler's lists, fixed capacity S * max_num with padding columns,
        and the fused head losses dividing by the device count (= len(tar_labels), the
        reference's sampled avg_factor, anchor_head.py:123-126)."""
        return (self.allow_sync_free and device.type == 'cuda' and train_cfg.get('sampler', None) is not None and
                ops.sampler_mode() == 'device' and losses.fused_kinds(self.loss_cls, self.loss_bbox))

    def _targets(self, cls_outs, reg_outs, gt_bboxes, gt_labels, img_metas, train_cfg, sync=True):
        dev = cls_outs[0].device
        grid_sizes = [tuple(c.shape[-2:]) for c in cls_outs]
        anchors = self._flat_anchors(grid_sizes, dev)
        masks = self._valid_masks(anchors, grid_sizes, img_metas, train_cfg.allowed_border)
        B, N = masks.shape
        assigner = train_cfg.assigner
        if isinstance(assigner, dict):
            from ..builder import build_module
            assigner = build_module(assigner)
        sampler = train_cfg.get('sampler', None)
        if isinstance(sampler, dict):
            from ..builder import build_module
            sampler = build_module(sampler)
        gts, gcnt, gmax = ops.pack_boxes([g.float() for g in gt_bboxes], dev)
        glab = ops.pack_labels(gt_labels, gmax, dev) if gt_labels is not None else None
        num = self._cached(('num', B, N, dev), lambda: torch.full((B,), N, dtype=torch.int32, device=dev))
        labels, _ = ops.maxiou_assign(anchors, 0, num, N, gts, gcnt, gmax, assigner.pos_iou, assigner.neg_iou,
                                      assigner.min_pos_iou, valid=masks, valid_seg_stride=masks.stride(0))
        r = anchor_targets_batched(labels, num, N, anchors, gts, glab, sampler, self.target_means,
                                   self.target_stds, sync=sync)
        tar_cls = ops.gather_level_outputs(cls_outs, r['chosen_idx'], r['seg_of'], self.cls_channels)
        tar_reg = ops.gather_level_outputs(reg_outs, r['chosen_idx'], r['seg_of'], 4)
        return tar_cls, tar_reg, r['tar_labels'], r['tar_param'], r.get('n_dev')

    def single_image_targets(self, level_cls_outs, level_reg_outs, gt_bbox, gt_label, level_anchors, input_size,
                             grid_sizes, img_meta, train_cfg):
        """Reference per-image entry (anchor_head.py:69-111), via the batched path with B = 1."""
        return self.targets_batched([c.unsqueeze(0) for c in level_cls_outs], [r.unsqueeze(0) for r in level_reg_outs],
                                    [gt_bbox], [gt_label] if gt_label is not None else None, [img_meta], train_cfg)

    def calc_loss(self, tar_cls_out, tar_reg_out, tar_labels, tar_param, train_cfg):
        """anchor_head.py:113-139.  The regression loss over the positive columns is
        computed as a masked sum (zeroed negative columns contribute exactly 0 to the
        reference's sum-reduced losses), which avoids the host synchronisation of
        boolean indexing; with no positives it is 0 as in the reference."""
        dev = tar_cls_out.device
        cls_loss, reg_loss = losses.zero_loss(dev), losses.zero_loss(dev)
        sampling = 'sampler' in train_cfg
        avg_factor = len(tar_labels) if sampling else (tar_labels > 0).sum()
        if tar_labels.numel() != 0:
            # both losses and their scaling in one launch (HIP losses, sampled avg_factor)
            fused = losses.head_losses(self.loss_cls, self.loss_bbox, tar_cls_out.t(), tar_labels,
                                       lambda: ops._l1_args(tar_reg_out, tar_param, tar_labels, 1), avg_factor)
            if fused is not None:
                return fused
            cls_loss = self.loss_cls(tar_cls_out.t(), tar_labels) / avg_factor
            if isinstance(self.loss_bbox, losses.SmoothL1Loss):
                # fused masked smooth-L1 over the positive columns of [4, S] (one kernel, no sync)
                reg_loss = self.loss_bbox.masked(tar_reg_out, tar_param, tar_labels, rows_dim=1) / avg_factor
            else:
                m = (tar_labels > 0).view(1, -1)
                z = tar_reg_out.new_zeros(())
                reg_loss = self.loss_bbox(torch.where(m, tar_reg_out, z), torch.where(m, tar_param, z)) / avg_factor
        else:
            logging.warning('%s recieved no samples to train, return dummy zero losses', type(self).__name__)
        return cls_loss, reg_loss

    def loss(self, cls_outs, reg_outs, gt_bboxes, gt_labels, img_metas, train_cfg):
        if self.sync_free(train_cfg, cls_outs[0].device):
            # padded targets + device count: no host synchronisation between the sampler and the loss
            tc, tr, tl, tp, n_dev = self._targets(cls_outs, reg_outs, gt_bboxes, gt_labels, img_metas, train_cfg,
                                                  sync=False)
            return losses.head_losses(self.loss_cls, self.loss_bbox, tc.t(), tl,
                                      lambda: ops._l1_args(tr, tp, tl, 1), None, div_count=n_dev)
        tc, tr, tl, tp = self.targets_batched(cls_outs, reg_outs, gt_bboxes, gt_labels, img_metas, train_cfg)
        return self.calc_loss(tc, tr, tl, tp, train_cfg)

    def forward_train(self, feats, gt_bboxes, gt_labels, img_metas, train_cfg):
        cls_outs, reg_outs = self.forward(feats)
        return self.loss(cls_outs, reg_outs, gt_bboxes, gt_labels, img_metas, train_cfg)

    # ------------------------------------------------------------ inference (multi-class heads)
    def image_candidates(self, level_cls_outs, level_reg_outs, level_anchors, img_meta, test_cfg):
        """anchor_head.py:215-249 for one image: per-level top-k by the best class score,
        decode + clamp.  Returns scores [C, n], boxes [4, n] and the min-size mask [n] (or
        None) -- rows the reference drops stay in place, masked (no host sync)."""
        cls_outs = [c.reshape(self.cls_channels, -1) for c in level_cls_outs]
        reg_outs = [r.reshape(4, -1) for r in level_reg_outs]
        anchors = [a.reshape(4, -1) for a in level_anchors]
        img_size = img_meta['img_shape'][:2]
        min_size = img_meta['scale_factor'] * test_cfg.min_bbox_size
        scores, boxes = [], []
        for co, ro, an in zip(cls_outs, reg_outs, anchors):
            sc = co.sigmoid() if self.use_sigmoid else co.softmax(dim=0)
            if 0 < test_cfg.pre_nms < sc.shape[1]:
                mx = sc.max(0)[0] if self.use_sigmoid else sc[1:, :].max(0)[0]
                _, idx = mx.topk(test_cfg.pre_nms)
                sc, ro, an = sc[:, idx], ro[:, idx], an[:, idx]
            scores.append(sc)
            boxes.append(utils.param2bbox(an, ro, self.target_means, self.target_stds, img_size))
        sc, bx = torch.cat(scores, 1), torch.cat(boxes, 1)
        valid = None
        if min_size > 0:
            valid = ((bx[2] - bx[0] + 1) >= min_size) & ((bx[3] - bx[1] + 1) >= min_size)
        return sc, bx, valid

    def _nms_labels(self):
        if self.use_sigmoid:
            return list(range(0, self.num_classes - 1)), 1
        return list(range(1, self.num_classes)), 0

    def predict_single_image(self, level_cls_outs, level_reg_outs, level_anchors, img_meta, test_cfg):
        """anchor_head.py:207-262: per-level top-k, decode, min-size filter, multiclass NMS."""
        return [x[0] for x in self._predict_batch([self.image_candidates(level_cls_outs, level_reg_outs,
                                                                         level_anchors, img_meta, test_cfg)],
                                                  test_cfg)]

    def _predict_batch(self, cands, test_cfg):
        """One class-wise batched multiclass NMS (csrc/mcnms.hip) over the images' candidates
        (every image has the same row count: the per-level top-k sizes)."""
        labels, adjust = self._nms_labels()
        scores = torch.stack([sc.t() for sc, _, _ in cands])
        boxes = torch.stack([bx.t() for _, bx, _ in cands])
        valid = None
        if any(v is not None for _, _, v in cands):
            valid = torch.stack([v if v is not None else torch.ones_like(sc[0], dtype=torch.bool)
                                 for sc, _, v in cands])
        res = ops.multiclass_nms_batched(boxes, scores, labels, test_cfg.nms_iou, test_cfg.min_score,
                                         test_cfg.max_per_img, mode=test_cfg.get('nms_type', 'official'),
                                         row_valid=valid)
        return [[kb.t() for kb, _, _ in res], [ks for _, ks, _ in res], [kl + adjust for _, _, kl in res]]

    def predict_bboxes(self, feats, img_metas, test_cfg):
        cls_outs, reg_outs = self.forward(feats)
        return self.predict_bboxes_from_output(cls_outs, reg_outs, img_metas, test_cfg)

    def predict_bboxes_from_output(self, cls_outs, reg_outs, img_metas, test_cfg):
        """anchor_head.py:264-289 batched over the images: per-image candidates (device
        ops, no sync), then ONE multiclass NMS launch sequence for all images."""
        grid_sizes = [tuple(c.shape[-2:]) for c in cls_outs]
        level_anchors = self.create_anchors(grid_sizes)
        cands = [self.image_candidates([c[i] for c in cls_outs], [r[i] for r in reg_outs], level_anchors, meta,
                                       test_cfg) for i, meta in enumerate(img_metas)]
        return self._predict_batch(cands, test_cfg)

    def to(self, *args, **kwargs):
        return super().to(*args, **kwargs)

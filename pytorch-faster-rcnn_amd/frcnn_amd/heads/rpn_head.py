"""RPNHead (reference lib/heads/rpn_head.py).

Convs stay on PyTorch-ROCm.  `predict_bboxes_from_output` runs the whole
proposal stage (rpn_head.py:68-120: per-level score top-k, decode + clamp,
min-size filter, NMS, post_nms cut, cross-level top-k) for every image and
level in one `frh_rpn_proposals` call, with no host synchronisation: the
per-image proposal tensors are materialised lazily.
"""
import logging

import torch
from torch import nn

from .. import ops
from ..bbox import PropBatch
from ..utils import init_module_normal
from .anchor_head import AnchorHead


class LazyPropList(PropBatch):
    """List of per-image proposals [4, n_i] cut from the batched RPN buffer.

    Items (and their data-dependent shapes) are materialised on first list
    access; batched consumers read `buffer` / `counts_dev` and never sync."""

    def __init__(self, buffer, counts_dev, what='boxes'):
        super().__init__()
        self.buffer = buffer
        self.counts_dev = counts_dev
        self._what = what
        self._n = buffer.shape[0]
        self._done = False

    def _materialise(self):
        if not self._done:
            self._done = True
            counts = self.counts_dev.cpu().tolist()
            for b, c in enumerate(counts):
                list.append(self, self.buffer[b, :, :c] if self._what == 'boxes' else self.buffer[b, :c])

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        self._materialise()
        return list.__getitem__(self, i)

    def __iter__(self):
        self._materialise()
        return list.__iter__(self)

    def __repr__(self):
        self._materialise()
        return list.__repr__(self)


class RPNHead(AnchorHead):
    def __init__(self, in_channels, feat_channels, anchor_scales=(8,), anchor_ratios=(0.5, 1.0, 2.0),
                 anchor_strides=(4, 8, 16, 32, 64), anchor_center_lt=False, target_means=(0.0, 0.0, 0.0, 0.0),
                 target_stds=(1.0, 1.0, 1.0, 1.0), loss_cls=None, loss_bbox=None):
        self.in_channels = in_channels
        self.feat_channels = feat_channels
        super().__init__(num_classes=2, anchor_scales=anchor_scales, anchor_ratios=anchor_ratios,
                         anchor_strides=anchor_strides, anchor_center_lt=anchor_center_lt,
                         target_means=target_means, target_stds=target_stds, loss_cls=loss_cls,
                         loss_bbox=loss_bbox)
        self.init_layers()

    def init_layers(self):
        self.conv = nn.Conv2d(self.in_channels, self.feat_channels, kernel_size=3, stride=1, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.classifier = nn.Conv2d(self.feat_channels, self.num_anchors * self.cls_channels, kernel_size=1)
        self.regressor = nn.Conv2d(self.feat_channels, self.num_anchors * 4, kernel_size=1)

    def init_weights(self):
        for m in (self.conv, self.classifier, self.regressor):
            init_module_normal(m, mean=0.0, std=0.01)

    def forward(self, xs):
        # relu(conv(x)); on channels-last HIP levels the bias add + ReLU is one pass (ops.conv_bias_relu)
        hidden = [ops.conv_bias_relu(self.conv, x) for x in xs]
        return [self.classifier(h) for h in hidden], [self.regressor(h) for h in hidden]

    def predict_bboxes_from_output(self, cls_outs, reg_outs, img_metas, test_cfg):
        """Returns [props, scores, labels] lists like unpack_multi_result of
        predict_single_image (rpn_head.py:68-120); props/scores are lazy."""
        with torch.no_grad():
            dev = cls_outs[0].device
            grid_sizes = [tuple(c.shape[-2:]) for c in cls_outs]
            anchors = self._flat_anchors(grid_sizes, dev)
            img_hw = [tuple(float(v) for v in m['img_shape'][:2]) for m in img_metas]
            min_sizes = [float(m['scale_factor'] * test_cfg.min_bbox_size) for m in img_metas]
            boxes, scores, counts = ops.rpn_proposals(
                [c.detach() for c in cls_outs], [r.detach() for r in reg_outs], anchors, self.num_anchors,
                self.cls_channels, self.target_means, self.target_stds, img_hw, min_sizes, int(test_cfg.pre_nms),
                int(test_cfg.post_nms), int(test_cfg.max_num), float(test_cfg.nms_iou))
        props = LazyPropList(boxes, counts, 'boxes')
        scs = LazyPropList(scores, counts, 'scores')
        return [props, scs, [None] * len(img_metas)]

    def predict_single_image(self, level_cls_outs, level_reg_outs, level_anchors, img_meta, test_cfg):
        p, s, _ = self.predict_bboxes_from_output([c.unsqueeze(0) for c in level_cls_outs],
                                                  [r.unsqueeze(0) for r in level_reg_outs], [img_meta], test_cfg)
        return p[0], s[0], None

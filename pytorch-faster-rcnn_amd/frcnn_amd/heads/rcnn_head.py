"""RCNNHead (reference lib/heads/rcnn_head.py): shared FCs + cls/reg FCs.

Dense GEMMs stay on PyTorch-ROCm (hipBLASLt).  Takes the RoI extractor's
batch tensor directly when available instead of re-concatenating the
per-image views.
"""
from torch import nn
import torch

from ..utils import init_module_normal, to_pair
from .bbox_head import BBoxHead, HeadOutputs


class RCNNHead(BBoxHead):
    def __init__(self, in_channels, roi_out_size=7, with_avg_pool=False, fc_channels=(1024, 1024), num_classes=21,
                 target_means=(0.0, 0.0, 0.0, 0.0), target_stds=(0.1, 0.1, 0.2, 0.2), reg_class_agnostic=False,
                 loss_cls=None, loss_bbox=None):
        super().__init__(num_classes, target_means, target_stds, reg_class_agnostic, loss_cls, loss_bbox)
        self.in_channels = in_channels
        self.roi_out_size = to_pair(roi_out_size)
        self.with_avg_pool = with_avg_pool
        self.fc_channels = list(fc_channels) if fc_channels else []
        self.init_layers()

    def init_layers(self):
        ch = self.in_channels
        spatial = self.roi_out_size[0] * self.roi_out_size[1]
        if self.with_avg_pool:
            self.avg_pool = nn.AvgPool2d(self.roi_out_size)
            spatial = 1
        self.with_shared_fcs = bool(self.fc_channels)
        if self.with_shared_fcs:
            layers = []
            for c in self.fc_channels:
                layers += [nn.Linear(ch * spatial, c), nn.ReLU(inplace=True)]
                ch, spatial = c, 1
            self.shared_fcs = nn.Sequential(*layers)
        self.classifier = nn.Linear(ch * spatial, self.cls_channels)
        self.regressor = nn.Linear(ch * spatial, 4 if self.reg_class_agnostic else self.num_classes * 4)

    def init_weights(self):
        if self.with_shared_fcs:
            for m in self.shared_fcs:
                if isinstance(m, nn.Linear):
                    nn.init.xavier_uniform_(m.weight)
                    nn.init.constant_(m.bias, 0)
        init_module_normal(self.classifier, mean=0.0, std=0.01)
        init_module_normal(self.regressor, mean=0.0, std=0.001)

    def forward(self, rois):
        sizes = [r.shape[0] for r in rois]
        flat = getattr(rois, 'flat', None)
        x = flat if flat is not None else torch.cat(list(rois), 0)
        if self.with_avg_pool:
            x = self.avg_pool(x)
        x = x.reshape(x.shape[0], -1)
        if self.with_shared_fcs:
            x = self.shared_fcs(x)
        cls_out, reg_out = self.classifier(x), self.regressor(x)
        cls_outs, reg_outs = HeadOutputs(), HeadOutputs()
        off = 0
        for s in sizes:
            cls_outs.append(cls_out[off:off + s])
            reg_outs.append(reg_out[off:off + s])
            off += s
        cls_outs.flat = (cls_out, reg_out)
        return cls_outs, reg_outs

"""FCOS / ATSS detector (reference lib/detectors/fcos.py)."""
from torch import nn


class FCOS(nn.Module):
    def __init__(self, backbone=None, neck=None, bbox_head=None, train_cfg=None, test_cfg=None):
        super().__init__()
        from ..builder import build_module
        self.backbone = build_module(backbone)
        self.with_neck = neck is not None
        if self.with_neck:
            self.neck = build_module(neck)
        self.bbox_head = build_module(bbox_head)
        self.train_cfg, self.test_cfg = train_cfg, test_cfg

    def init_weights(self):
        self.backbone.init_weights()
        if self.with_neck:
            self.neck.init_weights()
        self.bbox_head.init_weights()

    def extract_feat(self, x):
        x = self.backbone(x)
        return self.neck(x) if self.with_neck else x

    def forward_train(self, img_data, gt_bboxes, gt_labels, img_metas):
        return self.bbox_head.forward_train(self.extract_feat(img_data), gt_bboxes, gt_labels, img_metas,
                                            self.train_cfg)

    def forward_test(self, img_data, img_metas):
        return self.bbox_head.predict_bboxes(self.extract_feat(img_data), img_metas, self.test_cfg)

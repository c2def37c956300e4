"""RetinaHead (reference lib/heads/retina_head.py): 9 octave anchors per location,
stacked conv towers (PyTorch-ROCm); targets/NMS through AnchorHead's HIP path."""
import numpy as np
from torch import nn

from .anchor_head import AnchorHead


def _normal_init(m, std, bias=0.0):
    nn.init.normal_(m.weight, 0.0, std)
    nn.init.constant_(m.bias, bias)


class RetinaHead(AnchorHead):
    def __init__(self, num_classes, in_channels, stacked_convs, feat_channels, octave_base_scale=4,
                 scales_per_octave=3, anchor_ratios=(0.5, 1.0, 2.0), anchor_strides=(8, 16, 32, 64, 128),
                 anchor_center_lt=False, target_means=(0.0, 0.0, 0.0, 0.0), target_stds=(1.0, 1.0, 1.0, 1.0),
                 loss_cls=None, loss_bbox=None):
        self.in_channels = in_channels
        self.feat_channels = feat_channels
        self.stacked_convs = stacked_convs
        self.octave_base_scale = octave_base_scale
        self.scales_per_octave = scales_per_octave
        scales = [octave_base_scale * 2 ** (i / scales_per_octave) for i in range(scales_per_octave)]
        super().__init__(num_classes, scales, anchor_ratios, anchor_strides, anchor_center_lt, target_means,
                         target_stds, loss_cls, loss_bbox)
        self.cls_channels = num_classes - 1
        self.init_layers()

    def init_layers(self):
        def tower():
            layers = []
            for i in range(self.stacked_convs):
                cin = self.in_channels if i == 0 else self.feat_channels
                layers += [nn.Conv2d(cin, self.feat_channels, 3, padding=1), nn.ReLU(inplace=True)]
            return nn.Sequential(*layers)
        self.cls_convs = tower()
        self.reg_convs = tower()
        self.retina_cls = nn.Conv2d(self.feat_channels, self.num_anchors * self.cls_channels, 3, padding=1)
        self.retina_reg = nn.Conv2d(self.feat_channels, self.num_anchors * 4, 3, padding=1)

    def init_weights(self):
        for tower in (self.cls_convs, self.reg_convs):
            for m in tower:
                if isinstance(m, nn.Conv2d):
                    _normal_init(m, 0.01)
        _normal_init(self.retina_cls, 0.01, float(-np.log((1 - 0.01) / 0.01)))
        _normal_init(self.retina_reg, 0.01)

    def forward(self, xs):
        cls = [self.retina_cls(self.cls_convs(x)) for x in xs]
        reg = [self.retina_reg(self.reg_convs(x)) for x in xs]
        return cls, reg

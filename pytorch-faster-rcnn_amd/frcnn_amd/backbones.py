"""ResNet backbone (stays on PyTorch-ROCm: MIOpen convs, MFMA f32).

Behaviour follows the reference's own ResNet (`lib/backbones.py:133-255`):
bottleneck blocks with the stride on the 3x3 conv, a 1x1 conv + BN projection
on the first block of every stage, frozen-BN training mode and
`frozen_stages` parameter freezing.  Parameter names are kept identical
(`conv1`, `bn1`, `layerK.i.convJ`, `layerK.0.downsample.{0,1}`) so state
dicts move between the two frameworks unchanged.

No pretrained download exists here (no network); `init_weights` uses a
deterministic Kaiming init when `pretrained` is requested and cannot be
satisfied, and says so.
"""
import logging

import torch
from torch import nn

from .ops import bn_act, bn_act_maxpool

# blocks per stage for each depth
_STAGE_BLOCKS = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}
_STAGE_WIDTH = (64, 256, 512, 1024, 2048)


def _conv_bn(cin, cout, k, stride=1, pad=0):
    return nn.Conv2d(cin, cout, k, stride=stride, padding=pad, bias=False), nn.BatchNorm2d(cout)


class Bottleneck(nn.Module):
    """1x1 -> 3x3 (strided) -> 1x1, expansion 4 (reference `backbones.py:133-168`)."""

    def __init__(self, in_channels, out_channels, downsample=False):
        super().__init__()
        mid = out_channels // 4
        first_stage = in_channels * 4 == out_channels
        stride = 2 if (downsample and not first_stage) else 1
        self.conv1, self.bn1 = _conv_bn(in_channels, mid, 1)
        self.conv2, self.bn2 = _conv_bn(mid, mid, 3, stride=stride, pad=1)
        self.conv3, self.bn3 = _conv_bn(mid, out_channels, 1)
        self.relu = nn.ReLU(inplace=True)
        self.do_downsample = downsample
        if downsample:
            self.downsample = nn.Sequential(*_conv_bn(in_channels, out_channels, 1, stride=stride))

    def forward(self, x):
        # frozen BN (+ residual) + ReLU as one HIP epilogue pass per conv (ops.bn_act)
        y = bn_act(self.conv1(x), self.bn1)
        y = bn_act(self.conv2(y), self.bn2)
        skip = bn_act(self.downsample[0](x), self.downsample[1], relu=False) if self.do_downsample else x
        return bn_act(self.conv3(y), self.bn3, skip=skip)


class ResNet(nn.Module):
    def __init__(self, depth=50, frozen_stages=1, out_layers=(1, 2, 3, 4), pretrained=True):
        super().__init__()
        if depth not in _STAGE_BLOCKS:
            raise AssertionError('unsupported ResNet depth {}'.format(depth))
        self.depth = depth
        self.pretrained = pretrained
        self.frozen_stages = frozen_stages
        self.out_layers = tuple(out_layers)
        self.conv_cfg = _STAGE_BLOCKS[depth]
        self.conv1, self.bn1 = _conv_bn(3, 64, 7, stride=2, pad=3)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        for s, nblk in enumerate(self.conv_cfg):
            cin, cout = _STAGE_WIDTH[s], _STAGE_WIDTH[s + 1]
            blocks = [Bottleneck(cin, cout, True)] + [Bottleneck(cout, cout) for _ in range(nblk - 1)]
            setattr(self, 'layer{}'.format(s + 1), nn.Sequential(*blocks))

    def forward(self, x):
        # frozen stem: BN + ReLU + max pool as one HIP pass (ops.bn_act_maxpool)
        x = bn_act_maxpool(self.conv1(x), self.bn1, self.maxpool)
        outs = []
        for s in range(1, 5):
            x = getattr(self, 'layer{}'.format(s))(x)
            if s in self.out_layers:
                outs.append(x)
        return outs

    def freeze_stages(self, stages):
        frozen = []
        if stages >= 0:
            self.bn1.eval()
            frozen += [self.conv1, self.bn1]
        for s in range(1, stages + 1):
            layer = getattr(self, 'layer{}'.format(s))
            layer.eval()
            frozen.append(layer)
        for m in frozen:
            for p in m.parameters():
                p.requires_grad = False

    def train(self, mode=True):
        super().train(mode)
        self.freeze_stages(self.frozen_stages)
        if mode:
            # BN statistics stay frozen during training (reference backbones.py:241-247)
            for m in self.modules():
                if isinstance(m, nn.BatchNorm2d):
                    m.eval()
        return self

    def init_weights(self):
        if self.pretrained:
            logging.warning('ResNet: pretrained weights unavailable offline; using random init')
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)


class ResLayerC5(nn.Module):
    """Stage-5 shared head for C4 detectors (reference `backbones.py:100-127`)."""

    def __init__(self, depth=50):
        super().__init__()
        nblk = _STAGE_BLOCKS[depth][3]
        self.res_layer = nn.Sequential(Bottleneck(1024, 2048, True),
                                       *[Bottleneck(2048, 2048) for _ in range(nblk - 1)])

    def train(self, mode=True):
        super().train(mode)
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()
        return self

    def forward(self, x):
        return self.res_layer(x)

    def init_weights(self):
        pass

"""FPN neck (convolutions on PyTorch-ROCm).

Same topology and parameter names as the reference FPN (`lib/necks.py:7-90`):
1x1 laterals, top-down nearest upsample-add, 3x3 output convs, and extra
levels either by stride-2 subsampling of the last output
(`max_pool2d(k=1, s=2)`, `necks.py:89`) or by stride-2 3x3 convs.

On a HIP device the levels come out channels-last (NHWC): the top-down merge
of every level is one HIP pass (`ops.fpn_merge_nhwc`: lateral + its conv bias +
nearest upsample of the merged coarser level, written NHWC), and the output convs run
in MIOpen's NHWC layout (channels-last weights, `utils.ChannelsLastConvs`) --
2.64 -> 2.41 ms for the FPN output convs + RPN head at cfg2 on MI355X
(`tools/probe_fpn_layout.py`).  The heads and the RoIAlign read NHWC levels
directly (strided kernels, the channel-quad RoIAlign).  CPU tensors take the
reference's NCHW ops.
"""
import torch
import torch.nn.functional as F
from torch import nn

from .utils import ChannelsLastConvs
from . import ops


class FPN(ChannelsLastConvs):
    def __init__(self, in_channels, out_channels, num_outs, start_level=0, end_level=-1,
                 extra_use_convs=False, extra_convs_on_inputs=True,
                 relu_before_extra_convs=False, with_activation=False):
        super().__init__()
        if with_activation:
            raise AssertionError('with_activation is not supported for FPN')
        if not isinstance(in_channels, list):
            raise AssertionError('in_channels must be a list')
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_ins = len(in_channels)
        self.start_level = start_level
        self.end_level = self.num_ins if end_level == -1 else end_level
        if not (self.start_level < self.end_level <= self.num_ins):
            raise AssertionError('bad FPN level range')
        self.used_ins = self.end_level - self.start_level
        if num_outs < self.used_ins:
            raise AssertionError('num_outs must cover the used inputs')
        self.num_outs = num_outs
        self.extra_use_convs = extra_use_convs
        self.extra_convs_on_inputs = extra_convs_on_inputs
        self.relu_before_extra_convs = relu_before_extra_convs

        self.lateral_convs = nn.ModuleList(
            nn.Conv2d(in_channels[i], out_channels, 1) for i in range(self.start_level, self.end_level))
        self.fpn_convs = nn.ModuleList(
            nn.Conv2d(out_channels, out_channels, 3, padding=1) for _ in range(self.used_ins))
        if extra_use_convs:
            for j in range(num_outs - self.used_ins):
                cin = in_channels[self.end_level - 1] if (j == 0 and extra_convs_on_inputs) else out_channels
                self.fpn_convs.append(nn.Conv2d(cin, out_channels, 3, stride=2, padding=1))

    def init_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.xavier_uniform_(m.weight)
                nn.init.zeros_(m.bias)

    def forward(self, inputs):
        if len(inputs) != self.num_ins:
            raise AssertionError('FPN expects {} inputs'.format(self.num_ins))
        x0 = inputs[self.start_level]
        if x0.is_cuda and x0.dtype == torch.float32:
            # lateral 1x1 convs without their bias; the bias add and the top-down merge into
            # channels-last levels are one HIP pass per level
            lat = [F.conv2d(inputs[self.start_level + i], conv.weight, None, conv.stride, conv.padding)
                   for i, conv in enumerate(self.lateral_convs)]
            bias = [conv.bias for conv in self.lateral_convs]
            merged = [None] * self.used_ins
            merged[-1] = ops.fpn_merge_nhwc(lat[-1], None, bias[-1])
            for i in range(self.used_ins - 1, 0, -1):
                merged[i - 1] = ops.fpn_merge_nhwc(lat[i - 1], merged[i], bias[i - 1])
            lat = merged
        else:
            lat = [conv(inputs[self.start_level + i]) for i, conv in enumerate(self.lateral_convs)]
            for i in range(self.used_ins - 1, 0, -1):
                lat[i - 1] = lat[i - 1] + F.interpolate(lat[i], size=lat[i - 1].shape[2:], mode='nearest')
        outs = [self.fpn_convs[i](lat[i]) for i in range(self.used_ins)]
        for i in range(self.used_ins, self.num_outs):
            if self.extra_use_convs:
                src = inputs[self.end_level - 1] if (i == self.used_ins and self.extra_convs_on_inputs) else outs[-1]
                y = self.fpn_convs[i](src)
                if self.relu_before_extra_convs:
                    y = F.relu(y)
                outs.append(y)
            else:
                outs.append(outs[-1][:, :, ::2, ::2])
        return outs

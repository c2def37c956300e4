"""Backbone + FPN convolution time in NCHW vs channels-last (MIOpen solvers, cfg2 shapes).

    python tools/probe_backbone_layout.py [--iters 10]

The bench's cfg2 model (random init); backbone + neck forward under no_grad, torch.profiler
kernel times summed per category: MIOpen kernels (convolutions and the transposes /
OpTensor kernels its solvers launch), at::native kernels (max-pool, bias adds, copies) and
frh:: kernels.  Layout 'nchw' is the product layout (NCHW backbone, channels-last FPN);
'nhwc' also runs the backbone channels-last (weights + input), with the frozen-BN epilogue
as plain torch ops on the NHWC tensor (its cost is not what is compared: the frh NCHW pass
and an NHWC pass move the same bytes).
"""
import argparse
import collections
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=10)
    args = ap.parse_args()
    import bench
    from frcnn_amd import backbones, ops
    from frcnn_amd.utils import conv_layout
    from torch.profiler import profile, ProfilerActivity
    dev = torch.device('cuda', 0)
    torch.backends.cudnn.benchmark = False
    model, _ = bench.make_model(dev, seed=0)
    imgs = bench.make_batch(dev, 2, seed=0)[0]
    orig_bn_act = ops.bn_act

    def nhwc_bn_act(x, bn, skip=None, relu=True):
        if x.is_contiguous():
            return orig_bn_act(x, bn, skip, relu)
        s = bn.weight * torch.rsqrt(bn.running_var + bn.eps)
        y = x * s.view(1, -1, 1, 1) + (bn.bias - bn.running_mean * s).view(1, -1, 1, 1)
        if skip is not None:
            y = y + skip
        return torch.relu_(y) if relu else y
    res = {}
    for layout in ('nchw', 'nhwc'):
        x = imgs
        if layout == 'nhwc':
            conv_layout(model.backbone)
            backbones.bn_act = nhwc_bn_act
            x = imgs.contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            for _ in range(3):
                model.neck(model.backbone(x))
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                model.neck(model.backbone(x))
            e1.record()
            torch.cuda.synchronize()
            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                for _ in range(args.iters):
                    model.neck(model.backbone(x))
                torch.cuda.synchronize()
        cat = collections.defaultdict(float)
        top = collections.defaultdict(float)
        for e in prof.events():
            if e.device_type != torch.autograd.DeviceType.CUDA:
                continue
            n = e.name
            c = 'frh' if 'frh::' in n else ('native' if 'at::native' in n else 'miopen')
            if c == 'miopen' and ('transpose' in n.lower() or 'SubTensor' in n or 'OpTensor' in n):
                c = 'miopen_aux'
            cat[c] += e.time_range.elapsed_us() / args.iters
            top[n[:80]] += e.time_range.elapsed_us() / args.iters
        res[layout] = {'us_per_forward_event': round(e0.elapsed_time(e1) * 1e3 / args.iters, 1),
                       'kernel_us_by_category': {k: round(v, 1) for k, v in cat.items()},
                       'top_kernels': {k: round(v, 1) for k, v in sorted(top.items(), key=lambda kv: -kv[1])[:25]}}
        print(layout, json.dumps(res[layout]['kernel_us_by_category']), res[layout]['us_per_forward_event'],
              flush=True)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()

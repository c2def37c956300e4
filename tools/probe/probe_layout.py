"""Trunk convolution cost by memory format (tools only).

    python tools/probe/probe_layout.py
Times the cfg2 trunk forward (backbone -> FPN -> RPN head convs, B=2, MIOpen Find on)
with the default NCHW tensors and with the FPN neck + RPN head in channels_last (NHWC
feature maps for an NHWC RoIAlign), plus the eager forward_train of both."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd'), os.path.join(REPO, 'tools', 'probe')]
import torch  # noqa: E402
import bench  # noqa: E402
from probe_roi import timeit  # noqa: E402
from frcnn_amd.graphs import Trunk  # noqa: E402


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device('cuda', 0)
    model, _ = bench.make_model(dev, seed=0)
    imgs, boxes, labels, metas = bench.make_batch(dev, 2, seed=1)
    trunk = Trunk(model.backbone, model.neck, model.rpn_head)
    with torch.no_grad():
        for name in ('nchw', 'neck_nhwc', 'nchw_again'):
            if name == 'neck_nhwc':
                model.neck.to(memory_format=torch.channels_last)
                model.rpn_head.to(memory_format=torch.channels_last)
            if name == 'nchw_again':
                model.neck.to(memory_format=torch.contiguous_format)
                model.rpn_head.to(memory_format=torch.contiguous_format)
            outs = trunk(imgs)
            print(name, 'feat strides', [tuple(o.stride()) for o in outs[:2]], flush=True)
            t = timeit(lambda: trunk(imgs), iters=20, warm=5)
            f = timeit(lambda: model.forward_train(imgs, boxes, labels, metas), iters=10, warm=3)
            print('{:12s} trunk {:8.1f} us   forward_train {:8.1f} us'.format(name, t, f), flush=True)


if __name__ == '__main__':
    main()

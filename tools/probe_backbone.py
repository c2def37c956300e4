"""GPU probe: fp32 ResNet50+FPN forward time at [2,3,608,1024], NCHW vs channels_last,
with MIOpen's heuristic algorithm choice or its benchmarked search (--benchmark)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'pytorch-faster-rcnn_amd'))
import torch  # noqa: E402
from frcnn_amd.backbones import ResNet  # noqa: E402
from frcnn_amd.necks import FPN  # noqa: E402


def run(fmt, grad, iters=10):
    torch.manual_seed(0)
    bb = ResNet(50, pretrained=False).cuda()
    nk = FPN([256, 512, 1024, 2048], 256, 5).cuda()
    bb.init_weights()
    nk.init_weights()
    bb.train()
    nk.train()
    x = torch.randn(2, 3, 608, 1024, device='cuda')
    if fmt == 'cl':
        bb = bb.to(memory_format=torch.channels_last)
        nk = nk.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    ctx = torch.enable_grad() if grad else torch.no_grad()
    with ctx:
        t0 = time.time()
        for _ in range(3):
            outs = nk(bb(x))
        torch.cuda.synchronize()
        warm = time.time() - t0
        t0 = time.time()
        for _ in range(iters):
            outs = nk(bb(x))
        torch.cuda.synchronize()
        dt = (time.time() - t0) / iters
    print(f'{fmt} grad={grad} benchmark={torch.backends.cudnn.benchmark}: {dt * 1e3:.2f} ms/step '
          f'(warmup {warm:.1f} s)  P2 stride={outs[0].stride()}', flush=True)


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--benchmark', action='store_true')
    ap.add_argument('--formats', default='nchw,cl')
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = args.benchmark
    print(torch.cuda.get_device_name(0), flush=True)
    for fmt in args.formats.split(','):
        for grad in (False, True):
            run(fmt, grad)

"""GPU probe: fp32 ResNet50+FPN forward time at [2,3,608,1024], NCHW vs channels_last."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'pytorch-faster-rcnn_amd'))
import torch
from frcnn_amd.backbones import ResNet
from frcnn_amd.necks import FPN


def run(fmt, grad, iters=10):
    torch.manual_seed(0)
    bb = ResNet(50, pretrained=False).cuda()
    nk = FPN([256, 512, 1024, 2048], 256, 5).cuda()
    bb.init_weights(); nk.init_weights(); bb.train(); nk.train()
    x = torch.randn(2, 3, 608, 1024, device='cuda')
    if fmt == 'cl':
        bb = bb.to(memory_format=torch.channels_last); nk = nk.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)
    ctx = torch.enable_grad() if grad else torch.no_grad()
    with ctx:
        for _ in range(3):
            outs = nk(bb(x))
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(iters):
            outs = nk(bb(x))
        torch.cuda.synchronize()
        dt = (time.time() - t0) / iters
    print(f'{fmt} grad={grad}: {dt*1e3:.2f} ms/step  P2 stride={outs[0].stride()} shape={tuple(outs[0].shape)}', flush=True)


if __name__ == '__main__':
    print(torch.cuda.get_device_name(0), flush=True)
    for fmt in ('nchw', 'cl'):
        for grad in (False, True):
            run(fmt, grad)

"""GPU probe: cost of channels-last (NHWC) FPN outputs for RoIAlign.

Times, on the cfg2 batch (2 x 608 x 1024, f32, MIOpen search on as in bench.py), the part
of the trunk whose layout would change: the FPN output convs (3x3, 256 -> 256, P2..P5 from
the lateral sums), the P6 subsample, and the RPN head (3x3 conv + ReLU, 1x1 cls / reg
convs on P2..P6) -- NCHW as today vs NHWC (channels_last weights and inputs; the inputs'
conversion is NOT timed: a fused transpose-add in the top-down pass would produce them).
Also times the plain NCHW -> NHWC copy of P2..P5 (what a separate transpose would cost)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'pytorch-faster-rcnn_amd'))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    grids = [(152, 256), (76, 128), (38, 64), (19, 32)]
    lat = [torch.randn(2, 256, h, w, device=dev) for h, w in grids]
    fpn = [torch.nn.Conv2d(256, 256, 3, padding=1).to(dev) for _ in range(4)]
    rpn = torch.nn.Conv2d(256, 256, 3, padding=1).to(dev)
    cls = torch.nn.Conv2d(256, 3, 1).to(dev)
    reg = torch.nn.Conv2d(256, 12, 1).to(dev)

    def trunk(lat_in):
        with torch.no_grad():
            outs = [c(x) for c, x in zip(fpn, lat_in)]
            outs.append(outs[-1][:, :, ::2, ::2])
            hid = [F.relu(rpn(o)) for o in outs]
            return outs, [cls(h) for h in hid], [reg(h) for h in hid]

    res = {}
    res['nchw_fpn_rpn_us'] = timeit(lambda: trunk(lat))
    with torch.no_grad():
        res['nchw_to_nhwc_copy_P2_P5_us'] = timeit(lambda: [x.contiguous(memory_format=torch.channels_last) for x in lat])
    for m in fpn + [rpn, cls, reg]:
        m.to(memory_format=torch.channels_last)
    lat_cl = [x.contiguous(memory_format=torch.channels_last) for x in lat]
    res['nhwc_fpn_rpn_us'] = timeit(lambda: trunk(lat_cl))
    outs, c, r = trunk(lat_cl)
    res['nhwc_P2_strides'] = list(outs[0].stride())
    res['nhwc_cls_strides'] = list(c[0].stride())
    print(res, flush=True)


if __name__ == '__main__':
    main()

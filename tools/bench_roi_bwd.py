"""Micro-benchmark of the RoIAlign backward kernels on the RoIs of a real cfg2 forward pass.

    python tools/bench_roi_bwd.py [--iters 20]
Times the product backward (frh_roi_align_bwd_strided into an NCHW gradient, separable
row-run sums) and the tools-library alternatives (frh_roi_align_bwd_cl: channels_last
gradient with 64-B atomic segments; frh_roi_align_bwd_tiled: tile lists + LDS gather), each
after the gradient clear it needs, with HIP events around back-to-back launches, and prints
the max |difference| between the gradients."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from frcnn_amd import ops, _lib, set_sampler_mode  # noqa: E402
import toolslib  # noqa: E402  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    set_sampler_mode('device', seed=1)
    model, batch = bench.make_model_and_batch(dev, batch=2)
    ops.ROI_ALIGN_PROFILE['on'] = True
    with torch.no_grad():
        model.forward_train(*batch)
    ops.ROI_ALIGN_PROFILE['on'] = False
    _, _, rois, levels, shapes, (ph, pw), feats, scales, sr = ops.ROI_ALIGN_PROFILE['records'][-1]
    K, B, C = rois.shape[0], shapes[0][0], shapes[0][1]
    g = torch.randn(K, C, ph, pw, device=dev)
    grads = {m: [torch.empty(s, device=dev) for s in shapes] for m in ('tiled', 'atomic')}
    grads['channels_last'] = [torch.empty(s, device=dev, memory_format=torch.channels_last) for s in shapes]
    hw_cl, st_cl = ops._feat_desc(grads['channels_last'])
    hw, st = ops._feat_desc(grads['tiled'])
    wsb = toolslib.load().frh_roi_align_bwd_workspace(len(shapes), hw, B, K)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    stream = _lib.stream_of(g)

    def tiled():
        gr = grads['tiled']
        toolslib.call('frh_roi_align_bwd_tiled', len(gr), _lib.ptr_array(gr), hw, st, _lib.f32_array(scales), B, C,
                  _lib.ptr(rois), _lib.ptr(levels), K, ph, pw, sr, 0, _lib.ptr(g), _lib.ptr(ws), wsb, stream)

    def atomic():
        gr = grads['atomic']
        for t in gr:
            t.zero_()
        _lib.call('frh_roi_align_bwd_strided', len(gr), _lib.ptr_array(gr), hw, st, _lib.f32_array(scales), B, C,
                  _lib.ptr(rois), _lib.ptr(levels), K, ph, pw, sr, 0, _lib.ptr(g), stream)

    def chlast():
        gr = grads['channels_last']
        for t in gr:
            t.zero_()
        toolslib.call('frh_roi_align_bwd_cl', len(gr), _lib.ptr_array(gr), hw_cl, st_cl, _lib.f32_array(scales), B,
                  C, _lib.ptr(rois), _lib.ptr(levels), K, ph, pw, sr, 0, _lib.ptr(g), stream)

    print('rois', K, 'level hist', np.bincount(levels.cpu().numpy(), minlength=len(shapes)).tolist(), flush=True)
    for name, fn in (('chlast', chlast), ('tiled', tiled), ('atomic', atomic)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print('{:>7}: {:8.1f} us per backward (incl. clearing the gradient where needed)'.format(name, e0.elapsed_time(e1) / args.iters * 1e3), flush=True)
    d = max(float((a - b).abs().max()) for a, b in zip(grads['tiled'], grads['atomic']))
    d2 = max(float((a - b).abs().max()) for a, b in zip(grads['channels_last'], grads['atomic']))
    print('max |channels_last - atomic| {:.3g}'.format(d2), flush=True)
    m = max(float(b.abs().max()) for b in grads['atomic'])
    print('max |tiled - atomic| {:.3g} (max |grad| {:.3g})'.format(d, m), flush=True)


if __name__ == '__main__':
    main()

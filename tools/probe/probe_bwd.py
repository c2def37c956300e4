"""RoIAlign backward: plane-sweep vs the per-RoI atomic kernel on the cfg2 RoIs (tools only).

    python tools/probe/probe_bwd.py
Times both (the atomic kernel including its gradient clearing, as the product runs it) and
prints the max |difference| of the gradients (float atomics: a few ulps expected)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd'), os.path.join(REPO, 'tools', 'probe')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from frcnn_amd import ops, _lib
import toolslib  # noqa: E402
from probe_roi import timeit  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    z = np.load(os.path.join(REPO, 'tools', 'data', 'cfg2_rois_cpu.npz'))
    shapes = [tuple(int(v) for v in s) for s in z['shapes']]
    scales = [float(s) for s in z['scales']]
    r5, lv = z['r5'], z['lv'].astype(np.int64)
    if os.environ.get('NODEGEN'):  # drop RoIs narrower / flatter than 1 px (contention experiment)
        keep = ((r5[:, 3] - r5[:, 1]) >= 1) & ((r5[:, 4] - r5[:, 2]) >= 1)
        r5, lv = r5[keep], lv[keep]
        print('kept', int(keep.sum()), 'of', len(keep), 'RoIs', flush=True)
    rois = torch.from_numpy(r5).to(dev)
    levels = torch.from_numpy(lv).to(dev)
    K, B, C = rois.shape[0], shapes[0][0], shapes[0][1]
    lib = toolslib.load()
    gout = torch.randn(K, C, 7, 7, device=dev)
    g_ref = [torch.empty(s, device=dev) for s in shapes]
    g_sw = [torch.full(s, float('nan'), device=dev) for s in shapes]
    hw, st = ops._feat_desc(g_ref)
    wsb = int(lib.frh_roi_align_sweep_workspace(ctypes.c_int64(K), 7, 7))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

    def atomic():
        for g in g_ref:
            g.zero_()
        s = lib.frh_roi_align_bwd_strided(len(shapes), _lib.ptr_array(g_ref), hw, st, _lib.f32_array(scales), B, C,
                                          _lib.ptr(rois), _lib.ptr(levels), K, 7, 7, 2, 0, _lib.ptr(gout),
                                          _lib.stream_of(gout))
        assert s == 0, lib.frh_last_error()

    def sweep():
        s = lib.frh_roi_align_bwd_sweep(len(shapes), _lib.ptr_array(g_sw), hw, st, _lib.f32_array(scales), B, C,
                                        _lib.ptr(rois), _lib.ptr(levels), K, 7, 7, 2, 0, _lib.ptr(gout),
                                        _lib.ptr(ws), wsb, _lib.stream_of(gout))
        assert s == 0, lib.frh_last_error()

    sweep()
    torch.cuda.synchronize()
    atomic()
    torch.cuda.synchronize()
    diff = max(float((a - b).abs().max()) for a, b in zip(g_ref, g_sw))
    mag = max(float(a.abs().max()) for a in g_ref)
    nan = sum(int(torch.isnan(b).sum()) for b in g_sw)
    print('max |diff| {:.3g} (max |grad| {:.3g}), NaN left {}'.format(diff, mag, nan), flush=True)
    print('atomic (incl. clearing): {:8.1f} us'.format(timeit(atomic, iters=10, warm=2)), flush=True)
    print('sweep                  : {:8.1f} us'.format(timeit(sweep, iters=10, warm=2)), flush=True)


if __name__ == '__main__':
    main()

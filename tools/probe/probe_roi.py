"""Memory-system probes for the RoIAlign forward redesign (tools only).

    python tools/probe/probe_roi.py
Times, on cfg2-shaped feature maps (2 images, P2..P5, C=256, random values) and the
1024 RoIs of tools/data/cfg2_rois_cpu.npz (a CPU run of the cfg2 forward):
  - the product RoIAlign forward variants,
  - plain streaming reads of every feature plane (106 MB), writes of the 51 MB output,
    and both in one launch: the floor of a plane-streaming design.
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from frcnn_amd import ops, _lib
import toolslib  # noqa: E402


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device('cuda', 0)
    z = np.load(os.path.join(REPO, 'tools', 'data', 'cfg2_rois_cpu.npz'))
    shapes = [tuple(int(v) for v in s) for s in z['shapes']]
    feats = [torch.randn(*s, device=dev) for s in shapes]
    rois = torch.from_numpy(z['r5']).to(dev)
    levels = torch.from_numpy(z['lv'].astype(np.int64)).to(dev)
    scales = [float(s) for s in z['scales']]
    K, C = rois.shape[0], shapes[0][1]
    lib = toolslib.load()
    hw, st = ops._feat_desc(feats)
    feat_bytes = sum(f.numel() * 4 for f in feats)
    out_bytes = K * C * 49 * 4
    print('rois', K, 'levels', np.bincount(z['lv'], minlength=4).tolist(), 'feat MB', feat_bytes / 1e6,
          'out MB', out_bytes / 1e6, flush=True)
    wsb = int(lib.frh_roi_align_workspace(ctypes.c_int64(K)))
    wsp = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    out = torch.empty(K, C, 7, 7, device=dev)
    ref = None
    for v in [int(x) for x in os.environ.get('VARIANTS', '10').split(',')]:
        def launch(v=v):
            s = lib.frh_roi_align_fwd_variant(v, len(feats), _lib.ptr_array(feats), hw, st, _lib.f32_array(scales),
                                              2, C, _lib.ptr(rois), _lib.ptr(levels), K, 7, 7, 2, 0, _lib.ptr(out),
                                              _lib.ptr(wsp), wsb, _lib.stream_of(out))
            assert s == 0, lib.frh_last_error()
        us = timeit(launch)
        if ref is None:
            ref = out.clone()
        print('roi_align variant {:3d}: {:7.1f} us  maxdiff {:.3g}'.format(v, us, float((out - ref).abs().max())),
              flush=True)

    pl = ctypes.CDLL(os.path.join(REPO, 'tools', 'probe', 'libprobe.so'))
    sink = torch.zeros(4, device=dev)
    flat = torch.cat([f.flatten() for f in feats])
    big_out = torch.empty(out_bytes // 4, device=dev)
    s = _lib.stream_of(flat)
    for grid in (1024, 2048, 4096):
        r = timeit(lambda: pl.probe_stream_read(ctypes.c_void_p(flat.data_ptr()), ctypes.c_int64(flat.numel() // 4),
                                                ctypes.c_void_p(sink.data_ptr()), grid, s))
        w = timeit(lambda: pl.probe_stream_write(ctypes.c_void_p(big_out.data_ptr()),
                                                 ctypes.c_int64(big_out.numel() // 4), grid, s))
        rw = timeit(lambda: pl.probe_stream_rw(ctypes.c_void_p(flat.data_ptr()), ctypes.c_int64(flat.numel() // 4),
                                               ctypes.c_void_p(big_out.data_ptr()), ctypes.c_int64(big_out.numel() // 4),
                                               ctypes.c_void_p(sink.data_ptr()), grid, s))
        print('grid {:5d}: read {:6.1f} us ({:5.2f} TB/s)  write {:6.1f} us ({:5.2f} TB/s)  read+write {:6.1f} us '
              '({:5.2f} TB/s)'.format(grid, r, feat_bytes / r / 1e6, w, out_bytes / w / 1e6, rw,
                                      (feat_bytes + out_bytes) / rw / 1e6), flush=True)
    # cold-ish: flush the caches with a 1 GB write between iterations
    junk = torch.empty(256 * 1024 * 1024, device=dev)

    def cold_rw():
        junk.fill_(1.0)
    torch.cuda.synchronize()
    tot = timeit(lambda: (cold_rw(), pl.probe_stream_rw(ctypes.c_void_p(flat.data_ptr()),
                                                         ctypes.c_int64(flat.numel() // 4),
                                                         ctypes.c_void_p(big_out.data_ptr()),
                                                         ctypes.c_int64(big_out.numel() // 4),
                                                         ctypes.c_void_p(sink.data_ptr()), 2048, s)), iters=10)
    only = timeit(cold_rw, iters=10)
    print('cold read+write: {:6.1f} us'.format(tot - only), flush=True)


if __name__ == '__main__':
    main()

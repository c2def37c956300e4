"""RoIAlign forward: does processing order matter?  The product kernel on the fixed RoI sets
of tools/bench_roi_sets.py in their own order, sorted by tap-window size descending (longest
items first: the launch's tail is the last items' lives) and ascending, µs per launch.  The
outputs land in the permuted order (this measures scheduling only).

    python tools/bench_roi_order.py [--sets bench,voc,train] [--iters 20] [--rounds 3]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tools'), os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from frcnn_amd import ops, _lib  # noqa: E402
from bench_roi_sets import load_set, tap_cells  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sets', default='bench,voc,train')
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    for name in args.sets.split(','):
        s = load_set(name, dev)
        if s is None:
            continue
        rois, levels, shapes, scales, feats = s
        K, C = rois.shape[0], shapes[0][1]
        cells = tap_cells(rois, levels, shapes, scales)
        r5 = rois.cpu().numpy()
        lvn = levels.cpu().numpy()
        sc_l = np.array(scales, np.float64)[lvn]
        cy = ((r5[:, 2] + r5[:, 4]) * 0.5 * sc_l).astype(np.int64)
        cx = ((r5[:, 1] + r5[:, 3]) * 0.5 * sc_l).astype(np.int64)

        def morton(y, x):
            z = np.zeros_like(y)
            for b in range(10):
                z |= ((y >> b) & 1) << (2 * b + 1) | ((x >> b) & 1) << (2 * b)
            return z
        img = r5[:, 0].astype(np.int64)
        orders = {'own': np.arange(K), 'desc': np.argsort(-cells, kind='stable'), 'asc': np.argsort(cells, kind='stable'),
                  'img_level': np.lexsort((np.arange(K), lvn, img)),
                  'morton': np.lexsort((morton(cy // 2, cx // 2), lvn, img)),
                  'raster8': np.lexsort((cx, cy // 8, lvn, img))}
        hw, st = ops._feat_desc(feats)
        sc = _lib.f32_array(scales)
        fp = _lib.ptr_array(feats)
        out = torch.empty(K, C, 7, 7, device=dev)
        res = {k: [] for k in orders}
        perm = {k: (rois[torch.from_numpy(o).to(dev)].contiguous(), levels[torch.from_numpy(o).to(dev)].contiguous())
                for k, o in orders.items()}
        for _ in range(args.rounds):
            for k, (r, lv) in perm.items():
                def f():
                    _lib.call('frh_roi_align_fwd_strided', len(feats), fp, hw, st, sc, shapes[0][0], C, _lib.ptr(r),
                              _lib.ptr(lv), K, 7, 7, 2, 0, _lib.ptr(out), _lib.stream_of(out))
                for _ in range(3):
                    f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.iters):
                    f()
                e1.record()
                torch.cuda.synchronize()
                res[k].append(e0.elapsed_time(e1) * 1e3 / args.iters)
        print('set {}: '.format(name) + ', '.join('{} {:.2f} us'.format(k, float(np.median(v))) for k, v in res.items()),
              flush=True)


if __name__ == '__main__':
    main()

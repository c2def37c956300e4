"""RoIAlign forward timing on RoI subsets / synthetic RoI sets (tools only).
Isolates the per-RoI kernel's cost structure: small vs large windows, repeated
(L2-hot) RoIs, spatial order."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np, torch
from frcnn_amd import ops, _lib
import toolslib


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


def window_area(r, lv, shapes, scales):
    out = []
    for k in range(len(r)):
        l = lv[k]; s = scales[l]; H, W = shapes[l][2], shapes[l][3]
        x1, y1, x2, y2 = r[k, 1:] * s
        w = max(x2 - x1, 1.0); h = max(y2 - y1, 1.0)
        out.append((min(h + 2, H)) * (min(w + 2, W)))
    return np.array(out)


def main():
    dev = torch.device('cuda', 0)
    z = np.load(os.path.join(REPO, 'tools', 'data', 'cfg2_rois_cpu.npz'))
    shapes = [tuple(int(v) for v in s) for s in z['shapes']]
    feats = [torch.randn(*s, device=dev) for s in shapes]
    scales = [float(s) for s in z['scales']]
    r5, lv = z['r5'], z['lv'].astype(np.int64)
    C = shapes[0][1]
    lib = toolslib.load()
    hw, st = ops._feat_desc(feats)
    area = window_area(r5, lv, shapes, scales)
    sets = {'all': np.arange(len(r5)), 'small<=256': np.nonzero(area <= 256)[0], 'large>256': np.nonzero(area > 256)[0]}
    rr = r5.copy()
    cy = (rr[:, 2] + rr[:, 4]) / 2
    sets['sorted_y'] = np.lexsort((cy, lv, rr[:, 0]))
    small = sets['small<=256']
    sets['rep_small'] = np.full(1024, small[len(small) // 2])
    big = sets['large>256']
    sets['rep_large'] = np.full(1024, big[np.argmax(area[big])])
    sets['rep_small_x4'] = np.full(4096, small[len(small) // 2])
    only = os.environ.get('SETS')
    for name, idx in sets.items():
        if only and name not in only.split(','):
            continue
        rois = torch.from_numpy(r5[idx]).to(dev).contiguous()
        levels = torch.from_numpy(lv[idx]).to(dev).contiguous()
        K = rois.shape[0]
        out = torch.empty(K, C, 7, 7, device=dev)
        ref_out = None
        for v in [int(x) for x in os.environ.get("VARIANTS", "10").split(",")]:
            out.fill_(float("nan"))
            if v == 60:
                wsb = int(lib.frh_roi_align_sweep_workspace(ctypes.c_int64(K), 7, 7))
                wsb0 = wsb
                ntask = 2 * (C // 2)
                wsb += ntask * 9 * 8
                wsp = torch.empty(wsb, dtype=torch.uint8, device=dev)
            def launch(v=v):
                if v == 60:
                    s = lib.frh_roi_align_fwd_sweep(len(feats), _lib.ptr_array(feats), hw, st, _lib.f32_array(scales),
                                                    2, C, _lib.ptr(rois), _lib.ptr(levels), K, 7, 7, 2, 0,
                                                    _lib.ptr(out), _lib.ptr(wsp), wsb, _lib.stream_of(out))
                    assert s == 0, lib.frh_last_error()
                    return
                s = lib.frh_roi_align_fwd_variant(v, len(feats), _lib.ptr_array(feats), hw, st,
                                                  _lib.f32_array(scales), 2, C, _lib.ptr(rois), _lib.ptr(levels), K,
                                                  7, 7, 2, 0, _lib.ptr(out), None, 0, _lib.stream_of(out))
                assert s == 0, lib.frh_last_error()
            us = timeit(launch, iters=int(os.environ.get('ITERS', '30')), warm=int(os.environ.get('WARM', '5')))
            if ref_out is None:
                ref_out = out.clone()
            if v == 60 and os.environ.get('FRH_SWEEP_DBG'):
                ntask = 2 * (C // 2)
                d = wsp[wsb0:wsb0 + ntask * 9 * 8].view(torch.int64).cpu().numpy()
                st_ = d[:ntask * 8].reshape(ntask, 8)
                cend = d[ntask * 8:ntask * 9]
                t0 = st_[:, 0].min()
                f = lambda a: np.percentile(a / 100.0, [10, 50, 90, 100]).round(2).tolist()
                print('  tasks', ntask, 'start', f(st_[:, 0] - t0), 'prologue', f(st_[:, 1] - st_[:, 0]),
                      'loader sweep', f(st_[:, 2] - st_[:, 1]), 'compute end', f(cend - st_[:, 0]),
                      'G', int(np.median(st_[:, 3])), 'npass', int(np.median(st_[:, 4])), flush=True)
            diff = float((out - ref_out).abs().max())
            print('{:14s} K {:5d} variant {:3d}: {:7.1f} us  ({:.3f} us per RoI, mean window {:.0f}) maxdiff {:.3g}'.format(
                name, K, v, us, us / K, area[idx].mean(), diff), flush=True)


if __name__ == '__main__':
    main()

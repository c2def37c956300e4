"""NMS scan micro-benchmark / timeline on RPN-shaped segments.

    python tools/bench_nms.py [--segs 10 --n 2000 --iters 20]
Synthetic proposals: anchor-like boxes (3 ratios on a stride-4..64 grid) with random
deltas, random scores, sorted per segment; IoU threshold 0.7 (RPN).  Times the legacy
and the pipelined scan (HIP events) and prints the pipelined resolver's per-block
timeline (wall_clock64 ticks: wait-for-tile, wait-for-helpers, resolve)."""
import argparse, ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np, torch
from frcnn_amd import ops, _lib


def make(segs, n, seed=0):
    rng = np.random.default_rng(seed)
    out = np.zeros((segs, n, 4), np.float32)
    for s in range(segs):
        stride = [4, 8, 16, 32, 64][s % 5]
        cx = rng.integers(0, 1000 // stride, n) * stride + stride / 2
        cy = rng.integers(0, 600 // stride, n) * stride + stride / 2
        ar = rng.choice([0.5, 1.0, 2.0], n)
        w = 8 * stride * np.sqrt(ar) * np.exp(rng.normal(0, 0.1, n))
        h = 8 * stride / np.sqrt(ar) * np.exp(rng.normal(0, 0.1, n))
        out[s] = np.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--segs', type=int, default=10)
    ap.add_argument('--n', type=int, default=2000)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--thr', type=float, default=0.7)
    ap.add_argument('--variants', default='0,1,2')
    ap.add_argument('--no-timeline', action='store_true')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _lib.load()
    lib.frh_nms_scan_debug.argtypes = [ctypes.c_int32, ctypes.c_void_p]
    boxes = torch.from_numpy(make(a.segs, a.n)).to(dev)
    counts = torch.full((a.segs,), a.n, dtype=torch.int32, device=dev)
    res = {}
    vs = [int(x) for x in a.variants.split(',')]
    for v in vs:
        lib.frh_nms_scan_debug(v, None)
        for _ in range(3):
            ops.nms_sorted(boxes, counts, a.n, a.thr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            keep, kc = ops.nms_sorted(boxes, counts, a.n, a.thr)
        e1.record()
        torch.cuda.synchronize()
        res[v] = (keep.clone(), kc.clone())
        print('scan variant {}: {:.1f} us per nms_sorted (mask + scan), kept {}'.format(
            v, e0.elapsed_time(e1) / a.iters * 1e3, kc.tolist()), flush=True)
    # mask kernel alone, by diagnostic mode (0 full, 1 no IoU loop, 2 no store); scan skipped via max_keep
    lib.frh_nms_mask_debug.argtypes = [ctypes.c_int32]
    for mode in (0, 1, 2):
        lib.frh_nms_mask_debug(mode)
        for _ in range(3):
            ops.nms_sorted(boxes, counts, a.n, a.thr)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            ops.nms_sorted(boxes, counts, a.n, a.thr)
        e1.record()
        torch.cuda.synchronize()
        print('mask mode {}: {:.1f} us per nms_sorted'.format(mode, e0.elapsed_time(e1) / a.iters * 1e3), flush=True)
    lib.frh_nms_mask_debug(0)
    for v in vs[1:]:
        ok = torch.equal(res[vs[0]][1], res[v][1])
        for sg in range(a.segs):
            k = int(res[vs[0]][1][sg])
            ok = ok and torch.equal(res[vs[0]][0][sg, :k], res[v][0][sg, :k])
        print('variant {} keep lists {} variant {}'.format(v, 'EQUAL to' if ok else 'DIFFER from', vs[0]), flush=True)
    if a.no_timeline:
        return
    dbg = torch.zeros(a.segs * 4 * 256, dtype=torch.int64, device=dev)
    lib.frh_nms_scan_debug(1, ctypes.c_void_p(dbg.data_ptr()))
    ops.nms_sorted(boxes, counts, a.n, a.thr)
    torch.cuda.synchronize()
    lib.frh_nms_scan_debug(1, None)
    t = dbg.view(a.segs, 256, 4).cpu().numpy().astype(np.int64)
    nb = (a.n + 63) // 64
    t0 = t[0, 0, 0]
    print('segment 0 resolver timeline (ticks from start): block, tile-wait, helper-wait, resolve')
    for b in range(nb):
        r = t[0, b] - t0
        print(b, r[0], r[1] - r[0], r[2] - r[1], r[3] - r[2])


if __name__ == '__main__':
    main()

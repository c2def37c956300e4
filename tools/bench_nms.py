"""NMS scan micro-benchmark / timeline on RPN-shaped segments.

    python tools/bench_nms.py [--segs 10 --n 2000 --iters 20]
Synthetic proposals: anchor-like boxes (3 ratios on a stride-4..64 grid) with random
deltas, random scores, sorted per segment; IoU threshold 0.7 (RPN).  Times one
nms_sorted call (mask + pipelined scan) with HIP events."""
import argparse, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pytorch-faster-rcnn_amd'), os.path.join(REPO, 'tools')]
import numpy as np, torch
from frcnn_amd import ops


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
    ap.add_argument('--timeline', action='store_true', help='per-block resolver stamps (tools library)')
    ap.add_argument('--ab', action='store_true', help='A/B against the exact-test mask (tools library)')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    boxes = torch.from_numpy(make(a.segs, a.n)).to(dev)
    counts = torch.full((a.segs,), a.n, dtype=torch.int32, device=dev)
    for _ in range(3):
        ops.nms_sorted(boxes, counts, a.n, a.thr)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        keep, kc = ops.nms_sorted(boxes, counts, a.n, a.thr)
    e1.record()
    torch.cuda.synchronize()
    print('{:.1f} us per nms_sorted (mask + scan), kept {}'.format(e0.elapsed_time(e1) / a.iters * 1e3, kc.tolist()),
          flush=True)
    if a.ab:  # exact-test mask (tools library) on the same segments: same keep lists, timed alike
        import ctypes
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import toolslib
        from frcnn_amd import _lib
        lib = toolslib.load()
        wsb = int(lib.frh_ex_nms_workspace(a.segs, a.n))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        kp = torch.full((a.segs, a.n), -1, dtype=torch.int32, device=dev)
        kc2 = torch.empty(a.segs, dtype=torch.int32, device=dev)
        for rnd in range(3):
            for name in ('frh_ex_nms_sorted', 'product'):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    if name == 'product':
                        keep, kc = ops.nms_sorted(boxes, counts, a.n, a.thr)
                    else:
                        toolslib.call(name, a.segs, _lib.ptr(boxes), a.n * 4, _lib.ptr(counts), a.n, a.thr, -1,
                                      _lib.ptr(kp), a.n, _lib.ptr(kc2), _lib.ptr(ws), wsb, _lib.stream_of(boxes))
                e1.record()
                torch.cuda.synchronize()
                print('  {:>18}: {:.1f} us per call'.format(name, e0.elapsed_time(e1) / a.iters * 1e3), flush=True)
        assert torch.equal(kc2, kc)
        for s_ in range(a.segs):
            n_ = int(kc[s_])
            assert torch.equal(kp[s_, :n_].cpu(), keep[s_, :n_].cpu()), s_
        print('  keep lists identical', flush=True)
    if a.timeline:
        import ctypes
        import numpy as np
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import toolslib
        from frcnn_amd import _lib
        lib = toolslib.load()
        stamps = torch.zeros(a.segs * 256 * 8, dtype=torch.int64, device=dev)
        wsb = int(lib.frh_tl_nms_workspace(a.segs, a.n))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        kp = torch.empty(a.segs, a.n, dtype=torch.int32, device=dev)
        kc2 = torch.empty(a.segs, dtype=torch.int32, device=dev)
        for on in (False, True):
            assert lib.frh_tl_nms_timeline(ctypes.c_void_p(stamps.data_ptr() if on else 0)) == 0
            toolslib.call('frh_tl_nms_sorted', a.segs, _lib.ptr(boxes), a.n * 4, _lib.ptr(counts), a.n, a.thr, -1,
                          _lib.ptr(kp), a.n, _lib.ptr(kc2), _lib.ptr(ws), wsb, _lib.stream_of(boxes))
            torch.cuda.synchronize()
        lib.frh_tl_nms_timeline(ctypes.c_void_p(0))
        assert torch.equal(kc2, kc)
        t = stamps.view(a.segs, 256, 8).cpu().numpy().astype(np.int64)
        nb = (a.n + 63) // 64
        print('segment 0 resolver, ticks of 10 ns: block, start, ready-wait, span OR, rounds, keep-list + publish')
        for b in range(nb):
            r = t[0, b]
            print(b, r[0] - t[0, 0, 0], r[1] - r[0], r[2] - r[1], r[3] - r[2], r[4] - r[3], flush=True)

if __name__ == '__main__':
    main()

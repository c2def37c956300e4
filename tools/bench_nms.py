"""NMS scan micro-benchmark / timeline on RPN-shaped segments.

    python tools/bench_nms.py [--segs 10 --n 2000 --iters 20]
Synthetic proposals: anchor-like boxes (3 ratios on a stride-4..64 grid) with random
deltas, random scores, sorted per segment; IoU threshold 0.7 (RPN).  Times one
nms_sorted call (mask + pipelined scan) with HIP events."""
import argparse, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
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

if __name__ == '__main__':
    main()

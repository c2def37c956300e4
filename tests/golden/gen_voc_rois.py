"""VOC-sized RoIs for the RoIAlign forward ("the RoIAlign microbenchmark
additionally uses VOC-sized RoIs"; random-init RoIs are degenerate: tiny boxes, ~85 % on P2).

    python -B tests/golden/gen_voc_rois.py

Writes tests/golden/cfg2_rois_voc.npz in the layout of cfg2_rois.npz (r5 [K, 5] rows
(image, x1, y1, x2, y2), lv [K] FPN levels, shapes [4, 4] of the cfg2 P2-P5 batch, scales).
Two images: the bench's own gts (tests/golden/voc_gts.npz images 0 and 1, the VOC07 boxes
bench.py's rank 0 trains on).  Per image, the mix the reference's RCNN sampler draws from a
trained RPN's proposals (lib/bbox.py:6-82 with configs/faster_rcnn_r50_fpn.py rcnn: max_num
512, pos_num 128, pos/neg IoU 0.5):
  * 128 positives: the prepended gts (lib/bbox.py:27-29) plus boxes jittered around the gts
    at IoU >= 0.5 (calc_iou's +1 rule, lib/utils.py:151-172);
  * 384 negatives (IoU < 0.5 to every gt): half near the objects (IoU in [0.1, 0.5)), half
    background boxes of VOC object sizes (sqrt(area) log-uniform in 32..500 px, aspect
    0.5..2).
Boxes are clamped to the 1000x600 image as the RPN's decode clamps them; rows are in a
random order (the sampler's ascending-proposal order is score order, unrelated to place).
Levels by the oracle's restatement of lib/region.py:256-264.  numpy PCG64 only: the same
file on every platform.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), 'oracle'))

import inputs  # noqa: E402

H_IMG, W_IMG = inputs.IMG_SHAPE
SHAPES = np.array([[2, 256, h, w] for h, w in inputs.FPN_GRIDS[:4]], np.int64)
SCALES = np.array([1.0 / s for s in inputs.FPN_STRIDES[:4]], np.float32)


def iou(a, g):
    """calc_iou (+1 widths, lib/utils.py:151-172) of boxes a [n, 4] against gts g [G, 4]."""
    tl = np.maximum(a[:, None, :2], g[None, :, :2])
    br = np.minimum(a[:, None, 2:], g[None, :, 2:])
    inter = np.prod(br - tl + 1, axis=2) * np.all(tl < br, axis=2)
    area = lambda b: (b[..., 2] - b[..., 0] + 1) * (b[..., 3] - b[..., 1] + 1)  # noqa: E731
    return inter / (area(a)[:, None] + area(g)[None, :] - inter)


def clamp(b):
    b = b.copy()
    b[:, 0::2] = np.clip(b[:, 0::2], 0, W_IMG - 1)
    b[:, 1::2] = np.clip(b[:, 1::2], 0, H_IMG - 1)
    ok = (b[:, 2] > b[:, 0]) & (b[:, 3] > b[:, 1])
    return b[ok]


def jitter(rng, g, n, sigma):
    """n boxes around gt g: centre shift ~ N(0, sigma * side), log-size ~ N(0, sigma)."""
    w, h = g[2] - g[0] + 1, g[3] - g[1] + 1
    cx, cy = (g[0] + g[2]) / 2, (g[1] + g[3]) / 2
    cx = cx + rng.normal(0, sigma, n) * w
    cy = cy + rng.normal(0, sigma, n) * h
    nw = w * np.exp(rng.normal(0, sigma, n))
    nh = h * np.exp(rng.normal(0, sigma, n))
    return clamp(np.stack([cx - nw / 2, cy - nh / 2, cx + nw / 2 - 1, cy + nh / 2 - 1], 1))


def background(rng, n):
    side = np.exp(rng.uniform(np.log(32), np.log(500), n))
    ar = np.exp(rng.uniform(np.log(0.5), np.log(2.0), n))
    w, h = side * np.sqrt(ar), side / np.sqrt(ar)
    x1 = rng.uniform(-0.1 * W_IMG, W_IMG, n)
    y1 = rng.uniform(-0.1 * H_IMG, H_IMG, n)
    return clamp(np.stack([x1, y1, x1 + w, y1 + h], 1))


def image_rois(rng, gt, n_pos=128, n=512):
    g = gt.T.astype(np.float64)  # [G, 4]
    pos = [g]
    while sum(len(p) for p in pos) < n_pos:
        k = int(rng.integers(len(g)))
        c = jitter(rng, g[k], 64, 0.12)
        pos.append(c[iou(c, g).max(1) >= 0.5])
    pos = np.concatenate(pos)[:n_pos]
    near, n_near = [], (n - n_pos) // 2
    while sum(len(p) for p in near) < n_near:
        k = int(rng.integers(len(g)))
        c = jitter(rng, g[k], 64, 0.45)
        m = iou(c, g).max(1)
        near.append(c[(m >= 0.1) & (m < 0.5)])
    near = np.concatenate(near)[:n_near]
    bg = []
    while sum(len(b) for b in bg) < n - n_pos - n_near:
        c = background(rng, 256)
        bg.append(c[iou(c, g).max(1) < 0.5])
    bg = np.concatenate(bg)[:n - n_pos - n_near]
    rest = np.concatenate([pos[len(g):], near, bg])
    rest = rest[rng.permutation(len(rest))]
    return np.concatenate([pos[:len(g)], rest]).astype(np.float32)


def main():
    import oracle
    rng = np.random.default_rng(20260518)
    gts = inputs.voc_gts()
    rows = []
    for b in range(2):
        r = image_rois(rng, gts[b][0])
        rows.append(np.concatenate([np.full((len(r), 1), b, np.float32), r], 1))
    r5 = np.ascontiguousarray(np.concatenate(rows), np.float32)
    lv = oracle.roi_level_map(r5, 56.0, 4)
    out = os.path.join(HERE, 'cfg2_rois_voc.npz')
    np.savez_compressed(out, r5=r5, lv=lv, shapes=SHAPES, scales=SCALES)
    side = np.sqrt((r5[:, 3] - r5[:, 1] + 1) * (r5[:, 4] - r5[:, 2] + 1))
    print('wrote {}: {} RoIs, levels {}, median side {:.0f} px'.format(
        out, len(r5), np.bincount(lv, minlength=4).tolist(), float(np.median(side))))


if __name__ == '__main__':
    main()

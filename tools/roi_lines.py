"""Distinct 128-B feature lines the RoIAlign tap windows of the cfg2 bench RoIs touch
(NCHW, per channel), against the line-uses of the per-RoI staging -- the floor on the
forward's feature traffic when every reuse hits in L2.

    python tools/roi_lines.py [tests/golden/cfg2_rois.npz]
Window rule as roi_align_fwd_pair_kernel stages it (torchvision legacy taps, 7x7 bins,
sampling 2; dense rows / columns while the window is at most 28 wide, else the tap list)."""
import sys

import numpy as np

P = 7


def taps(start, binsz, n):
    out = set()
    for p in range(P):
        for i in range(2):
            y = np.float32(start + p * binsz + (i + 0.5) * binsz / 2)
            if y < -1 or y > n:
                continue
            y = max(y, 0)
            lo = int(np.floor(y))
            hi = lo + 1
            if lo >= n - 1:
                lo = hi = n - 1
            out.update((lo, hi))
    return out


def main():
    d = np.load(sys.argv[1] if len(sys.argv) > 1 else 'tests/golden/cfg2_rois.npz')
    r5, lv, shapes, sc = d['r5'], d['lv'], d['shapes'], d['scales']
    uniq, uses = set(), 0
    for k in range(len(r5)):
        b, x1, y1, x2, y2 = r5[k]
        l = lv[k]
        H, W, s = shapes[l][2], shapes[l][3], sc[l]
        sw, sh = x1 * s, y1 * s
        rw, rh = max(x2 * s - sw, 1), max(y2 * s - sh, 1)
        ys, xs = taps(sh, rh / P, H), taps(sw, rw / P, W)
        if not ys or not xs:
            continue
        rows = range(min(ys), max(ys) + 1) if max(ys) - min(ys) + 1 <= 28 else sorted(ys)
        cols = range(min(xs), max(xs) + 1) if max(xs) - min(xs) + 1 <= 28 else sorted(xs)
        for y in rows:
            ls = {(y * W * 4 + c * 4) // 128 for c in cols}
            uses += len(ls)
            uniq.update((int(b), int(l), li) for li in ls)
    C = int(shapes[0][1])
    print('line uses per channel {}, distinct {}: {:.1f} MB staged without reuse, {:.1f} MB distinct (C = {})'.format(
        uses, len(uniq), uses * 128 * C / 1e6, len(uniq) * 128 * C / 1e6, C))


if __name__ == '__main__':
    main()

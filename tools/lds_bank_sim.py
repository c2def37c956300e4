"""Offline LDS bank model of the RoIAlign forward's tap reads (no GPU).

For every item of a RoI set (tests/golden/cfg2_rois*.npz) this rebuilds the addresses the
channels-last forward's ds_read_b128 tap reads use (pair_setup<16> in roi_kernels.h: lane =
bin, tap bases and row / column deltas), and counts LDS-array cycles with the gfx950 banking of
MI355X_MICROARCH.md §LDS: ds_read_b128 is serviced in 4 lane groups of 16, bank of byte a =
(a / 4) mod 64, a 16-B read covers 4 banks, identical addresses broadcast, each extra distinct
address on a busy bank in a group costs one cycle.  Layouts:
  quad   [quad][cell], 16 B per cell (windows <= 192 cells: the product's quad path, D = 4)
  ilv    [cell][2 quads], 32 B per cell (<= 480 cells), quad d at step d, or rotated
  band   [cell][16 ch], 64 B per cell, rotated quads (kRot)
and candidate swizzles.  Prints conflict cycles / all cycles (SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE) per path and set.

    python tools/lds_bank_sim.py [--sets bench,voc,train]
"""
import argparse
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETS = {'bench': 'cfg2_rois.npz', 'voc': 'cfg2_rois_voc.npz', 'train': 'cfg2_rois_train.npz'}
GROUPS_B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
               list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
               list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64))]
PH = PW = 7


def f32(x):
    return np.float32(x)


def make_tap(v, size):
    v = f32(v)
    if v < -1.0 or v > size:
        return None
    if v <= 0:
        v = f32(0)
    lo = int(v)
    if lo >= size - 1:
        return (size - 1, size - 1)
    return (lo, lo + 1)


def setup(roi, shape, scale):
    """pair_setup<16>: per lane (bin), the 4 samples' (valid, r0, r1, q0, q1) in slab cells, and
    the window's R, Cs, Cs2."""
    _, x1, y1, x2, y2 = [f32(v) for v in roi]
    H, W = shape
    sc = f32(scale)
    sw, sh, ew, eh = x1 * sc, y1 * sc, x2 * sc, y2 * sc
    rw, rh = max(f32(ew - sw), f32(1)), max(f32(eh - sh), f32(1))
    bh, bw = f32(rh / f32(PH)), f32(rw / f32(PW))

    def pos(start, b, p, i):
        return f32(f32(start + f32(f32(p) * b)) + f32(f32(f32(i) + f32(0.5)) * b) * f32(0.5))
    ty = [make_tap(pos(sh, bh, s >> 1, s & 1), H) for s in range(2 * PH)]
    tx = [make_tap(pos(sw, bw, s >> 1, s & 1), W) for s in range(2 * PW)]
    vy = [t for t in ty if t]
    vx = [t for t in tx if t]
    if not vy or not vx:
        return None
    y0, y1_ = min(t[0] for t in vy), max(t[1] for t in vy)
    x0, x1_ = min(t[0] for t in vx), max(t[1] for t in vx)
    dy, dx = y1_ - y0 + 1 <= 4 * PH, x1_ - x0 + 1 <= 4 * PW
    R = y1_ - y0 + 1 if dy else 4 * PH
    Cs = x1_ - x0 + 1 if dx else 4 * PW
    Cs2 = Cs | 1
    lanes = []
    for lane in range(64):
        b = lane if lane < PH * PW else 0
        py, px = b // PW, b % PW
        samp = []
        for iy in range(2):
            a = ty[2 * py + iy]
            r0 = (a[0] - y0 if dy else 2 * (py * 2 + iy)) if a else 0
            r1 = (a[1] - y0 if dy else 2 * (py * 2 + iy) + 1) if a else 0
            for ix in range(2):
                t = tx[2 * px + ix]
                q0 = (t[0] - x0 if dx else 2 * (px * 2 + ix)) if t else 0
                q1 = (t[1] - x0 if dx else 2 * (px * 2 + ix) + 1) if t else 0
                samp.append((bool(a and t), r0, r1, q0, q1))
        lanes.append(samp)
    return R, Cs, Cs2, lanes


def cycles(addrs):
    """LDS cycles of one ds_read_b128 (64 byte addresses)."""
    tot = 0
    for g in GROUPS_B128:
        slots = {}
        for ln in g:
            a = addrs[ln]
            slots.setdefault((a // 16) % 16, set()).add(a)
        tot += max(len(v) for v in slots.values())
    return tot


def item_reads(R, Cs2, lanes, cell_bytes, quad_off, rot=False, steps=4, cell_addr=None):
    """Tap-read addresses of one item: per step d (one quad / 16-B unit of the cell) and half-row
    (iy), 8 reads (ix, q).  cell_addr(cell) -> byte offset of the cell's first unit; quad_off(q)
    -> byte offset of unit q within the cell (or region)."""
    reads = []
    for d in range(steps):
        for iy in range(2):
            for ix in range(2):
                for q in range(4):
                    addrs = []
                    for lane in range(64):
                        valid, r0, r1, q0, q1 = lanes[lane][2 * iy + ix]
                        if not valid:
                            cell = 0
                        else:
                            cell = (r1 if q & 2 else r0) * Cs2 + (q1 if q & 1 else q0)
                        qq = (d + lane) % steps if rot else d
                        addrs.append(cell_addr(cell) + quad_off(qq))
                    reads.append(addrs)
    return reads


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sets', default='bench,voc,train')
    ap.add_argument('--limit', type=int, default=400, help='RoIs per set (a sample)')
    args = ap.parse_args()
    for name in args.sets.split(','):
        path = os.path.join(REPO, 'tests', 'golden', SETS[name])
        if not os.path.exists(path):
            continue
        z = np.load(path)
        rois, lv = z['r5'], z['lv']
        shapes = [tuple(int(v) for v in s[2:]) for s in z['shapes']]
        scales = [float(v) for v in z['scales']]
        idx = np.random.default_rng(0).permutation(len(rois))[:args.limit]
        stats = {}

        def add(key, reads):
            c = sum(cycles(a) for a in reads)
            s = stats.setdefault(key, [0, 0, 0])
            s[0] += c
            s[1] += 4 * len(reads)
            s[2] += 1
        for i in idx:
            st = setup(rois[i], shapes[lv[i]], scales[lv[i]])
            if st is None:
                continue
            R, Cs, Cs2, lanes = st
            ncell = R * Cs2
            def xs(c, b):  # XOR swizzle of a cell index: blocks of 2^b cells, low bits ^= block id
                return c ^ ((c >> b) & ((1 << b) - 1))
            if ncell <= 192:
                add('quad xor16', item_reads(R, Cs2, lanes, 16, lambda q: 3072 * q, cell_addr=lambda c: 16 * xs(c, 4)))
                add('quad xor16 rot+pad', item_reads(R, Cs2, lanes, 16, lambda q: 3072 * q + 16 * q, rot=True,
                                                     cell_addr=lambda c: 16 * xs(c, 4)))
                # quad path: region d at 3072-B steps, 16 B per cell
                add('quad', item_reads(R, Cs2, lanes, 16, lambda q: 3072 * q, cell_addr=lambda c: 16 * c))
                add('quad+pad16 rot', item_reads(R, Cs2, lanes, 16, lambda q: 3072 * q + 16 * q, rot=True,
                                                 cell_addr=lambda c: 16 * c))
                add('quad+pad16', item_reads(R, Cs2, lanes, 16, lambda q: 3072 * q + 16 * q,
                                             cell_addr=lambda c: 16 * c))
                add('quad+pad64 rot', item_reads(R, Cs2, lanes, 16, lambda q: 3072 * q + 64 * q, rot=True,
                                                 cell_addr=lambda c: 16 * c))
            elif ncell <= 480:
                for stage in range(2):
                    add('ilv', item_reads(R, Cs2, lanes, 32, lambda q: 16 * q, steps=2,
                                          cell_addr=lambda c: 32 * c))
                    add('ilv rot', item_reads(R, Cs2, lanes, 32, lambda q: 16 * q, rot=True, steps=2,
                                              cell_addr=lambda c: 32 * c))
                    add('ilv xor8', item_reads(R, Cs2, lanes, 32, lambda q: 16 * q, steps=2,
                                               cell_addr=lambda c: 32 * xs(c, 3)))
                    add('ilv xor8 rot', item_reads(R, Cs2, lanes, 32, lambda q: 16 * q, rot=True, steps=2,
                                                   cell_addr=lambda c: 32 * xs(c, 3)))
            else:
                add('band rot (one band)', item_reads(R, Cs2, lanes, 64, lambda q: 16 * q, rot=True,
                                                      cell_addr=lambda c: 64 * c))
                add('band (one band)', item_reads(R, Cs2, lanes, 64, lambda q: 16 * q,
                                                  cell_addr=lambda c: 64 * c))
                add('band xor4 rot', item_reads(R, Cs2, lanes, 64, lambda q: 16 * q, rot=True,
                                                cell_addr=lambda c: 64 * xs(c, 2)))
        print('set', name)
        for k, (c, base, n) in stats.items():
            print('  {:22s} items {:4d}  cycles/read {:.2f}  conflict share {:.1%}'.format(
                k, n, c / (base / 4), (c - base) / c))


if __name__ == '__main__':
    main()

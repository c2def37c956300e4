"""RoIAlign forward on fixed RoI sets: the product kernel, the round-4 library and tools
variants, µs per launch and algorithmic GB/s (SURVEY §8(d) bytes), bit-equality to the
product.

    python tools/bench_roi_sets.py [--sets bench,voc,train] [--variants 25] [--iters 20] [--rounds 3]
Sets (tests/golden): bench = cfg2_rois.npz (the RoIs of a random-init cfg2 step), voc =
cfg2_rois_voc.npz (gen_voc_rois.py: the RCNN sampler's mix around the bench images' VOC
gts), train = cfg2_rois_train.npz (a `bench.py --mode train` step's RoIs, dumped by
`bench.py --dump-rois`).  Features: N(0,1) channels-last P2-P5 of the set's shapes, C = 256
(the product trunk's FPN layout).  The round-4 library (tools/lib/r4/libfrcnn_amd_r4.so,
built from the round-4 commit by tools/build_r4_lib.sh) is the A/B reference for the
kernel that shipped then: 8-KB slab, per-lane global gathers for tap grids > 512 cells."""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd'),
                os.path.join(REPO, 'tests', 'golden')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from frcnn_amd import ops, _lib  # noqa: E402

SETS = {'bench': 'cfg2_rois.npz', 'voc': 'cfg2_rois_voc.npz', 'train': 'cfg2_rois_train.npz'}
STAMPED = {9, 15, 27, 29, 39, 56, 58, 94}  # tools variants writing per-item phase stamps (s_memrealtime)
STAMPED_CG = {94}  # channel-group kernel stamps: [start, setup, land, end, bands, cells, record, eval done]
R4_LIB = os.path.join(REPO, 'tools', 'lib', 'r4', 'libfrcnn_amd_r4.so')


def load_set(name, dev):
    path = os.path.join(REPO, 'tests', 'golden', SETS[name])
    if not os.path.exists(path):
        return None
    z = np.load(path)
    rois = torch.from_numpy(np.ascontiguousarray(z['r5'], np.float32)).to(dev)
    levels = torch.from_numpy(z['lv'].astype(np.int64)).to(dev)
    shapes = [tuple(int(v) for v in s) for s in z['shapes']]
    scales = [float(v) for v in z['scales']]
    g = torch.Generator(device='cpu').manual_seed(7)
    feats = [torch.randn(s, generator=g).to(dev).contiguous(memory_format=torch.channels_last) for s in shapes]
    return rois, levels, shapes, scales, feats


def algorithmic_bytes(rois, levels, shapes, ph=7, pw=7):
    K, C = rois.shape[0], shapes[0][1]
    used = torch.unique(rois[:, 0].long() * 64 + levels).cpu().tolist()
    return 4 * C * (K * ph * pw + sum(shapes[u % 64][2] * shapes[u % 64][3] for u in used)) + 20 * K


def tap_cells(rois, levels, shapes, scales):
    """Staged cells per RoI (the quad kernel's tap grid: rows x odd row stride)."""
    out = []
    for (b, x1, y1, x2, y2), l in zip(rois.cpu().numpy(), levels.cpu().numpy()):
        H, W, s = shapes[l][2], shapes[l][3], scales[l]

        def span(start, size, n):
            t = []
            for p in range(7):
                for i in range(2):
                    y = np.float32(start + p * size / 7 + (i + 0.5) * (size / 7) / 2)
                    if y < -1 or y > n:
                        continue
                    y = max(y, 0)
                    lo = int(np.floor(y))
                    t += [n - 1, n - 1] if lo >= n - 1 else [lo, lo + 1]
            return (min(28, max(t) - min(t) + 1)) if t else 0
        rw, rh = max(x2 * s - x1 * s, 1), max(y2 * s - y1 * s, 1)
        out.append(span(y1 * s, rh, H) * (span(x1 * s, rw, W) | 1))
    return np.array(out)


def cg_stamps_report(stm):
    stm = stm.reshape(-1, 16)  # 16 int64 per item
    """Per-item phases of the channel-group kernel (µs, 100 MHz clock): record landed, window /
    tables computed, first band landed (DMA + barrier), evaluation done (all bands), end (output
    block stored); by band count."""
    stm = stm[stm[:, 0] > 0]
    t0 = stm[:, 0].min()
    span = (stm[:, 3].max() - t0) / 100.0
    pc = lambda a: np.percentile(a / 100.0, [50, 90]).round(2).tolist()  # noqa: E731
    print('  {} items; span {:.1f} us'.format(len(stm), span))
    for nb in sorted(set(stm[:, 4].tolist())):
        x = stm[stm[:, 4] == nb]
        print('  bands={} items {:5d} cells p50 {:4.0f}: record {} setup {} land {} eval {} out {} life {}'.format(
            nb, len(x), np.median(x[:, 5]), pc(x[:, 6] - x[:, 0]), pc(x[:, 1] - x[:, 6]), pc(x[:, 2] - x[:, 1]),
            pc(x[:, 7] - x[:, 2]), pc(x[:, 3] - x[:, 7]), pc(x[:, 3] - x[:, 0])))
        print('      setup: geometry + taps {} window {} tables {} bands {}'.format(
            pc(x[:, 8] - x[:, 6]), pc(x[:, 9] - x[:, 8]), pc(x[:, 10] - x[:, 9]), pc(x[:, 1] - x[:, 10])))
    alive = np.zeros(int(span) + 1)
    for a, b in zip((stm[:, 0] - t0) / 100.0, (stm[:, 3] - t0) / 100.0):
        alive[int(a):int(b) + 1] += 1
    print('  items alive per CU by us: ' + ' '.join('%.1f' % (v / 256) for v in alive))
    print('  start-time percentiles 0/50/100:', np.percentile((stm[:, 0] - t0) / 100.0, [0, 50, 100]).round(1).tolist(),
          'end 50/90/100:', np.percentile((stm[:, 3] - t0) / 100.0, [50, 90, 100]).round(1).tolist(), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sets', default='bench,voc,train')
    ap.add_argument('--variants', default='25', help='tools-library variants to time beside the product')
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--json', help='write the summary here')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    sig = _lib.SIGNATURES['frh_roi_align_fwd_strided']
    r4 = None
    if os.path.exists(R4_LIB):
        r4 = ctypes.CDLL(R4_LIB)
        r4.frh_roi_align_fwd_strided.restype, r4.frh_roi_align_fwd_strided.argtypes = sig[0], sig[1]
    tools = None
    variants = [int(v) for v in args.variants.split(',') if v]
    if variants:
        import toolslib
        tools = toolslib.load()
    summary = {}
    for name in args.sets.split(','):
        s = load_set(name, dev)
        if s is None:
            print('set {}: fixture absent, skipped'.format(name), flush=True)
            continue
        rois, levels, shapes, scales, feats = s
        K, C = rois.shape[0], shapes[0][1]
        nbytes = algorithmic_bytes(rois, levels, shapes)
        cells = tap_cells(rois, levels, shapes, scales)
        hw, st = ops._feat_desc(feats)
        sc = _lib.f32_array(scales)
        fp = _lib.ptr_array(feats)
        outs = {}

        def runner(kind):
            out = torch.empty(K, C, 7, 7, device=dev)
            outs[kind] = out
            if kind == 'product':
                return lambda: _lib.call('frh_roi_align_fwd_strided', len(feats), fp, hw, st, sc, shapes[0][0], C,
                                         _lib.ptr(rois), _lib.ptr(levels), K, 7, 7, 2, 0, _lib.ptr(out),
                                         _lib.stream_of(out))
            if kind == 'r4':
                def f():
                    assert r4.frh_roi_align_fwd_strided(len(feats), fp, hw, st, sc, shapes[0][0], C, _lib.ptr(rois),
                                                        _lib.ptr(levels), K, 7, 7, 2, 0, _lib.ptr(out),
                                                        _lib.stream_of(out)) == 0
                return f
            v = int(kind[1:])
            ws = torch.empty(64 * K, dtype=torch.uint8, device=dev)
            if v in STAMPED:  # 8 int64 stamps per item after the output (<= K * C / 16 items)
                full = torch.zeros(K * C * 49 + (K * C // 16) * 16, device=dev)
                out = full[:K * C * 49].view(K, C, 7, 7)
                outs[kind] = out
                stamps[kind] = full[K * C * 49:].view(torch.int64).view(-1, 8)

            def g():
                r = tools.frh_roi_align_fwd_variant(v, len(feats), fp, hw, st, sc, shapes[0][0], C, _lib.ptr(rois),
                                                    _lib.ptr(levels), K, 7, 7, 2, 0, _lib.ptr(out), _lib.ptr(ws),
                                                    ws.numel(), _lib.stream_of(out))
                assert r == 0, tools.frh_last_error()
            return g
        stamps = {}
        kinds = ['product'] + (['r4'] if r4 else []) + ['v{}'.format(v) for v in variants]
        fns = {k: runner(k) for k in kinds}
        times = {k: [] for k in kinds}
        for _ in range(args.rounds):
            for k in kinds:
                for _ in range(3):
                    fns[k]()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.iters):
                    fns[k]()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1) * 1e3 / args.iters)
        print('set {}: K {} levels {} tap cells p50 {:.0f} p90 {:.0f} >512 {:.1%}; algorithmic {:.1f} MB'.format(
            name, K, np.bincount(levels.cpu().numpy(), minlength=4).tolist(), np.median(cells),
            np.percentile(cells, 90), (cells > 512).mean(), nbytes / 1e6), flush=True)
        summary[name] = {'rois': K, 'algorithmic_bytes': nbytes, 'tap_cells_p50': float(np.median(cells)),
                         'tap_cells_gt512': float((cells > 512).mean()), 'kernels': {}}
        for k in kinds:
            us = float(np.median(times[k]))
            same = bool(torch.equal(outs[k], outs['product']))
            frac = nbytes / (us * 1e-6) / 8e12
            summary[name]['kernels'][k] = {'us': us, 'frac': frac, 'bit_identical_to_product': same}
            print('  {:8s} {:8.2f} us  frac {:.3f}  bit-identical to product: {}'.format(k, us, frac, same), flush=True)
            if k in stamps and int(k[1:]) in STAMPED_CG:
                cg_stamps_report(stamps[k].cpu().numpy())
            elif k in stamps:
                from bench_roi_align import stamps_report
                stamps_report(stamps[k].cpu().numpy())
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(summary, f, indent=1)


if __name__ == '__main__':
    main()

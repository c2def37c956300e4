"""RoIAlign backward: the float-atomic form (frh_roi_align_bwd_strided, the default) against
the deterministic fixed-point form (frh_roi_align_bwd_fixed), µs per call including the
gradient clear / accumulator clear + conversion, on the fixed RoI sets of
tools/bench_roi_sets.py (cfg2 P2-P5, C = 256, channels-last gradients as the product trunk
makes them).  Also reports whether two deterministic calls -- the second on the RoIs in a
shuffled order -- give bit-identical gradients, and the largest difference to the atomic form.

    python tools/bench_roi_bwd.py [--sets bench,voc,train] [--iters 10]
Algorithmic bytes: 4*C*sum_K*49 gradient read + 2*4*C*sum H_l*W_l (clear +
accumulate once per cell)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tools'), os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from frcnn_amd import ops, _lib  # noqa: E402
from bench_roi_sets import load_set  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sets', default='bench,voc,train')
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--json')
    ap.add_argument('--variants', default='', help='tools backward variants (frh_roi_align_bwd_variant) beside the '
                    'product: 0 nhwc float, 1 register-resident float, 2 nhwc fixed, 3 register-resident fixed, 4 / 5 '
                    'readlane tap lists float / fixed')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    out = {}
    for name in args.sets.split(','):
        s = load_set(name, dev)
        if s is None:
            continue
        rois, levels, shapes, scales, feats = s
        K, B, C = rois.shape[0], shapes[0][0], shapes[0][1]
        g = torch.randn(K, C, 7, 7, device=dev, generator=torch.Generator(device=dev).manual_seed(3))
        hw, st = ops._feat_desc(feats)
        sc = _lib.f32_array(scales)

        def atomic():
            grads = [torch.zeros_like(f) for f in feats]
            _lib.call('frh_roi_align_bwd_strided', len(grads), _lib.ptr_array(grads), hw, st, sc, B, C,
                      _lib.ptr(rois), _lib.ptr(levels), K, 7, 7, 2, 0, _lib.ptr(g), _lib.stream_of(g))
            return grads

        word = torch.empty(1, dtype=torch.int32, device=dev)

        def fixed(r=rois, lv=levels, gg=g):
            grads = [torch.empty_like(f) for f in feats]
            accs = [torch.empty(f.shape, dtype=torch.int64, device=dev, memory_format=torch.channels_last).zero_()
                    for f in feats]
            _lib.call('frh_roi_align_bwd_fixed', len(grads), _lib.ptr_array(grads), _lib.ptr_array(accs), hw, st, sc,
                      B, C, _lib.ptr(r), _lib.ptr(lv), K, 7, 7, 2, 0, _lib.ptr(gg), _lib.ptr(word), _lib.stream_of(gg))
            return grads
        fns = [('atomic', atomic), ('fixed', fixed)]
        tools = None
        for v in [int(x) for x in args.variants.split(',') if x]:
            if tools is None:
                import toolslib
                tools = toolslib.load()

            def var(v=v):
                fx = v in (2, 3, 5, 12)
                grads = [torch.zeros_like(f) if not fx else torch.empty_like(f) for f in feats]
                accs = [torch.empty(f.shape, dtype=torch.int64, device=dev, memory_format=torch.channels_last).zero_()
                        for f in feats] if fx else grads
                rc = tools.frh_roi_align_bwd_variant(v, len(grads), _lib.ptr_array(grads), _lib.ptr_array(accs), hw, st,
                                                     sc, B, C, _lib.ptr(rois), _lib.ptr(levels), K, _lib.ptr(g),
                                                     _lib.ptr(word), _lib.stream_of(g))
                assert rc == 0, tools.frh_last_error()
                return grads
            fns.append(('v{}'.format(v), var))
        res = {}
        outs = {}
        for nm, fn in fns:
            outs[nm] = fn()
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[nm] = e0.elapsed_time(e1) * 1e3 / args.iters
        perm = torch.randperm(K, device=dev, generator=torch.Generator(device=dev).manual_seed(4))
        a, b = fixed(), fixed(rois[perm].contiguous(), levels[perm].contiguous(), g[perm].contiguous())
        at = atomic()
        same = all(torch.equal(x, y) for x, y in zip(a, b))
        diff = max(float((x - y).abs().max()) for x, y in zip(a, at))
        used = torch.unique(rois[:, 0].long() * 64 + levels).cpu().tolist()
        nbytes = 4 * C * (K * 49 + 2 * sum(shapes[u % 64][2] * shapes[u % 64][3] for u in used))
        for nm in res:
            if nm.startswith('v'):
                ref = outs['fixed' if int(nm[1:]) in (2, 3, 5, 12) else 'atomic']
                d = max(float((x - y).abs().max()) for x, y in zip(outs[nm], ref))
                print('  {}: {:.1f} us, max |diff| to the product form {:.3g}{}'.format(
                    nm, res[nm], d, ' (bit-identical)' if d == 0 else ''), flush=True)
        out[name] = {'atomic_us': res['atomic'], 'fixed_us': res['fixed'], 'fixed_bit_identical_permuted': same,
                     'variants_us': {k: v for k, v in res.items() if k.startswith('v')},
                     'max_abs_diff_fixed_vs_atomic': diff, 'algorithmic_bytes': nbytes}
        print('set {}: atomic {:.1f} us, deterministic {:.1f} us; deterministic bit-identical under a RoI '
              'permutation: {}; max |fixed - atomic| {:.3g}'.format(name, res['atomic'], res['fixed'], same, diff),
              flush=True)
    if args.json:
        json.dump(out, open(args.json, 'w'), indent=1)


if __name__ == '__main__':
    main()

"""RoIAlign forward laboratory: time the product kernel and candidate variants on the RoIs
and P2-P5 features of a real cfg2 forward pass.

    python tools/bench_roi_align.py [--variants 0,10] [--iters 20] [--rounds 3] [--cold]
Per variant: µs per launch back to back (warm: the features stay in L2 / Infinity Cache)
and, with --cold, after a 768 MB read that evicts both (difference of an evict+launch arm
and an evict-only arm); algorithmic GB/s (SURVEY §8(d) bytes); and whether the output is
bit-identical to the product kernel (variant 0).  Variant 1 (stamped product build)
prints the per-wave phase timeline.  --calib: known-byte launches for FETCH_SIZE
calibration (run under rocprofv3 --pmc FETCH_SIZE)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from frcnn_amd import ops, _lib, set_sampler_mode  # noqa: E402
import toolslib  # noqa: E402

STAMPED = {1, 9, 15}
STAMPED_NHWC = {6}  # channels-last stamped build: 8 int64 per 64-channel item
NHWC = set(range(2, 71)) | set(range(80, 100))  # channels-last kernels: run on channels_last copies of the same features


def calibrate(variants, dev, small=False):
    """Known-byte FETCH_SIZE calibration for this access pattern (MI355X_MICROARCH.md: only
    16-B/lane streaming reads are calibrated).  One RoI over a 29x29 map with 65536 channels:
    the 2x2-sampled 7x7 bins touch rows/cols 1..28 of every channel plane, i.e. every 128-B
    line of the 220 MB feature tensor (but the first of each plane's 3364 B), once.
    small=True: a 12x12 map of 262144 channels (151 MB) whose window takes the staged path."""
    lib = toolslib.load()
    C, S = (65536, 29) if not small else (262144, 12)
    rois = torch.tensor([[0.0, 0.0, 0.0, S - 1.0, S - 1.0]], device=dev)
    levels = torch.zeros(1, dtype=torch.int64, device=dev)
    print('calibration: feature bytes', C * S * S * 4, 'output bytes', C * 49 * 4, flush=True)
    for v in variants:
        feats = [torch.randn(1, C, S, S, device=dev)]
        if v in NHWC:
            feats = [f.contiguous(memory_format=torch.channels_last) for f in feats]
        hw, st = ops._feat_desc(feats)
        out = torch.empty(1, C, 7, 7, device=dev)
        ws = torch.empty(64, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        s = lib.frh_roi_align_fwd_variant(v, 1, _lib.ptr_array(feats), hw, st, _lib.f32_array([1.0]), 1, C,
                                          _lib.ptr(rois), _lib.ptr(levels), 1, 7, 7, 2, 0, _lib.ptr(out),
                                          _lib.ptr(ws), 64, _lib.stream_of(out))
        assert s == 0, lib.frh_last_error()
        torch.cuda.synchronize()
        print('variant', v, 'done', flush=True)


def stamps_report(stm):
    """Per-item stamps [start, setup done, first stage landed, end, D, cells, RoI record
    landed, xcd] (s_memrealtime, 100 MHz)."""
    stm = stm[stm[:, 0] > 0]
    t0 = stm[:, 0].min()
    span = (stm[:, 3].max() - t0) / 100.0
    print('  {} waves; span {:.1f} us'.format(len(stm), span))
    pc = lambda a: np.percentile(a / 100.0, [50, 90, 99]).round(2).tolist()  # noqa: E731
    for D in sorted(set(stm[:, 4].tolist())):
        x = stm[stm[:, 4] == D]
        if D < 0:  # the interleaved path (ilv_body) records only start and end: its phases are not stamped
            print('  D={} waves {:5d}: (phases not stamped) life {}'.format(D, len(x), pc(x[:, 3] - x[:, 0])))
            continue
        print('  D={} waves {:5d}: fetch {} taps {} land {} eval+rest {} life {}'.format(
            D, len(x), pc(x[:, 6] - x[:, 0]), pc(x[:, 1] - x[:, 6]), pc(x[:, 2] - x[:, 1]), pc(x[:, 3] - x[:, 2]),
            pc(x[:, 3] - x[:, 0])))
    alive = np.zeros(int(span) + 1)
    for a, b in zip((stm[:, 0] - t0) / 100.0, (stm[:, 3] - t0) / 100.0):
        alive[int(a):int(b) + 1] += 1
    print('  waves alive per CU by us: ' + ' '.join('%.1f' % (x / 256) for x in alive))
    print('  end-time percentiles 50/90/99/100:', np.percentile((stm[:, 3] - t0) / 100.0, [50, 90, 99, 100]).round(1).tolist(),
          flush=True)


def nhwc_stamps_report(stm):
    """[start, prologue done, first band landed, eval done, end, bands, first-band cells, xcd]"""
    stm = stm[stm[:, 0] > 0]
    t0 = stm[:, 0].min()
    pc = lambda a: np.percentile(a / 100.0, [50, 90, 99]).round(2).tolist()  # noqa: E731
    print('  {} waves; span {:.1f} us; start p50/90 {}'.format(len(stm), (stm[:, 4].max() - t0) / 100.0,
                                                          pc(stm[:, 0] - t0)[:2]))
    for nb in sorted(set(stm[:, 5].tolist())):
        x = stm[stm[:, 5] == nb]
        print('  bands={} waves {:5d} cells p50 {}: prologue {} land {} eval {} store {} life {}'.format(
            nb, len(x), int(np.median(x[:, 6])), pc(x[:, 1] - x[:, 0]), pc(x[:, 2] - x[:, 1]), pc(x[:, 3] - x[:, 2]),
            pc(x[:, 4] - x[:, 3]), pc(x[:, 4] - x[:, 0])), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--variants', default='0')
    ap.add_argument('--rounds', type=int, default=1)
    ap.add_argument('--cold', action='store_true')
    ap.add_argument('--after-write', action='store_true',
                    help='also time each launch right after the features are rewritten in place (x *= 1)')
    ap.add_argument('--calib', action='store_true')
    ap.add_argument('--calib-small', action='store_true')
    ap.add_argument('--dump', help='save the RoIs / levels / level shapes of the recorded launch to this .npz')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    variants = [int(x) for x in args.variants.split(',')]
    if args.calib:
        calibrate(variants, dev, args.calib_small)
        return
    set_sampler_mode('device', seed=1)
    model, batch = bench.make_model_and_batch(dev, batch=2)
    ops.ROI_ALIGN_PROFILE['on'] = True
    with torch.no_grad():
        model.forward_train(*batch)
    ops.ROI_ALIGN_PROFILE['on'] = False
    rec = ops.ROI_ALIGN_PROFILE['records'][-1]
    _, _, rois, levels, shapes, (ph, pw), feats, scales, sr = rec
    nbytes = bench.roi_align_bytes(rec)
    lv = levels.cpu().numpy()
    r = rois.cpu().numpy()
    side = np.sqrt((r[:, 3] - r[:, 1] + 1) * (r[:, 4] - r[:, 2] + 1))
    print('rois', r.shape[0], 'level hist', np.bincount(lv, minlength=4).tolist(),
          'side px p10/50/90', np.percentile(side, [10, 50, 90]).round(1).tolist(), 'bytes', nbytes, flush=True)
    if args.dump:
        np.savez(args.dump, rois=r, levels=lv, shapes=np.array(shapes), scales=np.array(scales))
    lib = toolslib.load()
    K, C = rois.shape[0], shapes[0][1]
    feats_cl = [f.contiguous(memory_format=torch.channels_last) for f in feats]
    hw, st = ops._feat_desc(feats)
    hw_cl, st_cl = ops._feat_desc(feats_cl)
    wsb = int(lib.frh_roi_align_workspace(K))
    wsp = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    scratch = torch.ones(768 * 2 ** 20 // 4, device=dev) if args.cold else None
    sink = torch.empty((), device=dev)
    ref = None
    summary = {}
    for v in variants * args.rounds:
        extra = (K * C // 16) * 16 if v in STAMPED else 0  # 8 int64 stamps per 16-channel item
        if v in STAMPED_NHWC:
            extra = (K * C // 64 + 8) * 16
        full = torch.zeros(K * C * ph * pw + extra, device=dev)
        out = full[:K * C * ph * pw].view(K, C, ph, pw)

        fv, hv, sv = (feats_cl, hw_cl, st_cl) if v in NHWC else (feats, hw, st)

        def launch():
            s = lib.frh_roi_align_fwd_variant(v, len(fv), _lib.ptr_array(fv), hv, sv, _lib.f32_array(scales),
                                              shapes[0][0], C, _lib.ptr(rois), _lib.ptr(levels), K, ph, pw, sr, 0,
                                              _lib.ptr(full), _lib.ptr(wsp), wsb, _lib.stream_of(out))
            assert s == 0, lib.frh_last_error()
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            launch()
        e1.record()
        torch.cuda.synchronize()
        warm = e0.elapsed_time(e1) / args.iters * 1e3
        cold = None
        if args.cold:
            arms = []
            for with_launch in (True, False):
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.iters):
                    torch.sum(scratch, dim=0, out=sink)
                    if with_launch:
                        launch()
                e1.record()
                torch.cuda.synchronize()
                arms.append(e0.elapsed_time(e1) * 1e3)
            cold = (arms[0] - arms[1]) / args.iters
        aw = None
        if args.after_write:  # does the Infinity Cache keep lines the trunk has just written?
            arms = []
            for with_launch in (True, False):
                torch.cuda.synchronize()
                e0.record()
                for _ in range(args.iters):
                    for f in fv:
                        f.mul_(1.0)
                    if with_launch:
                        launch()
                e1.record()
                torch.cuda.synchronize()
                arms.append(e0.elapsed_time(e1) * 1e3)
            aw = (arms[0] - arms[1]) / args.iters
            print('variant {:>3}: after a rewrite of the features {:7.2f} us'.format(v, aw), flush=True)
        summary.setdefault(v, []).append((warm, cold))
        if v in STAMPED:
            stamps_report(full[K * C * ph * pw:].view(torch.int64).view(-1, 8).cpu().numpy())
        if v in STAMPED_NHWC:
            nhwc_stamps_report(full[K * C * ph * pw:].view(torch.int64).view(-1, 8)[:K * C // 64].cpu().numpy())
        if ref is None:
            ref = out.clone()
        same = bool(torch.equal(out, ref))
        d = float((out - ref).abs().max())
        print('variant {:>3}: warm {:7.2f} us ({:6.0f} GB/s){}  bit-identical to variant {}: {} (max|diff| {:.3g})'.format(
            v, warm, nbytes / (warm * 1e-6) / 1e9,
            '' if cold is None else '  cold {:7.2f} us ({:6.0f} GB/s)'.format(cold, nbytes / (cold * 1e-6) / 1e9),
            variants[0], same, d), flush=True)
    if args.rounds > 1:
        print('median over {} rounds (us per launch, warm / cold):'.format(args.rounds))
        for v, xs in summary.items():
            w = float(np.median([x[0] for x in xs]))
            c = float(np.median([x[1] for x in xs])) if args.cold else float('nan')
            print('  variant {:>3}: {:7.2f} / {:7.2f}'.format(v, w, c))


if __name__ == '__main__':
    main()

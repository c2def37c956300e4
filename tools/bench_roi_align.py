"""Micro-benchmark of RoIAlign forward variants on the RoIs of a real cfg2 forward pass.

    python tools/bench_roi_align.py [--iters 50]
Prints per-variant average launch time (HIP events), algorithmic GB/s (SURVEY §8(d)
bytes) and the max |difference| to variant 0."""
import argparse, ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'tools'), REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd')]
import numpy as np, torch
import bench
from frcnn_amd import ops, _lib, set_sampler_mode  # noqa: E402
import toolslib  # noqa: E402


def calibrate(variants, dev, small=False):
    """Known-byte calibration of the FETCH_SIZE counter for this kernel's access pattern
    (MI355X_MICROARCH.md: only 16-B/lane streaming reads are calibrated).  One RoI over a
    29x29 map with 65536 channels: the 2x2-sampled 7x7 bins touch rows/cols 1..28 of every
    channel plane, i.e. every 128-B line of the 220 MB feature tensor (but the first of
    each plane's 3364 B), exactly once.  small=True: a 12x12 map of 262144 channels (151 MB)
    whose 12x13-float window takes the LDS-staged path of the default kernel; the large map
    takes its block-gather path.  Run under rocprofv3 --pmc FETCH_SIZE."""
    lib = toolslib.load()
    fn = lib.frh_roi_align_fwd_variant
    C, S = (65536, 29) if small is False else (262144, 12)
    rois = torch.tensor([[0.0, 0.0, 0.0, S - 1.0, S - 1.0]], device=dev)
    levels = torch.zeros(1, dtype=torch.int64, device=dev)
    print('calibration: feature bytes', C * S * S * 4, 'output bytes', C * 49 * 4, flush=True)
    for v in variants:
        feats = [torch.randn(1, C, S, S, device=dev)]  # fresh tensor per variant: no reuse across runs
        hw, st = ops._feat_desc(feats)
        out = torch.empty(1, C, 7, 7, device=dev)
        torch.cuda.synchronize()
        ws = torch.empty(64, dtype=torch.uint8, device=dev)
        s = fn(v, 1, _lib.ptr_array(feats), hw, st, _lib.f32_array([1.0]), 1, C, _lib.ptr(rois), _lib.ptr(levels),
               1, 7, 7, 2, 0, _lib.ptr(out), _lib.ptr(ws), 64, _lib.stream_of(out))
        assert s == 0, lib.frh_last_error()
        torch.cuda.synchronize()
        print('variant', v, 'done', flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--variants', default='0,10,50')
    ap.add_argument('--rounds', type=int, default=1, help='repeat the variant list; report medians of back-to-back replays')
    ap.add_argument('--calib', action='store_true', help='known-byte FETCH_SIZE calibration launches only')
    ap.add_argument('--calib-small', action='store_true', help='calibration on the staged (small-window) path')
    ap.add_argument('--sort', action='store_true',
                    help='order the RoIs by (image, level, 64-px tile) first (spatial locality experiment)')
    ap.add_argument('--dump', help='save the RoIs / levels / level shapes of the recorded launch to this .npz')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    if args.calib:
        calibrate([int(x) for x in args.variants.split(',')], dev, args.calib_small)
        return
    set_sampler_mode('device', seed=1)
    model, batch = bench.make_model_and_batch(dev, batch=2)
    ops.ROI_ALIGN_PROFILE['on'] = True
    model.forward_train(*batch)
    ops.ROI_ALIGN_PROFILE['on'] = False
    rec = ops.ROI_ALIGN_PROFILE['records'][-1]
    _, _, rois, levels, shapes, (ph, pw), feats, scales, sr = rec
    nbytes = bench.roi_align_bytes(rec)
    if args.sort:
        rr = rois.cpu().numpy()
        cx, cy = (rr[:, 1] + rr[:, 3]) / 2, (rr[:, 2] + rr[:, 4]) / 2
        key = ((rr[:, 0].astype(np.int64) * 8 + levels.cpu().numpy()) * 64 + (cy // 64).astype(np.int64)) * 64 + (cx // 64)
        perm = torch.from_numpy(np.argsort(key, kind='stable')).to(dev)
        rois, levels = rois[perm].contiguous(), levels[perm].contiguous()
    lv = levels.cpu().numpy()
    r = rois.cpu().numpy()
    side = np.sqrt((r[:, 3] - r[:, 1] + 1) * (r[:, 4] - r[:, 2] + 1))
    print('rois', r.shape[0], 'level hist', np.bincount(lv, minlength=4).tolist(),
          'side px p10/50/90', np.percentile(side, [10, 50, 90]).round(1).tolist(), 'bytes', nbytes)
    if args.dump:
        np.savez(args.dump, rois=r, levels=lv, shapes=np.array(shapes), scales=np.array(scales))
    lib = toolslib.load()
    K, C = rois.shape[0], shapes[0][1]
    hw, st = ops._feat_desc(feats)
    outs = {}
    wsb = int(lib.frh_roi_align_workspace(ctypes.c_int64(K)))
    wsp = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    summary = {}
    specs = args.variants.split(',') * args.rounds
    for spec in specs:
        v = int(spec)
        extra = 8 * 4096 * 8 if v == 51 else (K * C // 16 * 16 if v in (44, 45, 48) else 0)
        full = torch.zeros(K * C * ph * pw + extra, device=dev)  # stamps after
        out = full[:K * C * ph * pw].view(K, C, ph, pw)

        def launch():
            s = lib.frh_roi_align_fwd_variant(v, len(feats), _lib.ptr_array(feats), hw, st, _lib.f32_array(scales),
                                              shapes[0][0], C, _lib.ptr(rois), _lib.ptr(levels), K, ph, pw, sr, 0,
                                              _lib.ptr(full), _lib.ptr(wsp), wsb, _lib.stream_of(out))
            assert s == 0, lib.frh_last_error()
        for _ in range(5):
            launch()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); launch(); e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        ms = np.array([a.elapsed_time(b) for a, b in ts])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            launch()
        e1.record()
        torch.cuda.synchronize()
        summary.setdefault(spec, []).append(e0.elapsed_time(e1) / args.iters * 1e3)
        if v in (44, 45, 48):  # per-wave stamps [start, setup, landed, end, D, cells, roi, xcd] (s_memrealtime, 100 MHz)
            stm = full[K * C * ph * pw:].view(torch.int64).view(-1, 8).cpu().numpy()
            stm = stm[stm[:, 0] > 0]
            t0 = stm[:, 0].min()
            span = (stm[:, 3].max() - t0) / 100.0
            print('  {} waves; span {:.1f} us'.format(len(stm), span))
            for D in sorted(set(stm[:, 4].tolist())):
                x = stm[stm[:, 4] == D]
                pc = lambda a: np.percentile(a / 100.0, [50, 90, 99]).round(2).tolist()
                print('  D={} waves {:5d}: setup {} land {} eval+rest {} life {}'.format(
                    D, len(x), pc(x[:, 1] - x[:, 0]), pc(x[:, 2] - x[:, 1]), pc(x[:, 3] - x[:, 2]), pc(x[:, 3] - x[:, 0])),
                    flush=True)
            nb = int(span) + 1
            alive = np.zeros(nb)
            for a, b in zip((stm[:, 0] - t0) / 100.0, (stm[:, 3] - t0) / 100.0):
                i0, i1 = int(a), int(b)
                alive[i0:i1 + 1] += 1
            print('  waves alive per CU by us: ' + ' '.join('%.1f' % (x / 256) for x in alive), flush=True)
            ends = np.sort((stm[:, 3] - t0) / 100.0)
            print('  end-time percentiles 50/90/99/100:', np.percentile(ends, [50, 90, 99, 100]).round(1).tolist())
            late = stm[(stm[:, 3] - t0) / 100.0 > 0.9 * span]
            print('  last 10% of span: {} waves, D {} cells p50 {}'.format(
                len(late), np.bincount(late[:, 4]).tolist(), np.median(late[:, 5]) if len(late) else 0), flush=True)
        if v == 51:  # per-workgroup stamps [start, union, end, path | U << 8] (s_memrealtime, 100 MHz)
            allst = full[K * C * ph * pw:].view(torch.int64)
            steps = allst[8192:8192 + 128 * 20 * 4].view(64, 2, 20, 4).cpu().numpy()
            st = allst[:8192].view(-1, 4).cpu().numpy()
            st = st[st[:, 0] > 0]
            t0 = st[:, 0].min()
            dur, pro = (st[:, 2] - st[:, 0]) / 100.0, (st[:, 1] - st[:, 0]) / 100.0
            path = st[:, 3] & 255
            print('  {} workgroups; span {:.1f} us; start p50/90/max {}'.format(
                len(st), (st[:, 2].max() - t0) / 100.0, np.percentile((st[:, 0] - t0) / 100.0, [50, 90, 100]).round(1).tolist()))
            for wg in range(3):  # per-step timeline of waves 0 and 7: wait->barrier->eval done (us from WG start)
                for wv in (0, 1):
                    sw = steps[wg, wv]
                    sw = sw[sw[:, 0] > 0]
                    if len(sw):
                        b0 = st[wg, 0] if wg < len(st) else sw[0, 0]
                        print('  wg {} wave {} (B,D)={}: '.format(wg, 7 * wv, sw[0, 3]) + ' '.join(
                            '{:.1f}/{:.1f}/{:.1f}'.format((x[0] - b0) / 100, (x[1] - b0) / 100, (x[2] - b0) / 100)
                            for x in sw[:10]), flush=True)
            for pth in sorted(set(path.tolist())):
                m = path == pth
                print('  path {:3d}: n {:4d} dur p50/90/max {} prologue p50 {:.2f} U p50 {}'.format(
                    pth, m.sum(), np.percentile(dur[m], [50, 90, 100]).round(1).tolist(), np.median(pro[m]),
                    int(np.median(st[m, 3] >> 8))), flush=True)
        ref = outs[min(outs)] if outs else out
        outs[v] = out
        d = float((out - ref).abs().max())
        print('variant {:>4}: {:8.1f} us (min {:7.1f})  {:7.1f} GB/s algorithmic  max|diff| {:.3g}'.format(
            spec, ms.mean() * 1e3, ms.min() * 1e3, nbytes / (ms.mean() * 1e-3) / 1e9, d), flush=True)
        if d > 0:  # which RoIs differ: level, box, tap window of the scaled box
            per = (out - ref).abs().flatten(1).max(1).values.cpu().numpy()
            bad = np.nonzero(per > 0)[0]
            print('  {} RoIs differ; first: '.format(len(bad)), flush=True)
            for i in bad[:12]:
                sc = scales[lv[i]]
                bx = r[i, 1:] * sc
                print('   roi {} lvl {} box {} win w {:.1f} h {:.1f} maxdiff {:.3g} ch-diff {}'.format(
                    i, lv[i], r[i, 1:].round(1).tolist(), bx[2] - bx[0], bx[3] - bx[1], per[i],
                    int(((out[i] - ref[i]).abs().flatten(1).max(1).values > 0).sum())), flush=True)


    if args.rounds > 1:
        print('back-to-back replay, median over {} rounds (us per launch):'.format(args.rounds))
        for spec, v in summary.items():
            print('  variant {:>4}: {:7.2f}  (all: {})'.format(spec, float(np.median(v)), ' '.join('%.1f' % x for x in v)))


if __name__ == '__main__':
    main()

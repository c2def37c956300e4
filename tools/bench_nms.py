"""NMS laboratory: the RPN NMS call of a real cfg2 training step (10 segments of <= 2000
proposals), replayed with the product kernels and with the stamped scan build.

    python tools/bench_nms.py [--iters 20]
Prints µs per call (mask + scan, back to back) and, from the stamped build, the per-block
timeline of the scan of every segment: when the resolver started waiting for block b, when
b was ready (its staged span folded by a loader), when it was resolved, and when the
loader issued b's copies / published b's fold (µs from the launch's first stamp).  Then the
same for the RPN's one-launch NMS (nms_fused_kernel, the product's path inside
frh_rpn_proposals): µs per call, and per block of segment 0 when its column's last tile was
flagged, when the loader started / saw the column complete / published, when it was resolved."""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    set_sampler_mode('device', seed=1)
    model, batch = bench.make_model_and_batch(dev, batch=2)
    ops.NMS_PROFILE['on'] = True
    with torch.no_grad():
        model.forward_train(*batch)
    ops.NMS_PROFILE['on'] = False
    _, rows, cnt, P, thr, max_keep = ops.NMS_PROFILE['records'][-1]
    S = rows.shape[0]
    nbw = (P + 63) // 64
    print('segments', S, 'counts', cnt.cpu().tolist(), 'thr', thr, 'max_keep', max_keep, flush=True)
    lib = toolslib.load()
    ws = _lib.workspace(_lib.query('frh_nms_workspace', S, P), dev)
    keep = torch.empty(S, P, dtype=torch.int32, device=dev)
    kc = torch.empty(S, dtype=torch.int32, device=dev)
    stamps = torch.zeros(S * nbw * 8, dtype=torch.int64, device=dev)

    def plain():
        _lib.call('frh_nms_sorted', S, _lib.ptr(rows), rows.stride(0), _lib.ptr(cnt), P, thr, max_keep, _lib.ptr(keep),
                  keep.stride(0), _lib.ptr(kc), _lib.ptr(ws), ws.numel(), _lib.stream_of(rows))

    def stamped():
        s = lib.frh_nms_sorted_stamped(S, _lib.ptr(rows), rows.stride(0), _lib.ptr(cnt), P, thr, max_keep,
                                       _lib.ptr(keep), keep.stride(0), _lib.ptr(kc), _lib.ptr(ws), ws.numel(),
                                       _lib.ptr(stamps), _lib.stream_of(rows))
        assert s == 0, lib.frh_last_error()

    for fn, name in ((plain, 'product'), (stamped, 'stamped')):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print('{}: {:.2f} us per call (mask + scan)'.format(name, e0.elapsed_time(e1) / args.iters * 1e3), flush=True)
    ref_keep, ref_kc = keep.clone(), kc.clone()
    plain()
    torch.cuda.synchronize()
    assert torch.equal(kc, ref_kc) and all(torch.equal(keep[s, :int(kc[s])], ref_keep[s, :int(kc[s])]) for s in range(S))
    st = stamps.view(S, nbw, 8).cpu().numpy()
    t0 = st[:, :, :5][st[:, :, :5] > 0].min()
    counts = cnt.cpu().tolist()
    for s in range(S):
        nb = (counts[s] + 63) // 64
        x = (st[s, :nb, :5] - t0) / 100.0
        x[st[s, :nb, :5] == 0] = np.nan
        print('segment {} ({} boxes, {} kept): resolver done at {:.2f} us'.format(s, counts[s], int(kc[s]),
                                                                                   np.nanmax(x[:, 2])))
        per = np.diff(x[:, 2])
        print('  per block: wait->ready {:.2f}, ready->resolved {:.2f}, resolved-to-resolved {:.2f} (median us)'.format(
            float(np.nanmedian(x[:, 1] - x[:, 0])), float(np.nanmedian(x[:, 2] - x[:, 1])),
            float(np.nanmedian(per)) if len(per) else float('nan')))
        if s == 0:
            for b in range(nb):
                print('   b={:2d} wait {:6.2f} ready {:6.2f} resolved {:6.2f} | copies {:6.2f} fold {:6.2f}'.format(
                    b, *x[b, [0, 1, 2, 4, 3]]))

    # ---------------- the RPN's one-launch NMS (nms_fused_kernel)
    tri = nbw * (nbw + 1) // 2
    fws = _lib.workspace(_lib.query('frh_nms_workspace', S, P) + lib.frh_nms_fused_flag_bytes(S, P), dev)
    fst = torch.zeros(S * nbw * 8 + S * tri, dtype=torch.int64, device=dev)

    def fused(stm=None):
        r = lib.frh_nms_fused_stamped(S, _lib.ptr(rows), rows.stride(0), _lib.ptr(cnt), P, thr, max_keep,
                                      _lib.ptr(keep), keep.stride(0), _lib.ptr(kc),
                                      _lib.ptr(ops.status_word(dev)), _lib.ptr(fws), fws.numel(),
                                      _lib.ptr(stm), _lib.stream_of(rows))
        assert r == 0, lib.frh_last_error()
    for fn, name in ((fused, 'one-launch'), (lambda: fused(fst), 'one-launch stamped')):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print('{}: {:.2f} us per call (flag memset + kernel)'.format(name, e0.elapsed_time(e1) / args.iters * 1e3),
              flush=True)
        assert torch.equal(kc, ref_kc) and all(torch.equal(keep[s, :int(kc[s])], ref_keep[s, :int(kc[s])])
                                               for s in range(S))
    fs = fst.cpu().numpy()
    blk = fs[:S * nbw * 8].reshape(S, nbw, 8)
    til = fs[S * nbw * 8:].reshape(S, tri)
    t0 = min(blk[blk > 0].min(), til[til > 0].min())
    print('one-launch timeline (us from the first stamp): last tile flagged {:.2f}'.format((til.max() - t0) / 100.0))
    for s in range(S):
        nb = (counts[s] + 63) // 64
        x = (blk[s, :nb].astype(np.float64) - t0) / 100.0
        x[blk[s, :nb] == 0] = np.nan
        print('segment {} ({} boxes): resolver done at {:.2f}, last column complete {:.2f}'.format(
            s, counts[s], x[:, 3].max(), max(((til[s, c * (c + 1) // 2:c * (c + 1) // 2 + c + 1].max() - t0) / 100.0)
                                            for c in range(nb))))
        if s == 0:
            for b in range(nb):
                colc = (til[s, b * (b + 1) // 2:b * (b + 1) // 2 + b + 1].max() - t0) / 100.0
                print('   b={:2d} column flagged {:6.2f} | loader start {:6.2f} seen {:6.2f} last-batch wait {:6.2f} '
                      'got {:6.2f} published {:6.2f} | resolved {:6.2f}'.format(b, colc, *x[b, [0, 1, 4, 5, 2, 3]]))


if __name__ == '__main__':
    main()

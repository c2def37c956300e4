"""Timing of the one-launch selections (and the RPN's one-launch NMS) against their
multi-launch forms, with a phase timeline of the one-launch selection kernels (tools
library stamps).

    python tools/bench_select.py [--iters 50]

RPN proposals: the bench's cfg2 RPN head outputs (random-init model, channels-last) through
frh_rpn_proposals_strided (one-launch selection) and frh_rpn_proposals_launches (keys /
refine / collect / rank) and through frh_rpn_proposals_nms2 (one-launch selection, two-launch
NMS) and frh_rpn_proposals_merge_launch (the round-4 merge, rpn_merge_lds_kernel, after the
one-launch NMS instead of rpn_merge_wide_kernel), back to back between one event pair, µs per call (everything included); then one stamped call: per workgroup, s_memrealtime at the kernel's
phases, reported as medians relative to the workgroup's own start and to the launch's first
start.  Device sampler: the cfg2 RPN call's shape (2 x 155 520 anchors, 256 / 128) on
synthetic labels, the same three measurements.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

RPN_PHASES = ['start', 'keys+hist flushed', 'barrier 1 passed', 'bucket 1 found', 'hist 2 flushed',
              'barrier 2 passed', 'plan', 'slots reserved', 'selections decoded', 'barrier 3 passed',
              'ties loaded', 'ties sorted', 'records in LDS', 'ordered + stored']
SAMP_PHASES = ['start', 'keys + LDS hist', 'chunk hist stored', 'barrier 1 passed', 'plans', 'labels + lists',
               'barrier 2 passed', 'ties done', 'exit']


def timeline(stm, names):
    stm = stm.reshape(-1, 16)
    stm = stm[stm[:, 0] > 0]
    t0 = stm[:, 0].min()
    out = {}
    for q, nm in enumerate(names):
        col = stm[:, q]
        ok = col > 0
        if ok.sum() == 0:
            continue
        out[nm] = {'rel_wg_start_us': round(float(np.median((col[ok] - stm[ok, 0]) / 100.0)), 2),
                   'rel_launch_us_median': round(float(np.median((col[ok] - t0) / 100.0)), 2),
                   'rel_launch_us_max': round(float(((col[ok] - t0) / 100.0).max()), 2), 'wgs': int(ok.sum())}
    return out


def time_calls(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    args = ap.parse_args()
    import bench
    import toolslib
    from frcnn_amd import ops, _lib
    dev = torch.device('cuda', 0)
    lib = toolslib.load()
    res = {}

    # ---------------- RPN proposals on the bench's head outputs
    model, _ = bench.make_model(dev, seed=0)
    imgs = bench.make_batch(dev, 2, seed=0)[0]
    with torch.no_grad():
        feats = model.extract_feat(imgs)
        cls, reg = model.rpn_head(feats)
    head = model.rpn_head
    grids = [(c.shape[2], c.shape[3]) for c in cls]
    anchors = head._flat_anchors(grids, dev)
    argv = (cls, reg, anchors, head.num_anchors, 1, [0.0] * 4, [1.0] * 4, [(600.0, 1000.0)] * 2, [0.0] * 2,
            2000, 2000, 2000, 0.7)
    one = time_calls(lambda: ops.rpn_proposals(*argv), args.iters)
    four = time_calls(lambda: ops.rpn_proposals(*argv, _entry=(lib.frh_rpn_proposals_launches, 'launches')),
                      args.iters)
    nms2 = time_calls(lambda: ops.rpn_proposals(*argv, _entry=(lib.frh_rpn_proposals_nms2, 'nms2')), args.iters)
    mlaunch = time_calls(lambda: ops.rpn_proposals(*argv, _entry=(lib.frh_rpn_proposals_merge_launch, 'merge_launch')),
                         args.iters)
    gx = max(max((3 * h * w + 4095) // 4096, (2000 + 63) // 64) for h, w in grids)
    stm = torch.zeros(2 * len(grids), gx, 16, dtype=torch.int64, device=dev)

    def stamped(*a):
        a = list(a)
        stream = a.pop()
        return lib.frh_rpn_proposals_stamped(*a, _lib.ptr(stm), stream)
    ops.rpn_proposals(*argv, _entry=(stamped, 'stamped'))
    torch.cuda.synchronize()
    sa = stm.cpu().numpy()
    L = len(grids)
    nch0 = (3 * grids[0][0] * grids[0][1] + 4095) // 4096
    # the one-launch NMS (timing build): per segment, when its scan resolved its last block,
    # µs from the launch's first stamp
    S, P = 2 * len(grids), 2000
    nbw = (P + 63) // 64
    tri = nbw * (nbw + 1) // 2
    nst = torch.zeros(S * nbw * 8 + S * tri, dtype=torch.int64, device=dev)

    def nstamped(*a):
        a = list(a)
        stream = a.pop()
        return lib.frh_rpn_proposals_nms_stamped(*a, _lib.ptr(nst), stream)
    ops.rpn_proposals(*argv, _entry=(nstamped, 'nms_stamped'))
    torch.cuda.synchronize()
    na = nst.cpu().numpy()
    blk = na[:S * nbw * 8].reshape(S, nbw, 8)
    t0 = na[na > 0].min()
    res['nms_scan_resolved_last_us'] = [round(float((blk[sg, :, 3][blk[sg, :, 3] > 0].max() - t0) / 100.0), 2)
                                        if (blk[sg, :, 3] > 0).any() else None for sg in range(S)]
    res['rpn_proposals'] = {'us_per_call_one_launch_select': round(one, 2),
                            'us_per_call_four_launch_select': round(four, 2),
                            'us_per_call_two_launch_nms': round(nms2, 2),
                            'us_per_call_lds_merge': round(mlaunch, 2),
                            'timeline_one_launch_select': timeline(sa, RPN_PHASES),
                            'timeline_level0_key_workgroups': timeline(sa[0::L, :nch0], RPN_PHASES),
                            'timeline_level4': timeline(sa[L - 1::L], RPN_PHASES)}

    # ---------------- device sampler, cfg2 RPN shape
    S, n = 2, sum(3 * h * w for h, w in grids)
    rng = np.random.default_rng(0)
    lab = torch.from_numpy(rng.choice([-1, 0, 1, 2], size=(S, n), p=[0.3, 0.6995, 0.0003, 0.0002])
                           .astype(np.int64)).to(dev)
    num = torch.tensor([n] * S, dtype=torch.int32, device=dev)
    ops.set_sampler_mode('device', seed=5)
    one = time_calls(lambda: ops.sample_labels(lab, num, n, 256, 128, mode='device', lists=True), args.iters)
    two = time_calls(lambda: ops.sample_labels(lab, num, n, 256, 128, mode='device', lists=True,
                                               _entry=(lib.frh_sample_random_launches, 'launches')), args.iters)
    sst = torch.zeros(S, (n + 4095) // 4096, 16, dtype=torch.int64, device=dev)

    def sstamped(*a):
        a = list(a)
        stream = a.pop()
        return lib.frh_sample_random_stamped(*a, _lib.ptr(sst), stream)
    ops.sample_labels(lab, num, n, 256, 128, mode='device', lists=True, _entry=(sstamped, 'stamped'))
    torch.cuda.synchronize()
    res['sampler'] = {'us_per_call_one_launch': round(one, 2), 'us_per_call_two_launches': round(two, 2),
                      'timeline_one_launch': timeline(sst.cpu().numpy(), SAMP_PHASES)}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()

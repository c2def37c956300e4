"""Diagnostic: does forward_train depend on state carried between calls or on the
contents of uninitialised memory?

  python tools/diag_state.py [--config cascade_rcnn_r50_fpn] [--sync-free 0|1]

1. poison: torch.empty / empty_like (every Python caller, the frcnn_amd ops and
   workspaces included) return buffers filled with a byte pattern (0x00, 0xff, 0x7f);
   the same forward_train (same sampler stream) must give bit-identical losses.
   Per-op outputs are captured, and the first op call whose outputs differ is named.
2. sequence: forward_train(batch 1) fresh, then batch 0 forward+backward, then
   batch 1 again with the sampler stream reset: bit-identical losses.
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd'), os.path.join(REPO, 'tests', 'golden')]
import bench  # noqa: E402
import frcnn_amd  # noqa: E402
from frcnn_amd import ops  # noqa: E402

_empty, _empty_like = torch.empty, torch.empty_like
PATTERN = [None]


def _fill(t):
    if PATTERN[0] is not None and t.is_cuda and t.numel() and t.is_contiguous():
        t.view(-1).view(torch.uint8).fill_(PATTERN[0])
    return t


def p_empty(*a, **k):
    return _fill(_empty(*a, **k))


def p_empty_like(*a, **k):
    return _fill(_empty_like(*a, **k))


torch.empty, torch.empty_like = p_empty, p_empty_like

CAP = {'on': False, 'log': []}
OPS = ['maxiou_assign', 'sample_labels', 'anchor_target_batched', 'gather_level_outputs', 'prepend_gt_labels',
       'bbox_target_batched', 'rpn_proposals', 'roi_rows', 'roi_rows_dev', 'roi_align_multilevel', 'det_losses',
       'pack_boxes', 'pack_labels', 'param2bbox', 'bbox2param']


def _flat(x):
    if torch.is_tensor(x):
        return [x.detach().clone()]
    if isinstance(x, ops.SampleLists):
        # selection lists in no order: compare sorted valid prefixes
        sel, cnt = x.sel.detach(), x.sel_counts.detach().cpu()
        out = []
        for s in range(sel.shape[0]):
            for w in range(2):
                out.append(torch.sort(sel[s, w, :int(cnt[s, w])])[0].clone())
        return out + [x.sel_counts.detach().clone()]
    if isinstance(x, dict):
        return [v for k in sorted(x) for v in _flat(x[k])]
    if isinstance(x, (list, tuple)):
        return [v for e in x for v in _flat(e)]
    return []


def _wrap(name):
    f = getattr(ops, name)

    def g(*a, **k):
        r = f(*a, **k)
        if CAP['on']:
            CAP['log'].append((name, _flat(r)))
        return r
    setattr(ops, name, g)


for _n in OPS:
    _wrap(_n)


def run(model, batch, seed, backward=False):
    ops._SAMPLER.update({'mode': 'device', 'seed': seed, 'calls': 0})
    CAP['log'] = []
    CAP['on'] = True
    ls = model.forward_train(*batch)
    CAP['on'] = False
    if backward:
        sum(ls.values()).backward()
    torch.cuda.synchronize()
    return {k: float(v) for k, v in ls.items()}, CAP['log']


def diff_logs(la, lb, tag):
    first = None
    for i, ((na, ta), (nb, tb)) in enumerate(zip(la, lb)):
        assert na == nb, (na, nb)
        for j, (x, y) in enumerate(zip(ta, tb)):
            if x.shape != y.shape:
                print('  [{}] call {} {} out {}: shape {} vs {}'.format(tag, i, na, j, tuple(x.shape), tuple(y.shape)))
                first = first or (i, na)
                continue
            xe, ye = x.reshape(-1), y.reshape(-1)
            if x.is_floating_point():
                bad = ~((xe == ye) | (torch.isnan(xe) & torch.isnan(ye)))
            else:
                bad = xe != ye
            nb_ = int(bad.sum())
            if nb_:
                idx = bad.nonzero().view(-1)
                print('  [{}] call {} {} out {} shape {}: {} differ, first flat idx {} last {} ({} vs {})'.format(
                    tag, i, na, j, tuple(x.shape), nb_, int(idx[0]), int(idx[-1]), xe[idx[0]].item(),
                    ye[idx[0]].item()))
                first = first or (i, na)
    return first


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='cascade_rcnn_r50_fpn')
    ap.add_argument('--sync-free', type=int, default=-1, help='-1: the model default; 0/1: force the RPN choice')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    frcnn_amd.set_sampler_mode('device', seed=1)
    model, _ = bench.make_model(dev, seed=0, config=os.path.join(bench.CONFIG_DIR, args.config + '.py'))
    if args.sync_free >= 0 and hasattr(model.rpn_head, 'allow_sync_free'):
        model.rpn_head.allow_sync_free = bool(args.sync_free)
    b0 = bench.make_batch(dev, 2, seed=0, rank=0)
    b1 = bench.make_batch(dev, 2, seed=0, rank=1)
    print('config', args.config, 'rpn sync-free', getattr(model.rpn_head, 'allow_sync_free', None))
    # 1. poison
    res = {}
    for pat in (0x00, 0xff, 0x7f):
        PATTERN[0] = pat
        res[pat] = run(model, b1, 1235)
        print('pattern 0x{:02x}'.format(pat), res[pat][0])
    PATTERN[0] = None
    for pat in (0xff, 0x7f):
        same = res[pat][0] == res[0][0]
        print('poison 0x00 vs 0x{:02x}: losses {}'.format(pat, 'EQUAL' if same else 'DIFFER'))
        f = diff_logs(res[0][1], res[pat][1], '00/{:02x}'.format(pat))
        print('  first differing op call:', f)
    # 2. sequence
    model.zero_grad(set_to_none=True)
    a = run(model, b1, 1235)
    run(model, b0, 1234, backward=True)
    junk = torch.full((64 << 20,), float('nan'), device=dev)  # dirty 256 MB of the allocator
    del junk
    b = run(model, b1, 1235)
    print('sequence fresh', a[0])
    print('sequence after', b[0])
    print('sequence: losses {}'.format('EQUAL' if a[0] == b[0] else 'DIFFER'))
    f = diff_logs(a[1], b[1], 'seq')
    print('  first differing op call:', f)


if __name__ == '__main__':
    main()

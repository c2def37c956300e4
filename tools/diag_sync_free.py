"""Diagnostic: sync-free vs synced RCNN stage on cfg2 (losses, counts, RoI rows, features, head outputs)."""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from frcnn_amd import set_sampler_mode, ops  # noqa: E402

dev = torch.device('cuda', 0)
model, _ = bench.make_model(dev, seed=0)
imgs, boxes, labels, metas = bench.make_batch(dev, 2, seed=1)
seen = {0: {}, 1: {}}
cur = [0]


def wrap(mod, name, key, pick):
    f = getattr(mod, name)

    def g(*a, **k):
        r = f(*a, **k)
        seen[cur[0]][key] = pick(a, r)
        return r
    setattr(mod, name, g)


cl = lambda t: t.detach().clone()  # noqa: E731
wrap(ops, 'roi_rows', 'rows', lambda a, r: cl(r[0]))
wrap(ops, 'roi_rows_dev', 'rows', lambda a, r: cl(r[0]))
wrap(ops, 'roi_align_multilevel', 'feat', lambda a, r: cl(r))
wrap(ops, 'bbox_target_batched', 'bt', lambda a, r: {k: cl(v) for k, v in r.items() if torch.is_tensor(v)})
wrap(ops, 'sample_labels', 'samp%d' % 0, lambda a, r: r)
out = []
for mode in (0, 1):
    cur[0] = mode
    if mode:
        model.rpn_head.sync_free = lambda *a: False
        model._sync_free_rcnn = lambda *a: False
    set_sampler_mode('device', seed=21)
    with torch.no_grad():
        ls = model.forward_train(imgs, boxes, labels, metas)
    out.append({k: float(v) for k, v in ls.items()})
print(out)
A, B = seen[0], seen[1]
n = B['rows'].shape[0]
print('rows', A['rows'].shape, B['rows'].shape, 'rows diff', float((A['rows'][:n] - B['rows']).abs().max()))
print('feat diff', float((A['feat'][:n] - B['feat']).abs().max()))
for k in B['bt']:
    a, b = A['bt'][k], B['bt'][k]
    if a.dim() == 2:
        a = a[:, :b.shape[1]]
    elif k != 'n_dev' and k != 'counts_dev':
        a = a[:b.shape[0]]
    if a.shape == b.shape:
        print('bt', k, a.shape, float((a.double() - b.double()).abs().max()))
print('counts', A['bt'].get('counts_dev'), A['bt'].get('n_dev'))
bad = (A['rows'][:n] - B['rows']).abs().max(1)[0] > 0
print('bad rows', int(bad.sum()), bad.nonzero().view(-1)[:10].tolist())
i = bad.nonzero().view(-1)[:3]
print(A['rows'][i].tolist(), B['rows'][i].tolist())

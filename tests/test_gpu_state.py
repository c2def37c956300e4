"""State carried between forward_train calls in one process (round-3 review item): per-stream
workspaces whose counters every call must leave at zero (ops._ASSIGN_WS: the one-launch
MaxIoU colmax / arrivals / candidate count; ops._LOSS_WS: the fused losses' arrival
counter), the memoised gt packs (ops._PACKED), the heads' anchor / mask caches, the sampler
call counter -- and uninitialised memory (torch.empty outputs and workspaces).

For the sync-free graphs (cfg2: RPN + RCNN; cfg4: the RPN targets, its cascade stages keep
the per-image lists) and their synced twins:
  1. forward_train(batch B) from a fresh state (workspaces, packs and caches cleared);
  2. forward_train + backward of another batch A (other gt counts: the assignment
     workspace changes layout), then 256 MB of the caching allocator NaN-filled and freed;
  3. forward_train(B) again on the same sampler stream, with every torch.empty the Python
     side makes (ops outputs and kernel workspaces included) filled with 0xff bytes.
The losses of 1 and 3 must be bit-identical.  The trunk's convolutions run with MIOpen's
deterministic immediate mode (cudnn.deterministic) so that the comparison sees the
detection path only."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _clear(model):
    from frcnn_amd import ops
    ops._ASSIGN_WS.clear()
    ops._LOSS_WS.clear()
    ops._SAMPLE_WS.clear()
    del ops._PACKED[:]
    for head in (getattr(model, 'rpn_head', None), getattr(model, 'bbox_head', None)):
        if head is not None:
            head._anchor_cache.clear()
            head._mask_cache.clear()


@pytest.mark.parametrize('config,sync_free', [('faster_rcnn_r50_fpn', True), ('faster_rcnn_r50_fpn', False),
                                              ('cascade_rcnn_r50_fpn', True), ('cascade_rcnn_r50_fpn', False)])
def test_consecutive_calls_bit_identical(dev, monkeypatch, config, sync_free):
    import bench
    from frcnn_amd import set_sampler_mode
    flags = (torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic)
    torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = False, True
    try:
        model, _ = bench.make_model(dev, seed=0, config=os.path.join(bench.CONFIG_DIR, config + '.py'))
        if not sync_free:
            model.rpn_head.sync_free = lambda *a: False
            model._sync_free_rcnn = lambda *a: False
        else:
            assert model.rpn_head.allow_sync_free
        batch_a = bench.make_batch(dev, 2, seed=0, rank=0)
        batch_b = bench.make_batch(dev, 2, seed=0, rank=1)
        assert [b.shape[1] for b in batch_a[1]] != [b.shape[1] for b in batch_b[1]]

        def run(batch, backward=False):
            set_sampler_mode('device', seed=77)
            ls = model.forward_train(*batch)
            if backward:
                sum(ls.values()).backward()
            torch.cuda.synchronize()
            return {k: float(v) for k, v in ls.items()}

        _clear(model)
        fresh = run(batch_b)
        run(batch_a, backward=True)
        junk = torch.full((64 << 20,), float('nan'), device=dev)
        del junk
        empty, empty_like = torch.empty, torch.empty_like

        def fill(t):
            if t.is_cuda and t.numel() and t.is_contiguous():
                t.view(-1).view(torch.uint8).fill_(0xff)
            return t
        monkeypatch.setattr(torch, 'empty', lambda *a, **k: fill(empty(*a, **k)))
        monkeypatch.setattr(torch, 'empty_like', lambda *a, **k: fill(empty_like(*a, **k)))
        again = run(batch_b)
        monkeypatch.undo()
        assert fresh == again, (fresh, again)
    finally:
        torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = flags

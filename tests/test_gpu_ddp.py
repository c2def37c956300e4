"""Data-parallel training of the REAL detector on the HIP path: two `gloo` ranks share
cuda:0 (a one-GPU box cannot run two RCCL ranks), each running frcnn_amd.train.TrainStep
(DistributedDataParallel, bucketed gradient all-reduce) on the cfg4 Cascade R-CNN
(configs/cascade_rcnn_r50_fpn.py: 3 RCNN stages, refine, per-stage stds) with its own
2-image shard, for two iterations (a parameter DDP never saw a gradient for would fail
the second iteration's reduction).  Both ranks must hold identical parameters after each
iteration, and the first iteration's update must equal (to float-atomic tolerance: the
RoIAlign backward and MIOpen's backward convolutions sum in run-dependent order) one
single-process iteration on the rank-averaged gradient -- the reference's train_one_iter
(lib/trainer/trainer.py:100-127, hooks.py:55-59) with DDP averaging.  (Later iterations
are not compared with the reference: a last-bit difference in the updated weights can
flip the RPN's near-tied random-init scores, i.e. which proposals are selected.)"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CONFIG = 'cascade_rcnn_r50_fpn'
STEPS = 2
WORLD = 2


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(dev):
    import bench
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    model, cfg = bench.make_model(dev, seed=0, config=os.path.join(bench.CONFIG_DIR, CONFIG + '.py'))
    return model, cfg


def _worker(rank, world, port, q):
    try:
        import sys
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [repo, os.path.join(repo, 'pytorch-faster-rcnn_amd'), os.path.join(repo, 'tests', 'golden')]
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        dist.init_process_group('gloo', rank=rank, world_size=world)
        import bench
        import frcnn_amd
        from frcnn_amd.train import TrainStep
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        frcnn_amd.set_sampler_mode('device', seed=1234 + rank)
        model, cfg = _setup(dev)
        batch = bench.make_batch(dev, 2, seed=0, rank=rank)
        step = TrainStep(model, cfg.optimizer, cfg.optimizer_config.get('grad_clip'), world, dev, bucket_mb=25)
        import hashlib
        losses, snaps = [], []
        for it in range(STEPS):  # the first iteration's parameters in full, later ones as digests
            losses.append(float(step(*batch)))
            ps = [p.detach().cpu().numpy() for p in model.parameters()]
            snaps.append(ps if it == 0 else [hashlib.sha256(x.tobytes()).hexdigest() for x in ps])
        torch.cuda.synchronize()
        q.put((rank, losses, snaps))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on the queue
        import traceback
        q.put((rank, None, traceback.format_exc()[-3000:] + repr(e)))


def _reference(dev):
    """One iteration in one process on the rank-averaged gradient; each rank's device
    sampler stream is replayed (seed 1234 + rank, its own call counter)."""
    import bench
    from frcnn_amd import ops
    from frcnn_amd.train import build_optimizer
    model, cfg = _setup(dev)
    params = [p for p in model.parameters() if p.requires_grad]
    opt = build_optimizer(params, cfg.optimizer)
    clip = cfg.optimizer_config.get('grad_clip')
    batches = [bench.make_batch(dev, 2, seed=0, rank=r) for r in range(WORLD)]
    samplers = [{'mode': 'device', 'seed': 1234 + r, 'calls': 0} for r in range(WORLD)]
    saved = dict(ops._SAMPLER)
    losses = [[] for _ in range(WORLD)]
    try:
        for _ in range(1):
            opt.zero_grad(set_to_none=True)
            for r in range(WORLD):
                ops._SAMPLER.clear()
                ops._SAMPLER.update(samplers[r])
                loss = sum(model.forward_train(*batches[r]).values())
                (loss / WORLD).backward()
                samplers[r] = dict(ops._SAMPLER)
                losses[r].append(float(loss))
            if clip:
                torch.nn.utils.clip_grad_norm_(params, clip['max_norm'], clip.get('norm_type', 2))
            opt.step()
    finally:
        ops._SAMPLER.clear()
        ops._SAMPLER.update(saved)
    torch.cuda.synchronize()
    return losses, [p.detach().cpu().numpy() for p in model.parameters()]


def test_cascade_ddp_two_gloo_ranks_on_one_gpu(dev):
    import torch.multiprocessing as mp
    flags = (torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        out = sorted((q.get(timeout=240) for _ in procs), key=lambda x: x[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, losses, snaps in out:
        assert losses is not None, 'rank {} failed:\n{}'.format(rank, snaps)
    for p in procs:
        assert p.exitcode == 0
    (_, l0, s0), (_, l1, s1) = out
    try:
        ref_losses, ref = _reference(dev)
        init, _ = _setup(dev)
        init = [p.detach().cpu().numpy() for p in init.parameters()]
    finally:
        torch.backends.cudnn.benchmark, torch.backends.cudnn.deterministic = flags
    assert all(np.isfinite(l0)) and all(np.isfinite(l1)) and l0[0] != l1[0]  # each rank's own shard
    np.testing.assert_allclose([l0[0], l1[0]], [ref_losses[0][0], ref_losses[1][0]], rtol=1e-4)
    for it in range(STEPS):
        for a, b in zip(s0[it], s1[it]):
            if it == 0:
                np.testing.assert_array_equal(a, b)  # one all-reduced gradient: ranks stay in lock step
            else:
                assert a == b
    moved = 0
    for a, r, i in zip(s0[0], ref, init):
        d, dr = a - i, r - i  # the first update agrees to float-atomic summation noise
        scale = max(float(np.abs(dr).max()), 1e-12)
        assert float(np.abs(d - dr).max()) <= 1e-2 * scale + 1e-9, (float(np.abs(d - dr).max()), scale)
        moved += int(np.abs(dr).max() > 0)
    assert moved > len(ref) // 2

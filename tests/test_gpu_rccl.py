"""RCCL readiness on a one-GPU box: a world-size-1 `nccl` process group (RCCL on
ROCm) initialised with `device_id`, and frcnn_amd.train.TrainStep with DistributedDataParallel
forced on (`force_ddp`) for two cfg2 iterations -- DDP's bucketed gradient all-reduce runs
through RCCL -- against the plain (non-DDP) TrainStep of a copy of the same model on the same
device-sampler stream.  Under torch.use_deterministic_algorithms (MIOpen's deterministic
backward convolutions, the RoIAlign backward's fixed-point form) the losses and every
parameter after each iteration must be equal BIT FOR BIT: an all-reduce over one rank and the
/ 1 average are exact.  Reference loop: lib/trainer/trainer.py:100-127 (single process,
train.py:117-120); the data-parallel exchange is this build's own (§8(e)).

Runs in a spawned process so the test process never holds an RCCL communicator."""
import copy
import hashlib
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 2


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    try:
        import sys
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [repo, os.path.join(repo, 'pytorch-faster-rcnn_amd'), os.path.join(repo, 'tests', 'golden')]
        import torch.distributed as dist
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK='0', WORLD_SIZE='1')
        dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
        backend = dist.get_backend()
        import bench
        from frcnn_amd import set_sampler_mode
        from frcnn_amd.train import TrainStep
        torch.backends.cudnn.benchmark = False
        torch.backends.cudnn.deterministic = True
        torch.use_deterministic_algorithms(True, warn_only=True)
        model, cfg = bench.make_model(dev, seed=0)
        batch = bench.make_batch(dev, 2, seed=0, rank=0)
        ref_model = copy.deepcopy(model)
        clip = cfg.optimizer_config.get('grad_clip')

        def run(m, force):
            set_sampler_mode('device', seed=1234)
            step = TrainStep(m, cfg.optimizer, clip, 1, dev, bucket_mb=25, force_ddp=force)
            losses, digests = [], []
            for _ in range(STEPS):
                losses.append(float(step(*batch)))
                digests.append([hashlib.sha256(p.detach().cpu().numpy().tobytes()).hexdigest()
                                for p in m.parameters()])
            return type(step.net).__name__, losses, digests

        ref = run(ref_model, False)
        ddp = run(model, True)
        torch.cuda.synchronize()
        # one explicit collective on the communicator too: a device tensor all-reduced over RCCL
        t = torch.arange(1024, dtype=torch.float32, device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        q.put(dict(backend=backend, ref=ref, ddp=ddp, allreduce_ok=bool(torch.equal(
            t, torch.arange(1024, dtype=torch.float32, device=dev)))))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on the queue
        import traceback
        q.put(traceback.format_exc()[-3000:] + repr(e))


def test_world1_nccl_ddp_train_step_equals_plain_step(dev):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    try:
        res = q.get(timeout=400)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert isinstance(res, dict), res
    assert p.exitcode == 0
    assert res['backend'] == 'nccl'
    assert res['allreduce_ok']
    rname, rl, rd = res['ref']
    dname, dl, dd = res['ddp']
    assert rname == 'DetectorLoss' and dname == 'DistributedDataParallel'
    assert all(map(lambda v: v == v, rl)), rl  # finite (not NaN)
    assert rl == dl, (rl, dl)
    for it in range(STEPS):
        assert rd[it] == dd[it], it
    assert rd[0] != rd[1]  # the iterations moved the parameters

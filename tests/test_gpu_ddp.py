"""Data-parallel training of the REAL detectors on the HIP path: two `gloo` ranks share
cuda:0 (a one-GPU box cannot run two RCCL ranks), each running frcnn_amd.train.TrainStep
(DistributedDataParallel, bucketed gradient all-reduce) on its own 2-image shard for two
iterations (a parameter DDP never saw a gradient for fails the second iteration's
reduction), for
  * cfg4 Cascade R-CNN (configs/cascade_rcnn_r50_fpn.py: 3 RCNN stages, refine, per-stage
    stds; reference lib/detectors/cascade_rcnn.py:90-154), and
  * cfg5 ATSS (configs/fcos_r50_fpn_atss.py: FCOSHead with centerness, trainable level
    coefficients, GIoU; reference lib/detectors/fcos.py:42-57, lib/heads/fcos_head.py:525-568).

The reference iteration is computed IN EACH WORKER PROCESS, before its DDP step, on a deep
copy of the same model: the plain (non-DDP) forward_train + backward of the rank's shard on
the same device-sampler stream, the gradients averaged over ranks with one all-reduce of
their concatenation, then clip_grad_norm_ and SGD -- the reference's train_one_iter
(lib/trainer/trainer.py:100-127, hooks.py:55-59) on the rank-averaged gradient.  Checks:
  * each rank's DDP loss equals its own reference loss (the forward is the same
    computation in the same process);
  * after the first iteration every parameter equals the reference update BIT FOR BIT:
    the workers run with torch.use_deterministic_algorithms (which also selects the RoIAlign
    backward's fixed-point form, frh_roi_align_bwd_fixed, instead of float atomics) and
    cudnn.deterministic (MIOpen's deterministic backward convolutions); two ranks' sum and
    the / 2 average are exact in either order, so DDP's bucketed all-reduce matches the
    reference's one all-reduce of the concatenated gradient;
  * the ranks hold identical parameters after every iteration.

Why the reference runs in the worker and not in the test process: a second process is
not guaranteed the same convolution solutions (MIOpen's immediate mode reads a find
database that other processes may have updated), and a last-bit difference in the trunk's
outputs can flip which of the near-tied random-init RPN scores are selected -- round 3's
version of this test, which replayed both ranks in the pytest process, saw rank 1's loss
1.2e-3 away from the replay with the synced and the sync-free RPN targets alike, while
in-process replays of the same calls are bit-identical under poisoned workspaces
(tests/test_gpu_state.py, tools/diag_state.py)."""
import copy
import hashlib
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 2
WORLD = 2


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reference_step(model, cfg, batch, world, seed):
    """One plain iteration on a copy of `model`: returns (loss, updated trainable params)."""
    import torch.distributed as dist
    from frcnn_amd import set_sampler_mode
    from frcnn_amd.train import build_optimizer
    ref = copy.deepcopy(model)
    params = [p for p in ref.parameters() if p.requires_grad]
    opt = build_optimizer(params, cfg.optimizer)
    set_sampler_mode('device', seed=seed)
    loss = sum(ref.forward_train(*batch).values())
    loss.backward()
    grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
    flat = torch.cat([g.reshape(-1) for g in grads]).cpu()
    dist.all_reduce(flat)
    flat /= world
    off = 0
    for p in params:
        n = p.numel()
        # the averaged gradient in the parameter's own layout (channels-last conv weights keep
        # their strides: the gradient layout contract, which the fused SGD step requires)
        p.grad = torch.empty_like(p).copy_(flat[off:off + n].view(p.shape))
        off += n
    clip = cfg.optimizer_config.get('grad_clip')
    if clip:
        torch.nn.utils.clip_grad_norm_(params, clip['max_norm'], clip.get('norm_type', 2))
    opt.step()
    return float(loss), [p.detach().cpu().numpy() for p in ref.parameters()]


def _worker(rank, world, port, q, config):
    try:
        import sys
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [repo, os.path.join(repo, 'pytorch-faster-rcnn_amd'), os.path.join(repo, 'tests', 'golden')]
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        dist.init_process_group('gloo', rank=rank, world_size=world)
        import bench
        from frcnn_amd import set_sampler_mode
        from frcnn_amd.train import TrainStep
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        torch.backends.cudnn.benchmark = False
        torch.backends.cudnn.deterministic = True
        torch.use_deterministic_algorithms(True, warn_only=True)  # + the RoIAlign backward's fixed-point form
        model, cfg = bench.make_model(dev, seed=0, config=os.path.join(bench.CONFIG_DIR, config + '.py'))
        batch = bench.make_batch(dev, 2, seed=0, rank=rank)
        init = [p.detach().cpu().numpy() for p in model.parameters()]
        ref_loss, ref_params = _reference_step(model, cfg, batch, world, 1234 + rank)
        set_sampler_mode('device', seed=1234 + rank)  # the same sampler stream for the DDP step
        step = TrainStep(model, cfg.optimizer, cfg.optimizer_config.get('grad_clip'), world, dev, bucket_mb=25)
        losses, digests, first = [], [], None
        for it in range(STEPS):
            losses.append(float(step(*batch)))
            ps = [p.detach().cpu().numpy() for p in model.parameters()]
            digests.append([hashlib.sha256(x.tobytes()).hexdigest() for x in ps])
            if it == 0:
                first = ps
        torch.cuda.synchronize()
        # first update vs the reference update (0 under the deterministic algorithms)
        worst, moved = 0.0, 0
        for a, r, i in zip(first, ref_params, init):
            d, dr = a - i, r - i
            scale = max(float(np.abs(dr).max()), 1e-12)
            worst = max(worst, float(np.abs(d - dr).max()) / scale)
            moved += int(np.abs(dr).max() > 0)
        exact = all(np.array_equal(a, r) for a, r in zip(first, ref_params))
        q.put((rank, dict(losses=losses, ref_loss=ref_loss, digests=digests, worst=worst, moved=moved,
                          nparams=len(first), exact=exact)))
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on the queue
        import traceback
        q.put((rank, traceback.format_exc()[-3000:] + repr(e)))


@pytest.mark.parametrize('config', ['cascade_rcnn_r50_fpn', 'fcos_r50_fpn_atss'])
def test_ddp_two_gloo_ranks_on_one_gpu(dev, config):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, config)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        out = sorted((q.get(timeout=300) for _ in procs), key=lambda x: x[0])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, res in out:
        assert isinstance(res, dict), 'rank {} failed:\n{}'.format(rank, res)
    for p in procs:
        assert p.exitcode == 0
    r0, r1 = out[0][1], out[1][1]
    assert all(np.isfinite(r0['losses'])) and all(np.isfinite(r1['losses']))
    assert r0['losses'][0] != r1['losses'][0]  # each rank's own shard
    for r in (r0, r1):
        np.testing.assert_allclose(r['losses'][0], r['ref_loss'], rtol=1e-6)
        assert r['exact'], r['worst']  # round 4: |update - reference| <= 1e-2 x its scale (float atomics)
        assert r['moved'] > r['nparams'] // 2
    for it in range(STEPS):  # one all-reduced gradient: the ranks stay in lock step
        assert r0['digests'][it] == r1['digests'][it], it

"""Data-parallel training iteration (frcnn_amd.train.TrainStep) on CPU with a world_size-2
`gloo` group -- the GPU run is the same code over RCCL.  A stand-in detector (the real one's
HIP ops need a GPU) exposes the reference's forward_train(img, gt_bboxes, gt_labels,
img_metas) -> loss dict; after one step both ranks must hold identical parameters equal to
one clipped SGD step on the rank-averaged gradient (the reference's
lib/trainer/trainer.py:100-127 + hooks.py:55-59 semantics with DDP averaging)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

OPT = dict(type='SGD', lr=0.1, momentum=0.9, weight_decay=1e-4)
CLIP = dict(max_norm=0.5, norm_type=2)


class TinyDetector(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.backbone = nn.Linear(6, 4)
        self.head = nn.Linear(4, 2)
        self.frozen = nn.Linear(2, 2)
        for p in self.frozen.parameters():
            p.requires_grad = False

    def forward_train(self, img, gt_bboxes, gt_labels, img_metas):
        f = self.head(torch.relu(self.backbone(img.flatten(1))))
        cls = ((f[:, 0] - gt_labels.float()) ** 2).mean()
        reg = (f[:, 1] - gt_bboxes.sum(1)).abs().mean()
        return {'cls_loss': cls, 'reg_loss': reg}


def _batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return (torch.randn(3, 2, 3, generator=g), torch.randn(3, 4, generator=g),
            torch.randint(0, 5, (3,), generator=g), [{}] * 3)


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from frcnn_amd.train import TrainStep
    det = TinyDetector()
    step = TrainStep(det, OPT, CLIP, world_size=world, device=torch.device('cpu'), bucket_mb=1)
    loss = step(*_batch(rank))
    q.put((rank, float(loss), [p.detach().numpy().copy() for p in det.parameters()]))  # numpy: no shm handles
    dist.destroy_process_group()


def _expected(world):
    from frcnn_amd.train import build_optimizer
    det = TinyDetector()
    params = [p for p in det.parameters() if p.requires_grad]
    grads = [torch.zeros_like(p) for p in params]
    for r in range(world):
        det.zero_grad()
        sum(det.forward_train(*_batch(r)).values()).backward()
        for g, p in zip(grads, params):
            g += p.grad / world
    for g, p in zip(grads, params):
        p.grad = g
    nn.utils.clip_grad_norm_(params, CLIP['max_norm'], CLIP['norm_type'])
    build_optimizer(params, OPT).step()
    return [p.detach() for p in det.parameters()]


def test_two_rank_ddp_step_matches_averaged_gradient_step():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=120) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, l0, p0), (_, l1, p1) = out
    assert l0 != l1  # each rank's loss is its own shard's
    ref = _expected(2)
    for a, b, r in zip(p0, p1, ref):
        a, b = torch.from_numpy(a), torch.from_numpy(b)
        assert torch.equal(a, b)  # ranks stay in sync
        torch.testing.assert_close(a, r, rtol=1e-6, atol=1e-7)
    assert torch.equal(torch.from_numpy(p0[4]), TinyDetector().frozen.weight.detach())  # frozen: untouched


def test_single_process_step_is_plain_sgd():
    from frcnn_amd.train import TrainStep
    det = TinyDetector()
    step = TrainStep(det, OPT, None)
    before = [p.detach().clone() for p in det.parameters()]
    step(*_batch(0))
    assert any(not torch.equal(a, b) for a, b in zip(before, det.parameters()))

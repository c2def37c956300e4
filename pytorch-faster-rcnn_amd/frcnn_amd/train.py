"""One training iteration of the reference trainer, data-parallel over ranks.

Reference: `BasicTrainer.train_one_iter` (`lib/trainer/trainer.py:100-127`):
forward_train -> sum of the loss dict -> backward -> `OptimizerHook` gradient clipping
(`lib/trainer/hooks.py:55-59`, `clip_grad_norm_(max_norm, norm_type)`) -> SGD step, with
the optimizer of the config (`configs/faster_rcnn_r50_fpn.py:111-112`: SGD lr 0.0025,
momentum 0.9, weight decay 1e-4, grad_clip max_norm 35).

The reference is single-process (`README.md:8`, `train.py:117-120`).  Here each rank is
one process per GPU holding its own image shard; the only exchange is the gradient
all-reduce, done by DistributedDataParallel's bucketed all-reduce over RCCL (`nccl`
backend on ROCm) while backward runs, averaged over ranks.  Losses stay normalised per
rank (avg_factor of the local batch, `lib/heads/anchor_head.py:129`,
`lib/heads/bbox_head.py:62`), which equals the reference's per-iteration semantics at
imgs_per_gpu images per rank.  BN is frozen (eval-mode statistics, `lib/backbones.py:241-247`),
so no SyncBN and no buffer broadcast.
"""
import torch
from torch import nn

from . import ops

# Gradient bucket size for the all-reduce.  cfg2 has 41 M trainable f32 parameters
# (165 MB): 25 MB buckets give ~7 all-reduces that start while backward is still
# producing the earlier layers' gradients, and each is large enough to keep RCCL's
# channels over the 7 xGMI links busy.
DEFAULT_BUCKET_MB = 25


class DetectorLoss(nn.Module):
    """forward(*batch) = sum of forward_train's loss dict (what DDP wraps)."""

    def __init__(self, detector):
        super().__init__()
        self.detector = detector

    def forward(self, img, gt_bboxes, gt_labels, img_metas):
        losses = self.detector.forward_train(img, gt_bboxes, gt_labels, img_metas)
        return sum(losses.values())


def build_optimizer(params, cfg):
    """The reference's optimizer dict (type SGD) -> torch optimizer.  HIP parameters take the
    fused SGD kernel (one launch; it also honours a device `found_inf` flag, which TrainStep uses
    to skip a failed step's update without a host sync)."""
    cfg = dict(cfg or dict(type='SGD', lr=0.0025, momentum=0.9, weight_decay=0.0001))
    kind = cfg.pop('type')
    if kind != 'SGD':
        raise ValueError('unsupported optimizer type {}'.format(kind))
    params = list(params)
    if params and all(p.is_cuda for p in params):
        cfg.setdefault('fused', True)
    return torch.optim.SGD(params, **cfg)


class TrainStep:
    """Callable training iteration on this rank's batch; returns the (detached) local loss.

    Device status word (include/frcnn_amd.h FRH_DEVERR_*), with no host synchronisation:
      * the loss kernels read it, so a step whose in-launch wait ran out returns NaN losses
        (the reference's loop reads every loss each iteration, `lib/trainer/trainer.py:110-119`);
      * the fused SGD step takes `found_inf` = (word != 0), so that step's update is skipped on
        the device (momentum buffers are zero-initialised, so even a skipped first step leaves
        them defined);
      * the word is copied to pinned host memory after each step and the NEXT call raises
        (ops.check_device_status) once that copy has landed -- a finished event query, not a wait.
    `status_every=k` adds a synchronous check every k-th step before the update (0: never).

    `force_ddp` wraps the detector in DistributedDataParallel even at world size 1 (the RCCL
    readiness check on a one-GPU box: the bucketed all-reduce runs, over one rank)."""

    def __init__(self, detector, optimizer_cfg=None, grad_clip=None, world_size=1, device=None,
                 bucket_mb=DEFAULT_BUCKET_MB, status_every=0, force_ddp=False):
        self.detector = detector
        self.params = [p for p in detector.parameters() if p.requires_grad]
        if device is None and self.params:
            device = self.params[0].device
        self.device = torch.device(device) if device is not None else None
        self.status_every, self.steps = status_every, 0
        net = DetectorLoss(detector)
        if world_size > 1 or force_ddp:
            dev = self.device
            ids = [dev] if dev is not None and dev.type == 'cuda' else None
            net = nn.parallel.DistributedDataParallel(net, device_ids=ids, bucket_cap_mb=bucket_mb,
                                                      gradient_as_bucket_view=True, broadcast_buffers=False)
        self.net = net
        self.optimizer = build_optimizer(self.params, optimizer_cfg)
        self.grad_clip = dict(grad_clip) if grad_clip else None
        self._hip = self.device is not None and self.device.type == 'cuda'
        self._guard = self._hip and all(g.get('fused') for g in self.optimizer.param_groups)
        if self._guard:
            for g in self.optimizer.param_groups:
                if g.get('momentum', 0) != 0:
                    for p in g['params']:
                        self.optimizer.state[p]['momentum_buffer'] = torch.zeros_like(p)
            self._found = torch.zeros(1, dtype=torch.float32, device=self.device)
            self.optimizer.found_inf = self._found
        self._host_status = torch.zeros(1, dtype=torch.int32).pin_memory() if self._hip else None
        self._status_event = None

    def _lagged_check(self):
        """Raise if the previous step's status copy has landed and is nonzero (no wait)."""
        ev = self._status_event
        if ev is not None and ev.query():
            self._status_event = None
            if int(self._host_status[0]):
                ops.check_device_status(self.device)  # the word is still set: raises, clears it

    def __call__(self, img, gt_bboxes, gt_labels, img_metas):
        if self._hip:
            self._lagged_check()
        self.optimizer.zero_grad(set_to_none=True)
        loss = self.net(img, gt_bboxes, gt_labels, img_metas)
        loss.backward()
        if self.grad_clip:
            nn.utils.clip_grad_norm_(self.params, self.grad_clip['max_norm'],
                                     self.grad_clip.get('norm_type', 2))
        self.steps += 1
        if self.status_every and self.steps % self.status_every == 0 and self._hip:
            ops.check_device_status(self.device)  # synchronous: raises before a failed step's update
        if self._guard:
            self._found.copy_(ops.status_word(self.device).ne(0))  # device-side: no sync
        self.optimizer.step()
        if self._hip:
            self._host_status.copy_(ops.status_word(self.device), non_blocking=True)
            self._status_event = torch.cuda.Event()
            self._status_event.record()
        return loss.detach()

"""Detection losses (reference lib/losses.py), sum reductions.

On HIP tensors FocalLoss, CrossEntropyLoss and SmoothL1Loss run the fused loss
kernels (csrc/losses.hip): one streaming pass forward and one
backward instead of a dozen elementwise torch passes.  The torch expressions
below are the reference restatement; they serve CPU tensors and are the
numerics reference of the GPU tests.  Semantics follow the reference, including
its quirk that FocalLoss ignores the configured alpha/gamma/loss_weight
(losses.py:106-109).
"""
import torch
import torch.nn.functional as F
from torch import nn

from . import ops, utils


def zero_loss(device):
    return torch.zeros((), device=device, requires_grad=True)


def smooth_l1_loss_v2(x, y, beta):
    """losses.py:77-83: sum of 0.5 d^2 / beta (d < beta) or d - 0.5 beta."""
    if beta <= 0 or x.shape != y.shape:
        raise AssertionError('bad smooth-l1 arguments')
    d = torch.abs(x - y)
    small = (d < beta).float()
    return (small * (d ** 2) / (2 * beta) + (1 - small) * (d - 0.5 * beta)).sum()


def sigmoid_focal_loss(pred, target, alpha=0.25, gamma=2.0, fix_alpha=False):
    """losses.py:33-61: pred [n, C] logits, target [n] in 0..C (0 = background)."""
    n, c = pred.shape
    onehot = utils.one_hot_embedding(target, c + 1)[:, 1:].to(pred.dtype)
    p = pred.sigmoid()
    pt = p * onehot + (1 - p) * (1 - onehot)
    w = alpha if fix_alpha else alpha * onehot + (1 - alpha) * (1 - onehot)
    w = w * (1 - pt).pow(gamma)
    return (F.binary_cross_entropy_with_logits(pred, onehot, reduction='none') * w).sum()


def giou_loss(a, b):
    """losses.py:13-30: 1 - GIoU on [4, n] boxes (no +1 widths)."""
    tl = torch.max(a[:2], b[:2])
    br = torch.min(a[2:], b[2:])
    area_i = torch.prod(br - tl, dim=0) * (tl < br).all(0).float()
    area_a = torch.prod(a[2:] - a[:2], dim=0)
    area_b = torch.prod(b[2:] - b[:2], dim=0)
    area_u = area_a + area_b - area_i
    iou = area_i / area_u
    lo = torch.min(a[:2], b[:2])
    hi = torch.max(a[2:], b[2:])
    area_c = torch.prod(hi - lo, dim=0)
    return 1 - (iou - (area_c - area_u) / area_c)


class FocalLoss(nn.Module):
    def __init__(self, alpha=0.25, gamma=2.0, use_sigmoid=True, loss_weight=1.0):
        if not use_sigmoid:
            raise AssertionError('FocalLoss for non sigmoid is not implemented')
        super().__init__()
        self.use_sigmoid = True
        self.alpha, self.gamma, self.loss_weight = 0.25, 2.0, 1.0  # reference ignores the cfg values

    def forward(self, pred, target):
        if pred.is_cuda:
            return self.loss_weight * ops.cls_loss(pred, target, ops.CLS_FOCAL, self.alpha, self.gamma)
        return self.loss_weight * sigmoid_focal_loss(pred, target, self.alpha, self.gamma)


class SmoothL1Loss(nn.Module):
    def __init__(self, beta=1.0, loss_weight=1.0):
        super().__init__()
        self.beta, self.loss_weight = beta, loss_weight

    def forward(self, x, y):
        if x.is_cuda and x.dim() == 2:
            return self.loss_weight * ops.smooth_l1_loss(x, y, self.beta)
        return self.loss_weight * smooth_l1_loss_v2(x, y, self.beta)

    def masked(self, x, y, label, rows_dim=0):
        """Sum over the rows with label > 0 only (the reference's positive-row selection,
        anchor_head.py:126-128, without its boolean-index host sync)."""
        if x.is_cuda:
            return self.loss_weight * ops.smooth_l1_loss(x, y, self.beta, label, rows_dim)
        m = (label > 0).view(-1, 1) if rows_dim == 0 else (label > 0).view(1, -1)
        z = x.new_zeros(())
        return self.loss_weight * smooth_l1_loss_v2(torch.where(m, x, z), torch.where(m, y, z), self.beta)

    def class_selected(self, reg_out, num_classes, target, label):
        """bbox_head.py:70-76: the labelled class's deltas of reg_out [n, 4*C] at the positive rows."""
        if reg_out.is_cuda:
            return self.loss_weight * ops.smooth_l1_class_select(reg_out, num_classes, target, label, self.beta)
        n = len(label)
        sel = reg_out.view(-1, 4, num_classes)[torch.arange(n), :, label]
        return self.masked(sel, target, label, 0)


class CrossEntropyLoss(nn.Module):
    def __init__(self, use_sigmoid=False, loss_weight=1.0):
        super().__init__()
        self.use_sigmoid, self.loss_weight = use_sigmoid, loss_weight

    def forward(self, pred, label):
        c = pred.shape[1]
        if pred.is_cuda:
            if self.use_sigmoid:
                kind = ops.CLS_SIGMOID_BCE
                label = label.reshape(-1)  # C == 1: label.view(-1, 1).float() is the target itself
            else:
                kind = ops.CLS_SOFTMAX_CE
            return ops.cls_loss(pred, label, kind) * self.loss_weight
        if self.use_sigmoid:
            if c == 1:
                tgt = label.view(-1, 1).float()
            else:
                tgt = utils.one_hot_embedding(label, c + 1)[:, 1:].to(pred.dtype)
            return F.binary_cross_entropy_with_logits(pred, tgt, reduction='none').sum() * self.loss_weight
        return F.cross_entropy(pred, label, reduction='none').sum() * self.loss_weight


def fused_kinds(loss_cls, loss_bbox):
    """True when head_losses can run this pair of loss modules as one launch."""
    return isinstance(loss_bbox, SmoothL1Loss) and isinstance(loss_cls, (FocalLoss, CrossEntropyLoss))


def head_losses(loss_cls, loss_bbox, cls_x, cls_label, l1_args, avg_factor, div_count=None):
    """(loss_cls(cls_x, cls_label) / avg_factor, loss_bbox.<masked | class_selected>(...) /
    avg_factor) as ONE HIP launch (ops.det_losses) when both modules are the HIP-backed
    kinds, the tensors are on the GPU and avg_factor is a host number (the sampled count);
    l1_args() builds the regression loss's arguments.  None when it does not apply (the
    caller then runs the modules one by one).  div_count (device int32 [1]) replaces
    avg_factor for sync-free targets: padding rows (label -1) are ignored."""
    if div_count is not None:
        if not (cls_x.is_cuda and fused_kinds(loss_cls, loss_bbox)):
            raise AssertionError('sync-free targets need the fused HIP head losses')
        avg_factor = div_count
    elif not (cls_x.is_cuda and isinstance(loss_bbox, SmoothL1Loss)) or isinstance(avg_factor, torch.Tensor):
        return None
    if isinstance(loss_cls, FocalLoss):
        kind, alpha, gamma = ops.CLS_FOCAL, loss_cls.alpha, loss_cls.gamma
    elif isinstance(loss_cls, CrossEntropyLoss):
        kind, alpha, gamma = (ops.CLS_SIGMOID_BCE if loss_cls.use_sigmoid else ops.CLS_SOFTMAX_CE), 0.25, 2.0
    else:
        return None
    return ops.det_losses(cls_x, cls_label.reshape(-1), kind, alpha, gamma, loss_cls.loss_weight, l1_args(),
                          loss_bbox.beta, loss_bbox.loss_weight, avg_factor)


class GIoULoss(nn.Module):
    def __init__(self, loss_weight=1.0):
        super().__init__()
        self.loss_weight = loss_weight

    def forward(self, a, b, weight=None, avg_factor=1.0):
        loss = giou_loss(a, b)
        if weight is not None:
            loss = loss * weight
        return loss.sum() * self.loss_weight / avg_factor


class IoULoss(nn.Module):
    def __init__(self, loss_weight=1.0):
        super().__init__()
        self.loss_weight = loss_weight

    def forward(self, a, b, weight=None, avg_factor=None):
        loss = -utils.elem_iou(a, b).log()
        if weight is not None:
            loss = loss * weight
        if avg_factor is not None:
            loss = loss / avg_factor
        return loss.sum() * self.loss_weight


def generalized_focal_loss(pred, tar, beta=2.0):
    """losses.py:221-224 (elementwise, logits pred)."""
    focal_weight = (tar - pred.sigmoid()).abs().pow(beta)
    return focal_weight * F.binary_cross_entropy_with_logits(pred, tar, reduction='none')


class QualityFocalLoss(nn.Module):
    """losses.py:226-249: pred [n, C] logits, quality [n], label [n] in 0..C."""

    def __init__(self, beta=2.0, use_sigmoid=True, loss_weight=1.0):
        if not use_sigmoid:
            raise AssertionError('QualityFocalLoss only support sigmoid activation')
        super().__init__()
        self.use_sigmoid, self.beta, self.loss_weight = use_sigmoid, beta, loss_weight

    def forward(self, pred, quality, label, weight=None, avg_factor=1.0):
        n, n_cls = pred.shape
        tar = pred.new_zeros((n, n_cls + 1))
        tar[torch.arange(n, device=pred.device), label] = quality
        loss = generalized_focal_loss(pred, tar[:, 1:], beta=self.beta)
        if weight is not None:
            loss = loss * weight
        return loss.sum() * self.loss_weight / avg_factor


def log_softmax_with_logits(logits):
    """losses.py:251-254: row-wise stable log-softmax."""
    c, _ = logits.detach().max(1)
    s = logits - c.unsqueeze(1)
    return s - s.exp().sum(1).log().unsqueeze(1)


class DistributionFocalLoss(nn.Module):
    """losses.py:256-285: pred [n, cls_channels] logits, y [n], left_idx [n]."""

    def __init__(self, cls_channels, stride, norm_prob, loss_weight=1.0):
        super().__init__()
        self.cls_channels, self.stride, self.norm_prob, self.loss_weight = cls_channels, stride, norm_prob, loss_weight

    def forward(self, pred, y, left_idx, weight=None, avg_factor=1.0):
        n = pred.shape[0]
        ar = torch.arange(n, device=pred.device)
        log_sigma = log_softmax_with_logits(pred)
        right_idx = left_idx + 1
        y_left, y_right = left_idx * self.stride, right_idx * self.stride
        loss = (y_right - y) * log_sigma[ar, left_idx] + (y - y_left) * log_sigma[ar, right_idx]
        if self.norm_prob:
            loss = loss / self.stride
        return -loss.sum() * self.loss_weight / avg_factor

"""Static-shape trunk captured as one HIP graph.

The reference runs the ResNet/FPN backbone, the neck and the RPN head's convs as
~190 eagerly dispatched kernels per step (``cascade_rcnn.py:90-100``:
``extract_feat`` then ``rpn_head(feats)``).  Their shapes depend only on the
padded batch shape, so the trunk's forward is captured once into a hipGraph and
replayed with a single launch behind one autograd node whose backward
recomputes the trunk eagerly (checkpointing; the train step does not use the
graph).  The host is then free to run ahead into the data-dependent detection path instead of spending
~25 us of dispatch per conv / epilogue kernel.

Replays use the convolution algorithms chosen before the capture, so graphed
and eager trunks agree within MIOpen's f32 solver differences (a captured call
may take another solver;
``tests/test_gpu_parity.py::test_graphed_trunk_matches_eager``).  Any batch whose
shape, dtype or device differs from the captured one takes the eager path.
"""
import torch
from torch import nn


class Trunk(nn.Module):
    """backbone -> neck -> RPN head convs as one module with a flat tensor output:
    (feats..., rpn_cls..., rpn_reg...), ``L`` levels each."""

    def __init__(self, backbone, neck, rpn_head):
        super().__init__()
        self.backbone = backbone
        self.neck = neck
        self.rpn_head = rpn_head

    def forward(self, img):
        feats = self.backbone(img)
        if self.neck is not None:
            feats = self.neck(feats)
        feats = list(feats) if isinstance(feats, (list, tuple)) else [feats]
        cls_outs, reg_outs = self.rpn_head(feats)
        return tuple(feats) + tuple(cls_outs) + tuple(reg_outs)


def split_trunk_outputs(outs):
    n = len(outs) // 3
    return list(outs[:n]), list(outs[n:2 * n]), list(outs[2 * n:])


class _TrunkReplay(torch.autograd.Function):
    """Forward = one graph replay; backward = the trunk's eager backward on a recomputed
    forward (activation checkpointing), so the outputs carry correct gradients without
    capturing the backward convolutions (whose MIOpen algorithm search would otherwise run
    inside the capture)."""

    @staticmethod
    def forward(ctx, owner, img, *params):
        owner.replay(img)
        ctx.owner = owner
        ctx.save_for_backward(img)
        return tuple(o.detach() for o in owner.static_out)

    @staticmethod
    def backward(ctx, *grads):
        owner = ctx.owner
        (img,) = ctx.saved_tensors
        x = img.detach().requires_grad_(img.requires_grad)
        with torch.enable_grad():
            outs = owner.trunk(x)
        pairs = [(o, g) for o, g in zip(outs, grads) if g is not None and o.requires_grad]
        wrt = ([x] if x.requires_grad else []) + list(owner.params)
        got = torch.autograd.grad([o for o, _ in pairs], wrt, [g for _, g in pairs], allow_unused=True)
        gimg = got[0] if x.requires_grad else None
        return (None, gimg) + tuple(got[1:] if x.requires_grad else got)


class GraphedTrunk:
    """The trunk's forward for one input shape captured as a hipGraph; ``matches(img)``
    says whether a batch can replay it."""

    def __init__(self, trunk, sample_img, num_warmup_iters=3):
        if not sample_img.is_cuda:
            raise RuntimeError('GraphedTrunk needs a HIP tensor (got {})'.format(sample_img.device))
        self.shape = tuple(sample_img.shape)
        self.dtype = sample_img.dtype
        self.device = sample_img.device
        self.trunk = trunk
        self.params = tuple(p for p in trunk.parameters() if p.requires_grad)
        self.static_in = sample_img.detach().clone()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side), torch.no_grad():
            for _ in range(num_warmup_iters):
                trunk(self.static_in)
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.static_out = trunk(self.static_in)

    def matches(self, img):
        return (img.is_cuda and tuple(img.shape) == self.shape and img.dtype == self.dtype
                and img.device == self.device)

    def replay(self, img):
        if img.data_ptr() != self.static_in.data_ptr():
            self.static_in.copy_(img)
        self.graph.replay()

    def __call__(self, img):
        if torch.is_grad_enabled():
            outs = _TrunkReplay.apply(self, img, *self.params)
        else:
            self.replay(img)
            outs = tuple(o.detach() for o in self.static_out)
        return split_trunk_outputs(outs)


def capture_trunk(detector, sample_img, num_warmup_iters=3):
    """Capture ``detector``'s backbone + neck + RPN head convs for ``sample_img``'s shape and
    attach it (``detector.graphed_trunk``).  Call after any convolution-algorithm search
    (``torch.backends.cudnn.benchmark`` warmup): the capture freezes the chosen kernels."""
    neck = detector.neck if getattr(detector, 'with_neck', False) else None
    trunk = Trunk(detector.backbone, neck, detector.rpn_head)
    torch.cuda.synchronize(sample_img.device)
    detector.graphed_trunk = GraphedTrunk(trunk, sample_img, num_warmup_iters)
    torch.cuda.synchronize(sample_img.device)
    return detector.graphed_trunk


def release_trunk(detector):
    detector.graphed_trunk = None

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
shape, dtype or device differs from the captured one takes the eager path, and so
does every batch after the trunk's parameters or buffers were moved, cast or
replaced (the graph has their capture-time storage baked in).

Output lifetime: every replay rewrites the same graph-owned output buffers.  Each
replay bumps their autograd version counter, so a backward through outputs of an
earlier replay raises instead of silently using the newer data, and
``GraphedTrunk.replays`` / ``is_current(t)`` tell a caller whether a kept output
is still the latest.  Callers that keep outputs across steps (gradient
accumulation, profiling records) pass ``clone_outputs=True`` to get private copies.
"""
import torch
from torch import nn
from torch.autograd.graph import increment_version


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

    def __init__(self, trunk, sample_img, num_warmup_iters=3, clone_outputs=False):
        if not sample_img.is_cuda:
            raise RuntimeError('GraphedTrunk needs a HIP tensor (got {})'.format(sample_img.device))
        self.shape = tuple(sample_img.shape)
        self.dtype = sample_img.dtype
        self.device = sample_img.device
        self.trunk = trunk
        self.clone_outputs = clone_outputs
        self.replays = 0
        self.params = tuple(p for p in trunk.parameters() if p.requires_grad)
        self._slots = self._state_slots()
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

    def _state_slots(self):
        """Every (owning dict, name, object, storage pointer) the capture baked in: the
        trunk's submodules, parameters and buffers.  ``.to()``/``.half()``/``.cuda()``
        give a tensor new storage; assigning a new Parameter, buffer or submodule
        replaces the dict entry; either makes ``matches`` fail."""
        slots = []
        for mod in self.trunk.modules():
            for d in (mod._modules, mod._parameters, mod._buffers):
                for n, x in d.items():
                    if x is not None:
                        slots.append((d, n, x, x.data_ptr() if torch.is_tensor(x) else 0))
        return slots

    def state_unchanged(self):
        for d, n, x, ptr in self._slots:  # ~0.2 us per entry: one dict lookup + pointer compare
            if d.get(n) is not x or (ptr and x.data_ptr() != ptr):
                return False
        return True

    def matches(self, img):
        return (img.is_cuda and tuple(img.shape) == self.shape and img.dtype == self.dtype
                and img.device == self.device and self.state_unchanged())

    def replay(self, img):
        if img.data_ptr() != self.static_in.data_ptr():
            self.static_in.copy_(img)
        self.graph.replay()
        self.replays += 1
        for o in self.static_out:
            increment_version(o)

    def is_current(self, t):
        """True when ``t`` (an output of this trunk) still holds the data of the replay that
        returned it, i.e. no later replay has overwritten it (cloned outputs always are)."""
        return getattr(t, '_frh_replay', self.replays) == self.replays

    def __call__(self, img):
        if torch.is_grad_enabled():
            outs = _TrunkReplay.apply(self, img, *self.params)
        else:
            self.replay(img)
            outs = tuple(o.detach() for o in self.static_out)
        if self.clone_outputs:
            outs = tuple(o.clone() for o in outs)
        else:
            for o in outs:
                o._frh_replay = self.replays
        return split_trunk_outputs(outs)


def capture_trunk(detector, sample_img, num_warmup_iters=3, clone_outputs=False):
    """Capture ``detector``'s backbone + neck + RPN head convs for ``sample_img``'s shape and
    attach it (``detector.graphed_trunk``).  Call after any convolution-algorithm search
    (``torch.backends.cudnn.benchmark`` warmup): the capture freezes the chosen kernels."""
    neck = detector.neck if getattr(detector, 'with_neck', False) else None
    trunk = Trunk(detector.backbone, neck, detector.rpn_head)
    torch.cuda.synchronize(sample_img.device)
    detector.graphed_trunk = GraphedTrunk(trunk, sample_img, num_warmup_iters, clone_outputs)
    torch.cuda.synchronize(sample_img.device)
    return detector.graphed_trunk


def release_trunk(detector):
    detector.graphed_trunk = None

"""Fused loss kernels (csrc/losses.hip) against the torch fp32 restatement
of lib/losses.py (frcnn_amd.losses' eager functions, the same expressions as the
reference), forward sums and gradients.  Floating point: sums within rtol 2e-5 (reduction
order differs), gradients within rtol 1e-4 / atol 1e-6."""
import pytest
import torch

from frcnn_amd import losses, ops

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _labels(n, hi, pos_frac, gen):
    lab = torch.randint(1, hi + 1, (n,), generator=gen)
    lab[torch.rand(n, generator=gen) > pos_frac] = 0
    return lab


def _check(fused_fn, eager_fn, x0, scale=0.37):
    xa = x0.clone().to(DEV).requires_grad_(True)
    xb = x0.clone().to(DEV).requires_grad_(True)
    la, lb = fused_fn(xa), eager_fn(xb)
    torch.testing.assert_close(la, lb, rtol=2e-5, atol=1e-6)
    (la * scale).backward()
    (lb * scale).backward()
    torch.testing.assert_close(xa.grad, xb.grad, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize('layout', ['rows', 'channel_major'])
def test_focal_loss(layout):
    g = torch.Generator().manual_seed(1)
    n, c = 6000, 20
    lab = _labels(n, c, 0.05, g).to(DEV)
    x0 = torch.randn(n, c, generator=g) * 3
    if layout == 'rows':
        _check(lambda x: ops.cls_loss(x, lab, ops.CLS_FOCAL), lambda x: losses.sigmoid_focal_loss(x, lab), x0)
    else:  # AnchorHead passes tar_cls_out.t(): a [C, S] tensor viewed [S, C]
        xt = x0.t().contiguous()
        _check(lambda x: ops.cls_loss(x.t(), lab, ops.CLS_FOCAL), lambda x: losses.sigmoid_focal_loss(x.t(), lab), xt)


def test_focal_loss_module_dispatch():
    g = torch.Generator().manual_seed(2)
    x = (torch.randn(300, 20, generator=g) * 2).to(DEV)
    lab = _labels(300, 20, 0.3, g).to(DEV)
    torch.testing.assert_close(losses.FocalLoss()(x, lab), losses.sigmoid_focal_loss(x, lab), rtol=2e-5, atol=1e-6)


@pytest.mark.parametrize('c', [1, 20])
def test_sigmoid_bce(c):
    g = torch.Generator().manual_seed(3 + c)
    n = 4096
    lab = (torch.rand(n, generator=g) < 0.3).long() if c == 1 else _labels(n, c, 0.2, g)
    lab = lab.to(DEV)
    x0 = torch.randn(n, c, generator=g) * 4
    eager = losses.CrossEntropyLoss(use_sigmoid=True)
    cpu_ref = lambda x: eager(x.cpu(), lab.cpu()).to(DEV)  # the module's torch path runs for CPU tensors
    _check(lambda x: losses.CrossEntropyLoss(use_sigmoid=True)(x, lab), cpu_ref, x0)


def test_sigmoid_bce_float_targets():
    # FCOS centerness: CrossEntropyLoss(use_sigmoid=True) on [n, 1] logits vs float targets
    g = torch.Generator().manual_seed(5)
    n = 777
    t = torch.rand(n, generator=g).to(DEV)
    x0 = torch.randn(n, 1, generator=g)
    ref = lambda x: torch.nn.functional.binary_cross_entropy_with_logits(x, t.view(-1, 1), reduction='none').sum()
    _check(lambda x: losses.CrossEntropyLoss(use_sigmoid=True)(x, t), ref, x0)


def test_softmax_ce():
    g = torch.Generator().manual_seed(6)
    n, c = 1024, 21
    lab = _labels(n, c - 1, 0.25, g).to(DEV)
    x0 = torch.randn(n, c, generator=g) * 3
    ref = lambda x: torch.nn.functional.cross_entropy(x, lab, reduction='none').sum()
    _check(lambda x: losses.CrossEntropyLoss()(x, lab), ref, x0)


def test_smooth_l1_masked_columns():
    # AnchorHead: tar_reg_out / tar_param [4, S], positives by column
    g = torch.Generator().manual_seed(7)
    s = 512
    lab = _labels(s, 1, 0.3, g).to(DEV)
    y = (torch.randn(4, s, generator=g) * 0.2).to(DEV)
    x0 = torch.randn(4, s, generator=g) * 0.2
    m = (lab > 0).view(1, -1)
    beta = 1.0 / 9.0
    ref = lambda x: losses.smooth_l1_loss_v2(torch.where(m, x, x.new_zeros(())), torch.where(m, y, y.new_zeros(())),
                                             beta)
    _check(lambda x: losses.SmoothL1Loss(beta).masked(x, y, lab, rows_dim=1), ref, x0)


def test_smooth_l1_unmasked():
    g = torch.Generator().manual_seed(8)
    y = torch.randn(300, 4, generator=g).to(DEV)
    x0 = torch.randn(300, 4, generator=g)
    _check(lambda x: losses.SmoothL1Loss(0.5)(x, y), lambda x: losses.smooth_l1_loss_v2(x, y, 0.5), x0)


def test_smooth_l1_class_select():
    # BBoxHead: reg_out [n, 4*C] viewed [n, 4, C], labelled class, positive rows, target tar_param.t()
    g = torch.Generator().manual_seed(9)
    n, c = 1024, 21
    lab = _labels(n, c - 1, 0.25, g).to(DEV)
    tp = (torch.randn(4, n, generator=g) * 0.5).to(DEV)
    x0 = torch.randn(n, 4 * c, generator=g) * 0.5

    def ref(x):
        sel = x.view(-1, 4, c)[torch.arange(n, device=DEV), :, lab]
        m = (lab > 0).view(-1, 1)
        z = x.new_zeros(())
        return losses.smooth_l1_loss_v2(torch.where(m, sel, z), torch.where(m, tp.t(), z), 1.0)

    _check(lambda x: losses.SmoothL1Loss(1.0).class_selected(x, c, tp.t(), lab), ref, x0)


def test_empty_inputs():
    x = torch.zeros(0, 20, device=DEV, requires_grad=True)
    lab = torch.zeros(0, dtype=torch.long, device=DEV)
    loss = ops.cls_loss(x, lab, ops.CLS_FOCAL)
    assert float(loss) == 0.0
    loss.backward()
    assert x.grad.shape == (0, 20)
    y = torch.zeros(4, 0, device=DEV)
    assert float(losses.SmoothL1Loss(1.0).masked(torch.zeros(4, 0, device=DEV), y, lab, rows_dim=1)) == 0.0


def test_bad_label_gives_nan():
    # a softmax label outside [0, C) poisons the sum instead of reading out of bounds
    x = torch.randn(8, 5, device=DEV)
    lab = torch.tensor([0, 1, 2, 3, 4, 5, 0, 1], device=DEV)
    assert torch.isnan(ops.cls_loss(x, lab, ops.CLS_SOFTMAX_CE))


@pytest.mark.parametrize('case', ['rpn_sigmoid', 'rpn_focal', 'rcnn_softmax_class_select', 'rcnn_agnostic'])
def test_det_losses_one_launch_equal_separate(case):
    """losses.head_losses (frh_det_loss_fwd: both losses of a head and their scaling in one
    launch) must equal the separate modules divided by avg_factor BIT FOR BIT (same
    partitioned sums, same f32 scaling), and give the same gradients (the reference's
    Div-then-Mul backward)."""
    g = torch.Generator().manual_seed(11)
    beta = 1.0 / 9.0
    if case.startswith('rpn'):
        S = 512
        c = 1 if case == 'rpn_sigmoid' else 20
        lab = _labels(S, c, 0.25, g).to(DEV)
        cls0 = (torch.randn(c, S, generator=g) * 2).to(DEV)       # AnchorHead: tar_cls_out [C, S]
        reg0 = torch.randn(4, S, generator=g).to(DEV)             # tar_reg_out [4, S]
        tgt = torch.randn(4, S, generator=g).to(DEV)
        loss_cls = (losses.CrossEntropyLoss(use_sigmoid=True) if c == 1 else losses.FocalLoss())
        l1 = lambda r: ops._l1_args(r, tgt, lab, 1)  # noqa: E731
        sep_reg = lambda r: losses.SmoothL1Loss(beta).masked(r, tgt, lab, rows_dim=1)  # noqa: E731
        cls_in = lambda x: x.t()  # noqa: E731
    else:
        n, C = 1024, 21
        lab = _labels(n, C - 1, 0.25, g).to(DEV)
        cls0 = torch.randn(n, C, generator=g).to(DEV)
        loss_cls = losses.CrossEntropyLoss()
        tgt = torch.randn(4, n, generator=g).to(DEV)              # tar_param [4, n]
        if case == 'rcnn_agnostic':
            reg0 = torch.randn(n, 4, generator=g).to(DEV)
            l1 = lambda r: ops._l1_args(r, tgt.t(), lab, 0)  # noqa: E731
            sep_reg = lambda r: losses.SmoothL1Loss(1.0).masked(r, tgt.t(), lab, rows_dim=0)  # noqa: E731
        else:
            reg0 = torch.randn(n, 4 * C, generator=g).to(DEV)
            l1 = lambda r: ops._l1_class_select_args(r, C, tgt.t(), lab)  # noqa: E731
            sep_reg = lambda r: losses.SmoothL1Loss(1.0).class_selected(r, C, tgt.t(), lab)  # noqa: E731
        beta = 1.0
        cls_in = lambda x: x  # noqa: E731
    loss_bbox = losses.SmoothL1Loss(beta)
    avg = lab.numel()
    xa, xb = cls0.clone().requires_grad_(True), cls0.clone().requires_grad_(True)
    ra, rb = reg0.clone().requires_grad_(True), reg0.clone().requires_grad_(True)
    fa = losses.head_losses(loss_cls, loss_bbox, cls_in(xa), lab, lambda: l1(ra), avg)
    assert fa is not None
    ca, qa = fa
    cb = loss_cls(cls_in(xb), lab) / avg
    qb = sep_reg(rb) / avg
    assert torch.equal(ca, cb) and torch.equal(qa, qb), (ca.item(), cb.item(), qa.item(), qb.item())
    (ca * 0.7 + qa * 1.3).backward()
    (cb * 0.7 + qb * 1.3).backward()
    assert torch.equal(xa.grad, xb.grad)
    assert torch.equal(ra.grad, rb.grad)


@pytest.mark.parametrize('case', ['rpn_sigmoid', 'rcnn_softmax_class_select', 'empty'])
def test_det_losses_padded_rows_device_count(case):
    """Sync-free targets: the fixed-capacity buffers carry padding rows (label -1) past the
    sampled total and the divisor is that total as a device int32 count.  The losses equal the
    unpadded ones with the host count (rtol 2e-5: the padded launch may partition the sum
    differently), the real rows' gradients are bit-identical and the padding rows' are 0; a
    count of 0 (every row padding) gives zero losses and zero gradients."""
    g = torch.Generator().manual_seed(5)
    n = 0 if case == 'empty' else 300
    pad = 212
    if case.startswith('rcnn'):
        C = 21
        lab = torch.cat([_labels(n, C - 1, 0.25, g), torch.full((pad,), -1, dtype=torch.int64)]).to(DEV)
        cls0 = torch.randn(n + pad, C, generator=g).to(DEV)
        reg0 = torch.randn(n + pad, 4 * C, generator=g).to(DEV)
        tgt = torch.randn(4, n + pad, generator=g).to(DEV)
        loss_cls, beta = losses.CrossEntropyLoss(), 1.0
        l1 = lambda r, k: ops._l1_class_select_args(r[:k], C, tgt.t()[:k], lab[:k])  # noqa: E731
        cls_in = lambda x, k: x[:k]  # noqa: E731
    else:
        lab = torch.cat([_labels(n, 1, 0.25, g), torch.full((pad,), -1, dtype=torch.int64)]).to(DEV)
        cls0 = (torch.randn(1, n + pad, generator=g) * 2).to(DEV)
        reg0 = torch.randn(4, n + pad, generator=g).to(DEV)
        tgt = torch.randn(4, n + pad, generator=g).to(DEV)
        loss_cls, beta = losses.CrossEntropyLoss(use_sigmoid=True), 1.0 / 9.0
        l1 = lambda r, k: ops._l1_args(r[:, :k], tgt[:, :k], lab[:k], 1)  # noqa: E731
        cls_in = lambda x, k: x[:, :k].t()  # noqa: E731
    loss_bbox = losses.SmoothL1Loss(beta)
    T = n + pad
    cnt = torch.tensor([n], dtype=torch.int32, device=DEV)
    xa, xb = cls0.clone().requires_grad_(True), cls0.clone().requires_grad_(True)
    ra, rb = reg0.clone().requires_grad_(True), reg0.clone().requires_grad_(True)
    ca, qa = losses.head_losses(loss_cls, loss_bbox, cls_in(xa, T), lab, lambda: l1(ra, T), None, div_count=cnt)
    if n == 0:
        assert float(ca) == 0.0 and float(qa) == 0.0
        (ca + qa).backward()
        assert not xa.grad.any() and not ra.grad.any()
        return
    cb, qb = losses.head_losses(loss_cls, loss_bbox, cls_in(xb, n), lab[:n], lambda: l1(rb, n), n)
    torch.testing.assert_close(ca.view(()), cb.view(()), rtol=2e-5, atol=0)
    torch.testing.assert_close(qa.view(()), qb.view(()), rtol=2e-5, atol=0)
    (ca * 0.7 + qa * 1.3).sum().backward()
    (cb * 0.7 + qb * 1.3).backward()
    real = (slice(None, n),) if case.startswith('rcnn') else (slice(None), slice(None, n))
    padr = (slice(n, None),) if case.startswith('rcnn') else (slice(None), slice(n, None))
    assert torch.equal(xa.grad[real], xb.grad[real]) and torch.equal(ra.grad[real], rb.grad[real])
    assert not xa.grad[padr].any() and not ra.grad[padr].any()


def test_level_gather_skips_padding_columns():
    """frh_gather_level_outputs / frh_scatter_level_grads: a column with seg_of -1 (a padding
    column of the sync-free anchor targets) gathers zeros and scatters nothing, even where a
    real column names the same location (no lost read-modify-write)."""
    g = torch.Generator().manual_seed(2)
    lv = [torch.randn(2, 3, 4, 5, generator=g).to(DEV).requires_grad_(True),
          torch.randn(2, 3, 2, 3, generator=g).to(DEV).requires_grad_(True)]
    idx = torch.tensor([0, 7, 25, 0, 0, 3], dtype=torch.int64, device=DEV)
    seg = torch.tensor([0, 1, 0, -1, -1, 1], dtype=torch.int32, device=DEV)
    out = ops.gather_level_outputs(lv, idx, seg, 3)
    flat = [torch.cat([l[b].reshape(3, -1) for l in lv], 1) for b in range(2)]
    want = torch.stack([flat[int(s)][:, int(i)] if s >= 0 else torch.zeros(3, device=DEV)
                        for i, s in zip(idx.tolist(), seg.tolist())], 1)
    assert torch.equal(out, want)
    gout = torch.randn(3, 6, generator=g).to(DEV)
    out.backward(gout)
    ref = [torch.zeros_like(l) for l in lv]
    rflat = [torch.cat([r[b].reshape(3, -1) for r in ref], 1) for b in range(2)]
    for j, (i, s) in enumerate(zip(idx.tolist(), seg.tolist())):
        if s >= 0:
            rflat[s][:, i] += gout[:, j]
    got = [torch.cat([l.grad[b].reshape(3, -1) for l in lv], 1) for b in range(2)]
    assert torch.equal(got[0], rflat[0]) and torch.equal(got[1], rflat[1])

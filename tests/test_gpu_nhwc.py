"""Channels-last (NHWC) FPN levels on the HIP path:

* ops.fpn_merge_nhwc -- the FPN top-down step lat + interpolate(up, 'nearest')
  (reference lib/necks.py:72-84) written as an NHWC level: bit-identical to torch's
  NCHW expression (exact 2x and non-2x level sizes, the top level alone), also with the
  lateral conv's bias folded in; gradients equal to torch's autograd of the same expression;
* ops.conv_bias_relu -- the RPN head's relu(conv(x)) as a bias-free NHWC conv + one HIP bias
  + ReLU pass: bit-identical to conv-with-bias + relu, same gradients;
* the FPN module's NHWC path against its NCHW torch path on the same weights (the merge is
  exact; the 3x3 convs run MIOpen NHWC vs NCHW solvers: f32 summation-order tolerance);
* RPN proposals (frh_rpn_proposals_strided) and the level gather / scatter
  (frh_*_level_*_strided) on channels-last head outputs: bit-identical to the same values
  in NCHW;
* the cfg2 detector's forward_train on the NHWC trunk against the same detector with the
  trunk forced to NCHW, on the same trunk values (the detection path only sees the layout).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import inputs

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize('shape,up_shape', [((2, 256, 152, 256), (76, 128)), ((2, 64, 25, 38), (13, 19)),
                                            ((1, 96, 19, 30), None), ((2, 8, 7, 6), (4, 3))])
def test_fpn_merge_nhwc_bit_exact(dev, shape, up_shape):
    from frcnn_amd import ops
    g = torch.Generator().manual_seed(3)
    lat = torch.randn(*shape, generator=g).to(dev)
    up = torch.randn(shape[0], shape[1], *up_shape, generator=g).to(dev) if up_shape else None
    out = ops.fpn_merge_nhwc(lat, _cl(up) if up is not None else None)
    assert out.is_contiguous(memory_format=torch.channels_last)
    want = lat if up is None else lat + F.interpolate(up, size=shape[2:], mode='nearest')
    assert torch.equal(out, want)
    # strided lateral (a view) takes the scalar path
    out2 = ops.fpn_merge_nhwc(lat[:, :, :, :shape[3] - 1], _cl(up) if up is not None else None)
    want2 = lat[:, :, :, :-1] if up is None else lat[:, :, :, :-1] + F.interpolate(up, size=(shape[2], shape[3] - 1),
                                                                                    mode='nearest')
    assert torch.equal(out2, want2)


@pytest.mark.parametrize('shape,up_shape', [((2, 256, 76, 128), (38, 64)), ((1, 96, 19, 30), None),
                                            ((2, 6, 7, 6), (4, 3))])
def test_fpn_merge_nhwc_bias_fold_bit_exact(dev, shape, up_shape):
    """The lateral conv's bias folded into the merge: (conv(x) + bias) + upsample, bit for bit
    (6 channels: the scalar path)."""
    from frcnn_amd import ops
    g = torch.Generator().manual_seed(6)
    lat = torch.randn(*shape, generator=g).to(dev)
    bias = torch.randn(shape[1], generator=g).to(dev)
    up = torch.randn(shape[0], shape[1], *up_shape, generator=g).to(dev) if up_shape else None
    out = ops.fpn_merge_nhwc(lat, _cl(up) if up is not None else None, bias)
    with_bias = lat + bias.view(1, -1, 1, 1)
    want = with_bias if up is None else with_bias + F.interpolate(up, size=shape[2:], mode='nearest')
    assert torch.equal(out, want)


def test_fpn_merge_nhwc_bias_gradient(dev):
    from frcnn_amd import ops
    g = torch.Generator().manual_seed(7)
    lat = torch.randn(2, 32, 38, 64, generator=g).to(dev).requires_grad_(True)
    bias = torch.randn(32, generator=g).to(dev).requires_grad_(True)
    gout = torch.randn(2, 32, 38, 64, generator=g).to(dev)
    ops.fpn_merge_nhwc(lat, None, bias).backward(gout)
    torch.testing.assert_close(bias.grad, gout.sum((0, 2, 3)), rtol=1e-6, atol=1e-5)
    assert torch.equal(lat.grad, gout)


@pytest.mark.parametrize('shape', [(2, 256, 152, 256), (2, 256, 10, 16), (1, 64, 7, 9)])
def test_conv_bias_relu_bit_exact(dev, shape):
    """RPN head's relu(conv(x)) on a channels-last level: the HIP bias + ReLU pass on a bias-free
    conv output equals torch's add + relu bit for bit; the whole op matches the module's conv
    (bias included) + relu; the same gradients as torch's autograd of conv + relu."""
    from frcnn_amd import ops
    from frcnn_amd.utils import conv_layout
    torch.manual_seed(8)
    conv = torch.nn.Conv2d(shape[1], shape[1], 3, padding=1).to(dev)
    torch.nn.init.normal_(conv.bias, std=0.5)
    conv_layout(conv)
    x = _cl(torch.randn(*shape, device=dev))
    with torch.no_grad():
        out = ops.conv_bias_relu(conv, x)
        # the epilogue on one conv output, bit for bit (two conv calls need not agree: MIOpen's
        # split-K solvers for small maps accumulate with atomics)
        y = torch.nn.functional.conv2d(x, conv.weight, None, 1, 1)
        ref = torch.relu(y + conv.bias.view(1, -1, 1, 1))
        fused = ops._BiasAct.apply(y.clone(), conv.bias, True)
    assert out.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(fused, ref)
    torch.testing.assert_close(out, torch.relu(conv(x)), rtol=1e-5, atol=1e-5)
    if shape[2] > 100:
        return
    xg = x.clone().requires_grad_(True)
    gout = torch.randn(*shape, device=dev)
    ops.conv_bias_relu(conv, xg).backward(gout)
    gx, gw, gb = xg.grad, conv.weight.grad.clone(), conv.bias.grad.clone()
    conv.zero_grad()
    x2 = x.clone().requires_grad_(True)
    torch.relu(conv(x2)).backward(gout)
    torch.testing.assert_close(gx, x2.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gw, conv.weight.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(gb, conv.bias.grad, rtol=1e-5, atol=1e-4)


def test_fpn_merge_nhwc_gradients(dev):
    from frcnn_amd import ops
    g = torch.Generator().manual_seed(4)
    lat = torch.randn(2, 32, 38, 64, generator=g).to(dev).requires_grad_(True)
    up = torch.randn(2, 32, 19, 32, generator=g).to(dev)
    upc = _cl(up).requires_grad_(True)
    gout = torch.randn(2, 32, 38, 64, generator=g).to(dev)
    ops.fpn_merge_nhwc(lat, upc).backward(gout)
    lat2 = lat.detach().clone().requires_grad_(True)
    up2 = up.clone().requires_grad_(True)
    (lat2 + F.interpolate(up2, size=(38, 64), mode='nearest')).backward(gout)
    assert torch.equal(lat.grad, lat2.grad)
    torch.testing.assert_close(upc.grad, up2.grad, rtol=1e-6, atol=1e-6)


def test_fpn_nhwc_path_matches_nchw(dev):
    """cfg2 FPN (necks.FPN on the 608x1024 backbone shapes): NHWC path vs torch's NCHW ops."""
    from frcnn_amd.necks import FPN
    torch.manual_seed(5)
    fpn = FPN([256, 512, 1024, 2048], 256, 5)
    fpn.init_weights()
    ins = [torch.randn(2, c, h, w) for c, (h, w) in zip([256, 512, 1024, 2048], [(152, 256), (76, 128), (38, 64),
                                                                               (19, 32)])]
    with torch.no_grad():
        ref = fpn(ins)  # CPU: NCHW reference ops
        fpn = fpn.to(dev)
        assert all(m.weight.is_contiguous(memory_format=torch.channels_last) for m in fpn.fpn_convs)
        outs = fpn([x.to(dev) for x in ins])
    assert outs[0].is_contiguous(memory_format=torch.channels_last)
    for o, r in zip(outs, ref):
        torch.testing.assert_close(o.cpu(), r, rtol=1e-4, atol=1e-4)
    cpu = fpn.cpu()  # back on the CPU: default-layout weights again
    assert all(m.weight.is_contiguous() for m in cpu.fpn_convs)


def _head_outputs(dev, seed, A, cls_ch, nhwc):
    cls, reg = inputs.head_outputs(seed, inputs.FPN_GRIDS, A, cls_ch, batch=2, reg_scale=0.5)
    cls = [torch.from_numpy(c).to(dev) for c in cls]
    reg = [torch.from_numpy(r).to(dev) for r in reg]
    if nhwc:
        cls, reg = [_cl(c) for c in cls], [_cl(r) for r in reg]
    return cls, reg


@pytest.mark.parametrize('cls_ch', [1, 2])
def test_rpn_proposals_channels_last_equal(dev, cls_ch):
    from frcnn_amd import ops
    from frcnn_amd.heads.rpn_head import RPNHead
    head = RPNHead(256, 256, loss_cls=dict(type='CrossEntropyLoss', use_sigmoid=cls_ch == 1),
                   loss_bbox=dict(type='SmoothL1Loss', beta=1.0 / 9.0)).to(dev)
    anchors = head._flat_anchors(inputs.FPN_GRIDS, dev)
    res = []
    for nhwc in (False, True):
        cls, reg = _head_outputs(dev, 600, 3, cls_ch, nhwc)
        res.append(ops.rpn_proposals(cls, reg, anchors, 3, cls_ch, [0.0] * 4, [1.0] * 4, [(600.0, 1000.0)] * 2,
                                     [0.0, 25.6], 2000, 2000, 2000, 0.7))
    torch.cuda.synchronize()
    assert torch.equal(res[0][2], res[1][2])
    for i, n in enumerate(res[0][2].tolist()):
        assert torch.equal(res[0][0][i, :, :n], res[1][0][i, :, :n])
        assert torch.equal(res[0][1][i, :n], res[1][1][i, :n])


def test_level_gather_scatter_channels_last_equal(dev):
    from frcnn_amd import ops
    rng = np.random.default_rng(7)
    N = sum(3 * h * w for h, w in inputs.FPN_GRIDS)
    chosen = torch.from_numpy(rng.choice(N, 700, replace=False)).to(dev)  # distinct: the scatter is a plain RMW
    seg = torch.from_numpy(rng.integers(-1, 2, 700).astype(np.int32)).to(dev)
    gin = torch.from_numpy(rng.standard_normal((4, 700)).astype(np.float32)).to(dev)
    res = []
    for nhwc in (False, True):
        _, reg = _head_outputs(dev, 601, 3, 1, nhwc)
        reg = [r.requires_grad_(True) for r in reg]
        out = ops.gather_level_outputs(reg, chosen, seg, 4)
        out.backward(gin)
        res.append((out.detach(), [r.grad for r in reg]))
    assert torch.equal(res[0][0], res[1][0])
    for a, b in zip(res[0][1], res[1][1]):
        assert b.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(a, b)


def test_forward_train_nhwc_trunk_equals_nchw(dev):
    """cfg2 forward_train with the device sampler on the same trunk VALUES in both layouts:
    the NHWC levels / RPN outputs of the product trunk vs NCHW copies of them -- same losses
    bit for bit (every detection kernel reads the layout through its strides)."""
    import bench
    from frcnn_amd import set_sampler_mode
    model, _ = bench.make_model(dev, seed=0)
    imgs, boxes, labels, metas = bench.make_batch(dev, 2, seed=1)
    with torch.no_grad():
        feats = model.extract_feat(imgs)
        rc, rr = model.rpn_head(feats)
    assert feats[0].is_contiguous(memory_format=torch.channels_last) and rc[0].stride(1) == 1
    out = []
    for nhwc in (True, False):
        f = [x if nhwc else x.contiguous() for x in feats]
        c = [x if nhwc else x.contiguous() for x in rc]
        r = [x if nhwc else x.contiguous() for x in rr]

        class Trunk(object):
            def matches(self, img_data):
                return True

            def __call__(self, img_data, f=f, c=c, r=r):
                return f, c, r
        model.graphed_trunk = Trunk()
        set_sampler_mode('device', seed=9)
        with torch.no_grad():
            out.append({k: float(v) for k, v in model.forward_train(imgs, boxes, labels, metas).items()})
    model.graphed_trunk = None
    assert out[0] == out[1], out

"""Whole-detector parity against the REFERENCE's own outputs, for every BASELINE config with a
trunk this repo builds (cfg2 Faster R-CNN FPN, cfg3 RetinaNet, cfg4 Cascade R-CNN, cfg5
ATSS): forward_train's loss dict and forward_test's detections of the reference model on
deterministic seeded weights (tests/golden/whole_<cfg>.{json,npz}, made by
gen_golden.gen_whole_detectors from /root/reference/lib through lib/builder.py; the
reference's torchvision nms / RoIAlign are the oracle's restatements there).

The product model gets the same weights (identical state_dict keys).  The dense convs and
FC layers -- backbone, FPN, RPN / Retina / FCOS head convs, the RCNN FCs: PyTorch
modules, not this library -- run on the CPU exactly as in the fixture, their outputs moved
to the GPU; every detection primitive between them runs on the HIP path: anchors,
assignment, sampling (numpy-RNG parity mode), targets, proposals + NMS, RoIAlign, ATSS,
refine, multiclass NMS and the fused losses.  Bars: losses rel 2e-5 (the fused losses sum
in double, torch CPU in float), detections in the reference's order with labels exact,
scores rel 1e-6 and boxes within a few f32 ulps (rel 2e-6: the decode's expf / the
ATSS ltrb scale round differently from torch's CPU vector math in the last bit)."""
import copy
import json
import os

import numpy as np
import pytest
import torch

import inputs

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {c[0]: c for c in inputs.WHOLE_DETECTORS}


def _model(fname, over):
    from frcnn_amd.config import Config
    from frcnn_amd.builder import build_module
    cfg = Config.fromfile(os.path.join(REPO, 'pytorch-faster-rcnn_amd', 'configs', fname))
    for k, v in over.items():
        cfg.test_cfg[k].update(v)
    model = build_module(cfg.model, train_cfg=cfg.train_cfg, test_cfg=cfg.test_cfg)
    sd = inputs.seeded_state({k: tuple(v.shape) for k, v in model.state_dict().items()})
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    model.train()
    return model


def _to(x, dev):
    if torch.is_tensor(x):
        return x.to(dev)
    if isinstance(x, (list, tuple)):
        return type(x)(_to(v, dev) for v in x)
    return x


def _on_cpu(module, dev):
    """Run `module` (a PyTorch conv / FC stack) on a CPU copy of itself, outputs back on dev."""
    cpu = copy.deepcopy(module).cpu()

    def forward(*args):
        with torch.no_grad():
            return _to(cpu(*[_to(a, 'cpu') for a in args]), dev)
    module.forward = forward


def _prepare(tag, dev):
    _, fname, over, shape = CASES[tag]
    model = _model(fname, over)
    img, boxes, labels, metas = inputs.ftrain_case(shape)
    x = torch.from_numpy(img)
    with torch.no_grad():
        feats = model.extract_feat(x)
    model = model.to(dev)
    dfeats = [f.to(dev) for f in feats]
    model.extract_feat = lambda img_data: dfeats
    if hasattr(model, 'rpn_head'):
        _on_cpu(model.rpn_head, dev)
        for h in model.rcnn_head:  # the FC stack only: RoI features come from the HIP RoIAlign
            for name in ('shared_fcs', 'classifier', 'regressor'):
                if getattr(h, name, None) is not None:
                    _on_cpu(getattr(h, name), dev)
    else:
        _on_cpu(model.bbox_head, dev)
    from frcnn_amd import set_sampler_mode
    set_sampler_mode('numpy')
    return model, x.to(dev), [torch.from_numpy(b).to(dev) for b in boxes], \
        [torch.from_numpy(l).to(dev) for l in labels], metas


@pytest.mark.parametrize('tag', sorted(CASES))
def test_whole_forward_train_losses_vs_reference(dev, tag):
    ref = json.load(open(inputs.golden_path('whole_{}.json'.format(tag))))
    model, x, boxes, labels, metas = _prepare(tag, dev)
    if hasattr(model, 'graphed_trunk'):  # CascadeRCNN's trunk hook: feats + RPN outputs of the CPU trunk
        feats = model.extract_feat(x)
        rpn = model.rpn_head(feats)

        class CpuTrunk(object):
            def matches(self, img_data):
                return True

            def __call__(self, img_data):
                return feats, rpn[0], rpn[1]
        model.graphed_trunk = CpuTrunk()
    np.random.seed(inputs.FTRAIN_NP_SEED)
    with torch.no_grad():
        losses = model.forward_train(x, boxes, labels, metas)
    assert set(losses) == set(ref['losses'])
    for k, v in ref['losses'].items():
        assert float(losses[k]) == pytest.approx(v, rel=2e-5), (k, float(losses[k]), v)


@pytest.mark.parametrize('tag', sorted(CASES))
def test_whole_forward_test_detections_vs_reference(dev, tag):
    z = np.load(inputs.golden_path('whole_{}.npz'.format(tag)))
    model, x, _, _, metas = _prepare(tag, dev)
    model.eval()
    with torch.no_grad():
        dets = model.forward_test(x, metas)
    boxes, scores, labels = dets[:3]
    assert len(boxes) == int(z['n'])
    for i in range(int(z['n'])):
        rb, rs, rl = z['boxes_{}'.format(i)], z['scores_{}'.format(i)], z['labels_{}'.format(i)]
        gb = boxes[i].t().cpu().numpy()
        gs, gl = scores[i].cpu().numpy(), labels[i].cpu().numpy()
        assert len(rs) > 0 and gs.shape == rs.shape, (gs.shape, rs.shape)
        np.testing.assert_array_equal(gl, rl)
        np.testing.assert_allclose(gs, rs, rtol=1e-6, atol=0)
        np.testing.assert_allclose(gb, rb, rtol=2e-6, atol=1e-4)  # a few f32 ulps (exp / ltrb decode)


def test_device_sampler_targets_and_losses_vs_oracle(dev):
    """The timed configuration's sampler (device RNG, sync-free targets) pinned to the reference's
    consumers: cfg2 forward_train with the device sampler, its selections captured; the CPU
    oracle's anchor_target / bbox_target (lib/anchor.py:11-76, lib/bbox.py:6-82; the oracle is
    pinned to the reference by test_oracle_golden) run on the same assignment with THAT
    selection injected in place of np.random, and the oracle pipeline
    (oracle/pipeline.forward_train_cpu: the reference's per-image loop) computes the loss dict
    from it.  Bars: the assignment labels and every target column (chosen anchors / rows,
    labels, anchors / proposals, gt boxes) bit-exact against the HIP path's non-padding columns,
    the encoded params within 1 ulp (logf); losses rel 2e-5 (as the whole-detector tests)."""
    import pipeline
    from frcnn_amd import ops, set_sampler_mode
    from frcnn_amd.config import Config
    _, fname, over, shape = CASES['cfg2']
    model, x, boxes, labels, metas = _prepare('cfg2', dev)
    cap = {'sample': [], 'anchor_target': [], 'bbox_target': []}
    orig = (ops.sample_labels, ops.anchor_target_batched, ops.bbox_target_batched)

    def sample_labels(lab, num, mb, mx, pn, **kw):
        out = orig[0](lab, num, mb, mx, pn, **kw)
        cap['sample'].append((lab.clone(), num.clone(), out))
        return out

    def anchor_target_batched(*a, **kw):
        r = orig[1](*a, **kw)
        cap['anchor_target'].append(r)
        return r

    def bbox_target_batched(rows, num_rows, num_gts, max_rows, props, pstride, *a, **kw):
        r = orig[2](rows, num_rows, num_gts, max_rows, props, pstride, *a, **kw)
        cap['bbox_target'].append((props.clone(), num_rows.clone(), num_gts.clone(), r))
        return r
    ops.sample_labels, ops.anchor_target_batched, ops.bbox_target_batched = \
        sample_labels, anchor_target_batched, bbox_target_batched
    try:
        set_sampler_mode('device', seed=77)
        with torch.no_grad():
            losses = model.forward_train(x, boxes, labels, metas)
        torch.cuda.synchronize()
    finally:
        ops.sample_labels, ops.anchor_target_batched, ops.bbox_target_batched = orig
        set_sampler_mode('numpy')
    assert len(cap['sample']) == 2 and cap['anchor_target'] and cap['bbox_target']
    assert all(isinstance(c[2], ops.SampleLists) for c in cap['sample']), 'not the device sampler lists path'

    def selection(call, i):
        sl = cap['sample'][call][2]
        cnt = sl.sel_counts[i].cpu().numpy()
        sel = sl.sel[i].cpu().numpy()
        return np.concatenate([sel[0, :cnt[0]], sel[1, :cnt[1]]]).astype(np.int64)

    def hook(stage, i, lab):
        call = 0 if stage == 'rpn' else 1
        dev_lab = cap['sample'][call][0][i].cpu().numpy()
        if stage == 'rpn':  # oracle labels over the inside anchors; device labels over all (outside: -1)
            mask = dev_lab >= -1  # every anchor
            inside = np.nonzero(hook.mask)[0]
            np.testing.assert_array_equal(dev_lab[inside], lab)
            assert (dev_lab[~hook.mask] == -1).all() and mask.all()
            pos = np.cumsum(hook.mask) - 1
            chosen = pos[selection(call, i)]
            assert hook.mask[selection(call, i)].all()
        else:  # the prepended [gts; proposals] rows, same order on both sides
            np.testing.assert_array_equal(dev_lab[:lab.shape[0]], lab)
            chosen = selection(call, i)
        out = np.full_like(lab, -1)
        out[chosen] = lab[chosen]
        hook.sampled[stage] = out
        return out
    hook.sampled = {}
    cfg = Config.fromfile(os.path.join(REPO, 'pytorch-faster-rcnn_amd', 'configs', fname))
    for k, v in over.items():
        cfg.test_cfg[k].update(v)
    cpu_model = _model(fname, over)
    head = cpu_model.rpn_head
    with torch.no_grad():
        cls_outs, _ = head(cpu_model.extract_feat(x.cpu()))
    grids = [tuple(c.shape[-2:]) for c in cls_outs]
    _, flat = pipeline._anchors(head, grids)
    hook.mask = pipeline._in_mask(head, flat, grids, metas[0]['img_shape'][:2], cfg.train_cfg.rpn.allowed_border)
    with torch.no_grad():
        ref = pipeline.forward_train_cpu(cpu_model, cfg, x.cpu(), [b.cpu() for b in boxes],
                                         [l.cpu() for l in labels], metas, sampler_hook=hook)
    assert set(ref) == set(losses)
    for k in ref:
        assert float(losses[k]) == pytest.approx(float(ref[k]), rel=2e-5), (k, float(losses[k]), float(ref[k]))
    # the RPN targets, column by column (image 0 = the first device segment)
    at = cap['anchor_target'][0]
    a = cfg.train_cfg.rpn.assigner
    gb = boxes[0].cpu().numpy()
    o = oracle_anchor_target(flat, hook.mask, gb, a, lambda lab: hook.sampled['rpn'])
    n = o[2].shape[0]
    assert int(at['counts_dev'][0]) == n
    np.testing.assert_array_equal(at['chosen_idx'][:n].cpu().numpy(), o[6])
    np.testing.assert_array_equal(at['tar_labels'][:n].cpu().numpy(), o[2])
    for key, j in (('tar_anchors', 3), ('tar_bbox', 4)):
        np.testing.assert_array_equal(at[key][:, :n].cpu().numpy(), o[j], err_msg=key)
    # the encoded params: log(w / w_a) by the device logf vs the C library's, <= 1 ulp apart
    np.testing.assert_allclose(at['tar_param'][:, :n].cpu().numpy(), o[5], rtol=4e-7, atol=4e-7)
    # the RCNN targets
    props, num_rows, num_gts, bt = cap['bbox_target'][0]
    sc = cfg.train_cfg.rcnn[0]
    G = int(num_gts[0])
    npr = int(num_rows[0]) - G
    rh = cpu_model.rcnn_head[0]
    ob = oracle_bbox_target(props[0, :, :npr].cpu().numpy(), gb, labels[0].cpu().numpy(), sc.assigner,
                            lambda lab: hook.sampled['rcnn0'], rh)
    m = ob[0].shape[1]
    assert int(bt['counts_dev'][0]) == m
    for key, j in (('tar_props', 0), ('tar_bbox', 1), ('tar_label', 2), ('tar_is_gt', 4)):
        got = bt[key][..., :m].cpu().numpy()
        np.testing.assert_array_equal(got, ob[j], err_msg=key)
    np.testing.assert_allclose(bt['tar_param'][:, :m].cpu().numpy(), ob[3], rtol=4e-7, atol=4e-7)


def oracle_anchor_target(flat, mask, gb, a, sampler):
    import oracle
    return oracle.anchor_target(np.zeros((1, flat.shape[1]), np.float32), np.zeros((4, flat.shape[1]), np.float32), 1,
                                np.ascontiguousarray(flat[:, mask]), mask, gb, np.ones(gb.shape[1], np.int64),
                                (a.pos_iou, a.neg_iou, a.min_pos_iou), sampler, [0.0] * 4, [1.0] * 4)


def oracle_bbox_target(props, gb, gl, assigner, sampler, rh):
    import oracle
    return oracle.bbox_target(props, gb, gl, (assigner.pos_iou, assigner.neg_iou, assigner.min_pos_iou), sampler,
                              rh.target_means, rh.target_stds)

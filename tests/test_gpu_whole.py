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

"""The tools-only RoIAlign variants (tools/lib/libfrcnn_tools.so, tools/csrc/): the
kernels measured on the way to the product's must agree with the oracle
and, for the forward, bit for bit with each other and with the product kernel -- so the
benchmark numbers in DESIGN compare equal work.  The product library does not contain
them (test_abi checks its exports)."""
import os
import sys

import numpy as np
import pytest
import torch

import inputs
import oracle

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'tools'))

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _rois(seed, n, batch):
    b = inputs.random_boxes(seed, n, min_wh=1.0, max_wh=500.0)
    b[:, :8] = np.array([[-20, -20, 10, 10], [990, 590, 1200, 700], [0, 0, 0, 0], [5, 5, 5.5, 5.2],
                         [998.9, 598.9, 999, 599], [-300, -300, -200, -100], [0, 0, 999, 599],
                         [100.25, 200.75, 101.0, 260.5]], np.float32).T
    bi = np.random.default_rng(seed + 1).integers(0, batch, n).astype(np.float32)
    return np.concatenate([bi[None], b], 0).T.copy()


@pytest.mark.parametrize('layout', ['nchw', 'nhwc'])
def test_forward_variants_identical(dev, layout):
    import toolslib
    from frcnn_amd import ops, _lib
    lib = toolslib.load()
    grids = [(152, 256), (76, 128), (38, 64), (19, 32)]
    feats = inputs.feature_maps(42, grids, 96, 2)
    rois = _rois(43, 600, 2)
    levels = oracle.roi_level_map(rois, 56.0, 4)
    scales = [1 / 4, 1 / 8, 1 / 16, 1 / 32]
    ref = oracle.roi_align(feats, rois, levels, scales, (7, 7), 2)
    ft = [T(f, dev) for f in feats]
    if layout == 'nhwc':  # no 16-B staging: unit-stride rows are required
        ft = [f.contiguous(memory_format=torch.channels_last) for f in ft]
    r, lv = T(rois, dev), T(levels, dev)
    K, C = r.shape[0], ft[0].shape[1]
    hw, st = ops._feat_desc(ft)
    wsb = int(lib.frh_roi_align_workspace(K))
    ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    outs = {}
    for v in ((0, 10, 20, 21, 22, 23, 24, 25, 27, 28, 29, 30, 38, 39, 40, 41, 46, 47, 49, 50, 52, 53, 55) if layout == 'nchw' else (0, 10, 20, 21, 22, 25, 28, 29, 38, 46, 50, 55)):
        out = torch.full((K, C, 7, 7), float('nan'), device=dev)
        toolslib.call('frh_roi_align_fwd_variant', v, len(ft), _lib.ptr_array(ft), hw, st, _lib.f32_array(scales), 2,
                      C, _lib.ptr(r), _lib.ptr(lv), K, 7, 7, 2, 0, _lib.ptr(out), _lib.ptr(ws), wsb,
                      _lib.stream_of(out))
        outs[v] = out.cpu().numpy()
    np.testing.assert_allclose(outs[0], ref, rtol=1e-5, atol=1e-5)
    prod = ops.roi_align_multilevel(ft, r, lv, scales, (7, 7), 2).cpu().numpy()
    assert np.array_equal(prod, outs[0])
    for v in outs:
        assert np.array_equal(outs[v], outs[0]), 'variant %d differs' % v


@pytest.mark.parametrize('kind', ['tiled', 'cl'])
def test_backward_variants_vs_oracle(dev, kind):
    import toolslib
    from frcnn_amd import ops, _lib
    grids, scales, C, K = [(152, 256), (76, 128)], [1 / 4, 1 / 8], 80, 300
    rois = _rois(61, K, 2)
    levels = oracle.roi_level_map(rois, 56.0, 2)
    g = np.random.default_rng(62).standard_normal((K, C, 7, 7)).astype(np.float32)
    fmt = torch.channels_last if kind == 'cl' else torch.contiguous_format
    grads = [torch.zeros(2, C, h, w, device=dev).contiguous(memory_format=fmt) for h, w in grids]
    hw, st = ops._feat_desc(grads)
    r, lv, gt = T(rois, dev), T(levels, dev), T(g, dev)
    if kind == 'tiled':
        wsb = int(toolslib.load().frh_roi_align_bwd_workspace(2, hw, 2, K))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        toolslib.call('frh_roi_align_bwd_tiled', 2, _lib.ptr_array(grads), hw, st, _lib.f32_array(scales), 2, C,
                      _lib.ptr(r), _lib.ptr(lv), K, 7, 7, 2, 0, _lib.ptr(gt), _lib.ptr(ws), wsb, _lib.stream_of(gt))
    else:
        toolslib.call('frh_roi_align_bwd_cl', 2, _lib.ptr_array(grads), hw, st, _lib.f32_array(scales), 2, C,
                      _lib.ptr(r), _lib.ptr(lv), K, 7, 7, 2, 0, _lib.ptr(gt), _lib.stream_of(gt))
    ref = oracle.roi_align_bwd([(2, C, h, w) for h, w in grids], rois, levels, scales, g, 2)
    for a, b in zip(grads, ref):
        np.testing.assert_allclose(a.cpu().numpy(), b, rtol=1e-4, atol=2e-5)

"""Hand-derived expectations for the rows whose third-party reference (torchvision
RoIAlign / RoIPool / nms) is absent here, so that the oracle is not its own only witness.

Each case's expected output comes from a closed form or a by-hand computation written in
the test, not from running an implementation:

* RoIAlign (legacy aligned=False, sampling 2) on affine feature maps f = a + b*y + c*x:
  bilinear interpolation reproduces an affine function exactly, so a sample's value is
  f at its clamped position -- y <- max(y, 0), and y <- H-1 once floor(y) >= H-1 -- and 0
  when y < -1 or y > H (likewise x); a bin is the sum of its 4 samples / 4 (invalid
  samples still count in the 4).  The RoIs hit every branch: y < -1, -1 <= y <= 0,
  floor(y) >= H-1 with y <= H, y > H, a sub-pixel RoI (width clamped to 1) and a RoI
  fully outside.
* RoIPool on the integer ramp f = 100*c + 10*y + x: a bin's max is its bottom-right
  cell; bins worked by hand (round-half-away-from-zero of the RoI corners, floor/ceil
  bin edges, clipping, empty bins = 0).
* NMS: five boxes whose IoUs are worked by hand (no +1 in areas), and the boundary case
  IoU == float(thr) that tells torchvision's CPU rule (float IoU > double thr: suppress)
  from its CUDA rule (float IoU > float thr: keep) apart at thr = 0.3.

The CPU tests check the oracle; the gpu-marked tests check the HIP kernels through the
product ops."""
import numpy as np
import pytest
import torch

import oracle

# ----------------------------------------------------------------- RoIAlign on affine maps
H, W, C = 20, 30, 3
COEF = np.array([[1.0, 0.5, -0.25], [-2.0, 0.0, 1.0], [3.5, -1.0, 0.75]])  # (a, b, c) per channel
AFFINE_ROIS = np.array([
    [0, 3.0, 2.0, 17.0, 11.0],      # interior
    [0, -9.0, -9.0, 8.0, 6.0],      # samples at y, x < -1 (invalid) and in [-1, 0] (clamped to 0)
    [1, 10.0, 14.0, 33.0, 23.5],    # samples with floor >= H-1 / W-1 (clamped) and > H / > W (invalid)
    [1, 12.3, 7.6, 12.5, 7.7],      # sub-pixel: width and height clamped to 1
    [0, -40.0, -30.0, -20.0, -5.0],  # fully outside: all zero
    [1, 28.2, 18.4, 40.0, 30.0],    # corner: mostly invalid, a few clamped samples
], np.float32)


def affine_maps():
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    f = np.stack([a + b * y + c * x for a, b, c in COEF])  # [C, H, W]
    return np.stack([f, f + 10.0]).astype(np.float32)  # image 1 = image 0 + 10


def affine_expected(rois, scale=1.0):
    out = np.zeros((len(rois), C, 7, 7))
    for k, (b, x1, y1, x2, y2) in enumerate(rois.astype(np.float64)):
        sw, sh = x1 * scale, y1 * scale
        rw, rh = max(x2 * scale - sw, 1.0), max(y2 * scale - sh, 1.0)
        bh, bw = rh / 7, rw / 7

        def clamp(v, size):
            if v < -1.0 or v > size:
                return None
            v = max(v, 0.0)
            return float(size - 1) if int(v) >= size - 1 else v

        for py in range(7):
            for px in range(7):
                acc = np.zeros(C)
                for iy in range(2):
                    yy = clamp(sh + py * bh + (iy + 0.5) * bh / 2, H)
                    for ix in range(2):
                        xx = clamp(sw + px * bw + (ix + 0.5) * bw / 2, W)
                        if yy is None or xx is None:
                            continue
                        acc += COEF[:, 0] + COEF[:, 1] * yy + COEF[:, 2] * xx + 10.0 * b
                out[k, :, py, px] = acc / 4
    return out


def test_affine_expected_covers_every_branch():
    e = affine_expected(AFFINE_ROIS)
    assert np.all(e[4] == 0)                      # fully outside
    assert np.any(e[1] != 0) and np.any(e[2] != 0)
    # the interior RoI's centre bin is f at the bin centre (all four samples valid, unclamped)
    cy, cx = 2.0 + 3.5 * (9.0 / 7), 3.0 + 3.5 * (14.0 / 7)
    np.testing.assert_allclose(e[0, :, 3, 3], COEF[:, 0] + COEF[:, 1] * cy + COEF[:, 2] * cx, rtol=1e-12)


def test_roi_align_affine_oracle():
    f = affine_maps()
    out = oracle.roi_align([f], AFFINE_ROIS, None, [1.0], (7, 7), 2)
    np.testing.assert_allclose(out, affine_expected(AFFINE_ROIS), rtol=1e-5, atol=2e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('layout', ['nchw', 'nhwc'])
def test_roi_align_affine_hip(dev, layout):
    from frcnn_amd import ops
    f = torch.from_numpy(affine_maps()).to(dev)
    if layout == 'nhwc':
        f = f.contiguous(memory_format=torch.channels_last)
    rois = torch.from_numpy(AFFINE_ROIS).to(dev)
    lv = torch.zeros(len(AFFINE_ROIS), dtype=torch.int64, device=dev)
    out = ops.roi_align_multilevel([f], rois, lv, [1.0], (7, 7), 2).cpu().numpy()
    np.testing.assert_allclose(out, affine_expected(AFFINE_ROIS), rtol=1e-5, atol=2e-5)


# ----------------------------------------------------------------- RoIPool on an integer ramp
def ramp(h=4, w=6, c=2):
    y, x = np.mgrid[0:h, 0:w]
    return np.stack([100 * ch + 10 * y + x for ch in range(c)])[None].astype(np.float32)  # [1, c, h, w]


# (roi, expected 2x2 pooled channel-0 values), worked by hand in the comments
POOL_CASES = [
    # corners (0,0)-(5,3): roi 6 x 4 cells, bins 3 x 2 cells: max at (y, x) = (1,2), (1,5), (3,2), (3,5)
    ([0, 0.0, 0.0, 5.0, 3.0], [[12, 15], [32, 35]]),
    # round(1.4, 0.6, 3.5, 2.5) = (1, 1, 4, 3) (half away from zero): roi 4 x 3, bin 2 x 1.5 cells;
    # rows [1,3) [2,4), cols [1,3) [3,5): maxima (2,2) (2,4) (3,2) (3,4)
    ([0, 1.4, 0.6, 3.5, 2.5], [[22, 24], [32, 34]]),
    # (4,2)-(9,6) leaves the 6 x 4 map: rows [2,4) and empty [4,4); cols [4,6) and empty [6,6)
    ([0, 4.0, 2.0, 9.0, 6.0], [[35, 0], [0, 0]]),
    # a point RoI: 1 x 1 cell, every bin covers cell (2, 3) (floor/ceil of 0.5-cell bins)
    ([0, 3.0, 2.0, 3.0, 2.0], [[23, 23], [23, 23]]),
]


@pytest.mark.parametrize('i', range(len(POOL_CASES)))
def test_roi_pool_ramp_oracle(i):
    roi, want = POOL_CASES[i]
    out, _ = oracle.roi_pool(ramp(), np.array([roi], np.float32), (2, 2), 1.0)
    np.testing.assert_array_equal(out[0, 0], np.array(want, np.float32))
    np.testing.assert_array_equal(out[0, 1], np.where(np.array(want) > 0, np.array(want) + 100, 0))


@pytest.mark.gpu
def test_roi_pool_ramp_hip(dev):
    from frcnn_amd.ops import RoIPool
    rois = torch.tensor([r for r, _ in POOL_CASES], dtype=torch.float32, device=dev)
    out = RoIPool((2, 2), 1.0)(torch.from_numpy(ramp()).to(dev), rois).cpu().numpy()
    for k, (_, want) in enumerate(POOL_CASES):
        np.testing.assert_array_equal(out[k, 0], np.array(want, np.float32))
        np.testing.assert_array_equal(out[k, 1], np.where(np.array(want) > 0, np.array(want) + 100, 0))


# ----------------------------------------------------------------- NMS worked by hand
# index: box, score.  IoUs (areas without +1): A-B 90/110 = 0.818, A-C 50/150 = 0.333,
# B-C 60/140 = 0.429, A-E 1, D apart from all.  Order by score (stable): D, A, E, B, C.
NMS_BOXES = np.array([[0, 0, 10, 10], [1, 0, 11, 10], [5, 0, 15, 10], [20, 20, 30, 30], [0, 0, 10, 10]],
                     np.float32)
NMS_SCORES = np.array([0.9, 0.8, 0.7, 0.95, 0.9], np.float32)
NMS_CASES = [
    (0.5, [3, 0, 2]),     # E, B suppressed by A; C kept (0.333)
    (0.3, [3, 0]),        # C suppressed too (0.333 > 0.3)
    (0.85, [3, 0, 1, 2]),  # B kept (0.818), C kept (0.333 with A, 0.429 with B); E still (IoU 1)
    (1.0, [3, 0, 4, 1, 2]),  # nothing exceeds 1
]
# IoU == float(thr): [0,0,10,10] vs [0,0,3,10] -> 30 / 100 == float(0.3) = 0.30000001.
# torchvision CPU (float > double 0.3): suppressed; torchvision CUDA (float > float(0.3)): kept.
# This library implements the CPU rule: keep = [0].
BOUNDARY = (np.array([[0, 0, 10, 10], [0, 0, 3, 10]], np.float32), np.array([0.9, 0.8], np.float32))


@pytest.mark.parametrize('thr,keep', NMS_CASES)
def test_nms_hand_oracle(thr, keep):
    assert list(oracle.nms(NMS_BOXES, NMS_SCORES, thr)) == keep


def test_nms_boundary_rule_oracle():
    assert np.float32(30) / np.float32(100) == np.float32(0.3) and float(np.float32(0.3)) > 0.3
    assert list(oracle.nms(*BOUNDARY, 0.3)) == [0]
    assert list(oracle.nms(*BOUNDARY, 0.7)) == [0, 1]  # 0.3 IoU below 0.7


@pytest.mark.gpu
def test_nms_hand_hip(dev):
    from frcnn_amd import ops
    for thr, keep in NMS_CASES:
        got = ops.nms(torch.from_numpy(NMS_BOXES).to(dev), torch.from_numpy(NMS_SCORES).to(dev), thr)
        assert got.cpu().tolist() == keep, thr
    b, s = (torch.from_numpy(a).to(dev) for a in BOUNDARY)
    assert ops.nms(b, s, 0.3).cpu().tolist() == [0]
    assert ops.nms(b, s, 0.7).cpu().tolist() == [0, 1]

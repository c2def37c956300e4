"""CPU check of the division-free IoU threshold test used by the HIP NMS mask kernel
(pytorch-faster-rcnn_amd/csrc/nms.hip: nms_thr / iou_above).

torchvision's NMS (reference call sites lib/heads/rpn_head.py:103, lib/utils.py:220)
suppresses when float(inter / union) > double(thr).  The kernel instead compares
inter > mid * union in double, mid being the midpoint between the two floats that
bracket thr (ties: round-half-even).  This restates that rule in numpy and checks it
against the float division on values concentrated around each threshold."""
import numpy as np
import pytest


def nms_thr(thr):
    up = np.float32(thr)
    if float(up) <= thr:
        up = np.nextafter(up, np.float32(2.0))
    dn = np.nextafter(up, np.float32(0.0))
    mid = 0.5 * (float(dn) + float(up))
    tie_up = (int(np.array(up, np.float32).view(np.uint32)) & 1) == 0
    return mid, tie_up


def above_fast(inter, union, mid, tie_up):
    lhs = inter.astype(np.float64)
    rhs = mid * union.astype(np.float64)
    return (lhs > rhs) | ((lhs == rhs) & tie_up)


def above_ref(inter, union, thr):
    with np.errstate(divide='ignore', invalid='ignore'):
        return (inter / union).astype(np.float64) > thr


@pytest.mark.parametrize('thr', [0.7, 0.5, 0.3, 0.6, 0.45, 0.1])
def test_division_free_threshold_matches_division(thr):
    rng = np.random.default_rng(int(thr * 1000))
    mid, tie_up = nms_thr(thr)
    union = rng.uniform(1.0, 1e5, 400000).astype(np.float32)
    # inter around thr * union, within a few float ulps of the boundary, plus exact midpoint hits
    inter = (union.astype(np.float64) * thr * (1 + rng.integers(-64, 65, union.size) * 2 ** -24)).astype(np.float32)
    k = union.size // 4
    inter[:k] = (np.float64(mid) * union[:k].astype(np.float64)).astype(np.float32)
    inter = np.minimum(inter, union)
    fast = above_fast(inter, union, mid, tie_up)
    ref = above_ref(inter, union, thr)
    assert fast.any() and (~fast).any()
    np.testing.assert_array_equal(fast, ref)


def test_exact_midpoint_tie_rounds_half_even():
    # union = 2 makes inter = mid * 2 representable when mid has <= 24 significant bits after scaling
    for thr in (0.7, 0.5, 0.3):
        mid, tie_up = nms_thr(thr)
        for union in (np.float32(2.0), np.float32(4.0), np.float32(1024.0)):
            inter = np.float32(mid * float(union))
            if float(inter) != mid * float(union):
                continue  # midpoint not representable at this union: no tie possible
            got = above_fast(np.array([inter]), np.array([union]), mid, tie_up)[0]
            assert got == above_ref(np.array([inter]), np.array([union]), thr)[0]

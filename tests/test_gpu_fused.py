"""One-launch selections against their multi-launch forms, bit for bit.

* RPN proposals: frh_rpn_proposals_strided's one-launch selection (rpn_select_kernel:
  keys -> two-level histogram -> collect + decode -> order, phases separated by in-launch
  segment barriers) against the tools library's four-launch selection (rpn_keys / refine /
  collect / rank, frh_rpn_proposals_launches) on the same head outputs: every output
  (boxes, scores, counts) equal, over score sets that take each branch of the selection
  (all keys taken, prefix ties sorted in LDS, > 2048 prefix ties -> workgroup 0's radix
  select + the fourth barrier), both score forms (sigmoid, 2-way softmax), NCHW and
  channels-last outputs, a min-size filter, 1, 2 and 4 images, and three calls in a row on
  the same shapes (workspace reuse).  The reference semantics of the selection are pinned
  by test_gpu_parity.py (rpn fixtures, tie-heavy oracle cases), which run the one-launch path.
* RPN NMS: frh_rpn_proposals_strided's one-launch NMS (nms_fused_kernel: the mask tiles and
  the scan of every segment in one launch, tile flags between them) against the tools
  library's two-launch NMS (mask kernel, then scan kernel; frh_rpn_proposals_nms2) on the
  same selection: outputs equal, over segments of 5..125 blocks (scans of more than 64
  columns poll their flags in two loads), a post_nms cut that stops the scan early,
  tie-heavy and sparse score sets, 1, 2 and 4 images, three calls in a row (the flags are
  zeroed per call).  The two-launch NMS is pinned by test_gpu_parity.py's oracle cases.
  After the one-launch NMS (which also writes the kept rows' scores compactly) the merge runs
  as rpn_merge_wide_kernel (one survivor per thread, ~40 workgroups) where (levels - 1) x P
  scores fit its LDS: the same comparison covers it -- the reference side runs the round-4
  rpn_merge_lds_kernel -- with a cut (the bench's call), without one (total <= max_num) and
  with post_nms stopping the scans; P = 8000 takes the old merge.  frh_rpn_proposals_merge_launch
  (the one-launch NMS, then rpn_merge_lds_kernel) is compared too.
* Device sampler: frh_sample_random's one-launch sampler (sampler_fused_kernel) against the
  tools library's keys + collect launches (frh_sample_random_launches): labels, selection
  sets and counts equal; the workspace's zero region is zero after every call.  The sampler's
  definition is pinned by test_gpu_parity.py's numpy restatement (test_device_sampler_*).
"""
import os
import sys

import numpy as np
import pytest
import torch

import inputs

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tools():
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    import toolslib
    return toolslib.load()


def _scores(case, rng, c):
    if case == 'all_equal':
        c[...] = 0.0
    elif case == 'four_values':
        c[...] = rng.choice(np.array([-1.0, 0.0, 0.5, 2.0], np.float32), size=c.shape)
    elif case == 'sparse_high':
        c[...] = -5.0
        flat = c.reshape(-1)
        m = min(flat.size, 150)
        flat[rng.choice(flat.size, m, replace=False)] = rng.uniform(1, 3, m)
    elif case == 'near_half':
        c[...] = (rng.integers(-4000, 4001, c.shape) * 1e-6).astype(np.float32)
    elif case == 'random_init':  # the bench's regime: scores within ~3e-3 of 0.5
        c[...] = (rng.standard_normal(c.shape) * 0.01).astype(np.float32)


def _run(dev, case, cls_ch, nhwc, batch, min_size, pre, post, mx, seed, other='frh_rpn_proposals_launches'):
    from frcnn_amd import ops
    from frcnn_amd.heads.rpn_head import RPNHead
    head = RPNHead(256, 256, loss_cls=dict(type='CrossEntropyLoss', use_sigmoid=cls_ch == 1),
                   loss_bbox=dict(type='SmoothL1Loss', beta=1.0 / 9.0)).to(dev)
    anchors = head._flat_anchors(inputs.FPN_GRIDS, dev)
    rng = np.random.default_rng(seed)
    cls, reg = inputs.head_outputs(seed, inputs.FPN_GRIDS, 3, cls_ch, batch=batch, reg_scale=0.5)
    for c in cls:
        _scores(case, rng, c)
    cls = [torch.from_numpy(c).to(dev) for c in cls]
    reg = [torch.from_numpy(r).to(dev) for r in reg]
    if nhwc:
        cls = [c.contiguous(memory_format=torch.channels_last) for c in cls]
        reg = [r.contiguous(memory_format=torch.channels_last) for r in reg]
    lib = _tools()
    args = (cls, reg, anchors, 3, cls_ch, [0.0] * 4, [1.0] * 4, [(600.0, 1000.0)] * batch, [min_size] * batch,
            pre, post, mx, 0.7)
    fused = [ops.rpn_proposals(*args) for _ in range(3)]
    launches = ops.rpn_proposals(*args, _entry=(getattr(lib, other), other))
    torch.cuda.synchronize()
    return fused, launches


@pytest.mark.parametrize('case,cls_ch,nhwc,batch,min_size', [
    ('random_init', 1, True, 2, 0.0),
    ('random_init', 2, False, 2, 0.0),
    ('random_init', 1, False, 4, 16.0),
    ('near_half', 1, True, 1, 0.0),
    ('four_values', 2, True, 2, 16.0),
    ('sparse_high', 1, False, 2, 0.0),
    ('all_equal', 1, False, 2, 0.0),
    ('all_equal', 2, True, 1, 16.0),
])
def test_rpn_one_launch_selection_equals_four_launches(dev, case, cls_ch, nhwc, batch, min_size):
    fused, ref = _run(dev, case, cls_ch, nhwc, batch, min_size, 2000, 2000, 2000, 40 + batch)
    rb, rs, rc = ref
    for fb, fs, fc in fused:
        assert torch.equal(fc, rc), (fc, rc)
        for i, n in enumerate(rc.tolist()):
            assert torch.equal(fb[i, :, :n], rb[i, :, :n]), (case, i)
            assert torch.equal(fs[i, :n], rs[i, :n]), (case, i)


@pytest.mark.parametrize('pre,post,mx', [(1000, 1000, 1000), (300, 300, 600), (2048, 2048, 1000)])
def test_rpn_one_launch_selection_pre_nms_sizes(dev, pre, post, mx):
    """pre_nms at the test config (1000), small (300: every level but the last cut), and at
    the one-launch path's record capacity (2048)."""
    fused, ref = _run(dev, 'random_init', 1, True, 2, 0.0, pre, post, mx, 77)
    rb, rs, rc = ref
    fb, fs, fc = fused[-1]
    assert torch.equal(fc, rc)
    for i, n in enumerate(rc.tolist()):
        assert torch.equal(fb[i, :, :n], rb[i, :, :n])
        assert torch.equal(fs[i, :n], rs[i, :n])


@pytest.mark.parametrize('case,batch,pre,post,mx', [
    ('random_init', 2, 2000, 2000, 2000),   # the bench's call
    ('random_init', 2, 2000, 300, 1000),    # post_nms stops every scan early
    ('four_values', 1, 1000, 1000, 1000),
    ('sparse_high', 2, 2000, 2000, 2000),
    ('near_half', 4, 2000, 2000, 4000),
    ('random_init', 1, 4000, 3000, 4000),   # 63 blocks (four-launch selection)
    ('random_init', 1, 8000, 2000, 2000),   # 125 blocks: column flags polled in two loads
    ('sparse_high', 2, 300, 300, 4000),     # no cut: the merge keeps the level concatenation
])
@pytest.mark.parametrize('other', ['frh_rpn_proposals_nms2', 'frh_rpn_proposals_merge_launch'])
def test_rpn_one_launch_nms_equals_two_launches(dev, case, batch, pre, post, mx, other):
    fused, ref = _run(dev, case, 1, True, batch, 0.0, pre, post, mx, 90 + batch, other=other)
    rb, rs, rc = ref
    assert int(rc.min()) > 0
    for fb, fs, fc in fused:
        assert torch.equal(fc, rc), (fc, rc)
        for i, n in enumerate(rc.tolist()):
            assert torch.equal(fb[i, :, :n], rb[i, :, :n]), (case, i)
            assert torch.equal(fs[i, :n], rs[i, :n]), (case, i)


# ------------------------------------------------------------------ device sampler
def _labels(rng, S, n, p):
    lab = rng.choice([-1, 0, 1, 2, 3], size=(S, n), p=p).astype(np.int64)
    return lab


@pytest.mark.parametrize('S,n,nums,max_num,pos_num,p', [
    (2, 155520, None, 256, 128, [0.30, 0.68, 0.01, 0.005, 0.005]),   # the cfg2 RPN call
    (2, 155520, None, 256, 128, [0.30, 0.6999, 0.0001, 0.0, 0.0]),  # few positives: negatives fill
    (4, 40000, [40000, 16385, 0, 39999], 512, 128, [0.3, 0.6, 0.04, 0.03, 0.03]),  # ragged, empty image
    (1, 2000000, None, 4096, 1024, [0.0, 1.0, 0.0, 0.0, 0.0]),  # > 4096 prefix ties: radix threshold
    (2, 20000, None, 256, 128, [0.999, 0.0005, 0.0005, 0.0, 0.0]),  # fewer candidates than slots
])
def test_sampler_one_launch_equals_two_launches(dev, S, n, nums, max_num, pos_num, p):
    """frh_sample_random's one-launch sampler (images above 16 384 boxes) against the tools
    library's keys + collect launches: same sampled labels, same selection sets and counts;
    three calls in a row with different draws on one workspace (its zero region is left
    zero by every call)."""
    from frcnn_amd import ops
    lib = _tools()
    rng = np.random.default_rng(S * 7 + n)
    num = torch.tensor(nums if nums else [n] * S, dtype=torch.int32, device=dev)
    for call in range(3):
        lab = torch.from_numpy(_labels(rng, S, n, p)).to(dev)
        res = []
        for entry in (None, (lib.frh_sample_random_launches, 'frh_sample_random_launches')):
            outs = []
            for lists in (False, True):
                ops.set_sampler_mode('device', seed=100 + call)
                outs.append(ops.sample_labels(lab, num, n, max_num, pos_num, mode='device', lists=lists,
                                              _entry=entry))
            res.append(outs)
        torch.cuda.synchronize()
        (a_lab, a_sl), (b_lab, b_sl) = res
        for s, ns in enumerate(num.tolist()):
            assert torch.equal(a_lab[s, :ns], b_lab[s, :ns]), (call, s)
        assert torch.equal(a_sl.sel_counts, b_sl.sel_counts), (call, a_sl.sel_counts, b_sl.sel_counts)
        for s in range(S):
            for c in range(2):
                k = int(a_sl.sel_counts[s, c])
                assert torch.equal(torch.sort(a_sl.sel[s, c, :k])[0], torch.sort(b_sl.sel[s, c, :k])[0]), (call, s, c)
        zb = int(ops._lib.query('frh_sample_zero_bytes', S))
        assert ops._SAMPLE_WS and all(int(ws[:zb].count_nonzero()) == 0 for ws in ops._SAMPLE_WS.values())
    ops.set_sampler_mode('numpy')


def test_sampler_workspace_reuse_across_num_segs_and_paths(dev):
    """a two-launch call (keys at the end of the zero region) with S = 2, then a
    one-launch call with S = 4 on the same cached workspace, dense positives: the zero region
    is the same for every S (frh_sample_zero_bytes), so the S = 4 call equals one on a fresh
    workspace."""
    from frcnn_amd import ops
    lib = _tools()
    rng = np.random.default_rng(11)
    n = 40000
    lab2 = torch.from_numpy(rng.choice([0, 1, 2], size=(2, n), p=[0.2, 0.4, 0.4]).astype(np.int64)).to(dev)
    lab4 = torch.from_numpy(rng.choice([0, 1, 2], size=(4, n), p=[0.2, 0.4, 0.4]).astype(np.int64)).to(dev)
    num2 = torch.full((2,), n, dtype=torch.int32, device=dev)
    num4 = torch.full((4,), n, dtype=torch.int32, device=dev)
    assert ops._lib.query('frh_sample_zero_bytes', 2) == ops._lib.query('frh_sample_zero_bytes', 64)
    ops._SAMPLE_WS.clear()
    ops.set_sampler_mode('device', seed=5)
    fresh = ops.sample_labels(lab4, num4, n, 512, 128, mode='device')
    ops._SAMPLE_WS.clear()
    ops.set_sampler_mode('device', seed=6)
    ops.sample_labels(lab2, num2, n, 512, 128, mode='device', _entry=(lib.frh_sample_random_launches, 'launches'))
    ops.set_sampler_mode('device', seed=5)
    reused = ops.sample_labels(lab4, num4, n, 512, 128, mode='device')
    torch.cuda.synchronize()
    ops.check_device_status(dev)
    assert torch.equal(fresh, reused)
    ops.set_sampler_mode('numpy')


@pytest.mark.parametrize('n,max_num,pos_num,p,fast', [
    (155520, 256, 128, [0.30, 0.68, 0.01, 0.005, 0.005], True),    # cfg2 RPN: positives cut in the window
    (155520, 256, 128, [0.30, 0.6999, 0.0001, 0.0, 0.0], True),   # few positives: all taken
    (40000, 512, 128, [0.3, 0.6, 0.04, 0.03, 0.03], False),       # > 256 positives in a chunk row
    (20000, 256, 128, [0.999, 0.0005, 0.0005, 0.0, 0.0], False),  # every negative taken, few in the window
])
def test_sampler_window_fast_path(dev, n, max_num, pos_num, p, fast):
    """The one-launch sampler's window-record path (round 6) is the one taken when the window
    holds the selection, and the histogram phases otherwise (stamp 9 of every workgroup of the
    tools timing build); either way the result equals the keys + collect launches."""
    from frcnn_amd import ops, _lib
    lib = _tools()
    S = 2
    rng = np.random.default_rng(n + max_num)
    lab = torch.from_numpy(_labels(rng, S, n, p)).to(dev)
    num = torch.full((S,), n, dtype=torch.int32, device=dev)
    sst = torch.zeros(S, (n + 4095) // 4096, 16, dtype=torch.int64, device=dev)

    def stamped(*a):
        a = list(a)
        stream = a.pop()
        return lib.frh_sample_random_stamped(*a, _lib.ptr(sst), stream)
    res = []
    for entry in ((stamped, 'stamped'), (lib.frh_sample_random_launches, 'frh_sample_random_launches')):
        for lists in (False, True):
            ops.set_sampler_mode('device', seed=77)
            res.append(ops.sample_labels(lab, num, n, max_num, pos_num, mode='device', lists=lists, _entry=entry))
    a_lab, a_sl, b_lab, b_sl = res
    torch.cuda.synchronize()
    ops.check_device_status(dev)
    st = sst.cpu().numpy()
    assert (st[:, :, 0] > 0).all()
    assert bool((st[:, :, 9] > 0).all()) == fast and bool((st[:, :, 9] > 0).any()) == fast
    assert torch.equal(a_lab, b_lab)
    assert torch.equal(a_sl.sel_counts, b_sl.sel_counts)
    for s in range(S):
        for c in range(2):
            k = int(a_sl.sel_counts[s, c])
            assert torch.equal(torch.sort(a_sl.sel[s, c, :k])[0], torch.sort(b_sl.sel[s, c, :k])[0]), (s, c)
    ops.set_sampler_mode('numpy')

"""The device status word (include/frcnn_amd.h FRH_DEVERR_*, ABI 2; loss entries take it, ABI 3).

The one-launch kernels (rpn_select_kernel, nms_fused_kernel, sampler_fused_kernel) hand data
between workgroups of one launch through bounded waits.  A wait that runs out must surface
as an error -- the kernel ORs a bit into the caller's status word and stops its work, and
frcnn_amd.ops.check_device_status() raises -- never as a silently wrong selection or keep
list (reference semantics that would break: lib/heads/rpn_head.py:68-120,
lib/region.py:43-57).  tools/lib/libfrcnn_spin.so is the product library rebuilt with
FRH_SPIN_TICKS=0: every wait not met at its first poll runs out at once."""
import ctypes
import os

import numpy as np
import pytest
import torch

import inputs

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPIN = os.path.join(REPO, 'tools', 'lib', 'libfrcnn_spin.so')


def _spin():
    from frcnn_amd import _lib
    if not os.path.exists(SPIN):
        pytest.fail('{} missing: python tools/build_tools.py'.format(SPIN))
    lib = ctypes.CDLL(SPIN)
    for name in ('frh_rpn_proposals_strided', 'frh_sample_random'):
        res, args = _lib.SIGNATURES[name]
        getattr(lib, name).restype, getattr(lib, name).argtypes = res, args
    return lib


def _rpn_inputs(dev, batch=2):
    from frcnn_amd.heads.rpn_head import RPNHead
    head = RPNHead(256, 256, loss_cls=dict(type='CrossEntropyLoss', use_sigmoid=True),
                   loss_bbox=dict(type='SmoothL1Loss', beta=1.0 / 9.0)).to(dev)
    anchors = head._flat_anchors(inputs.FPN_GRIDS, dev)
    cls, reg = inputs.head_outputs(5, inputs.FPN_GRIDS, 3, 1, batch=batch, cls_scale=0.01, reg_scale=0.5)
    cls = [torch.from_numpy(c).to(dev).contiguous(memory_format=torch.channels_last) for c in cls]
    reg = [torch.from_numpy(r).to(dev).contiguous(memory_format=torch.channels_last) for r in reg]
    return (cls, reg, anchors, 3, 1, [0.0] * 4, [1.0] * 4, [(600.0, 1000.0)] * batch, [0.0] * batch,
            2000, 2000, 2000, 0.7)


def test_status_word_stays_zero_on_the_product_path(dev):
    from frcnn_amd import ops
    args = _rpn_inputs(dev)
    for _ in range(3):
        ops.rpn_proposals(*args)
    lab = torch.from_numpy(np.random.default_rng(1).choice([-1, 0, 1], size=(2, 155520), p=[0.3, 0.69, 0.01])).to(dev)
    num = torch.full((2,), 155520, dtype=torch.int32, device=dev)
    ops.sample_labels(lab, num, 155520, 256, 128, mode='device')
    ops.check_device_status(dev)  # no raise
    assert int(ops.status_word(dev).item()) == 0


def test_rpn_wait_timeout_raises_not_wrong_proposals(dev):
    """RPN proposals through the zero-spin library: the selection's segment barriers and the
    one-launch NMS's column waits run out; the status word carries their bits and
    check_device_status raises.  The product path afterwards is clean and matches the
    outputs of a fresh call."""
    from frcnn_amd import ops
    lib = _spin()
    args = _rpn_inputs(dev)
    ref = ops.rpn_proposals(*args)
    ops.rpn_proposals(*args, _entry=(lib.frh_rpn_proposals_strided, 'spin'))
    torch.cuda.synchronize()
    v = int(ops.status_word(dev).item())
    assert v & 1, v  # FRH_DEVERR_SELECT_BARRIER (the NMS then runs on whatever the aborted selection left)
    with pytest.raises(RuntimeError, match='in-launch wait timed out'):
        ops.check_device_status(dev)
    assert int(ops.status_word(dev).item()) == 0  # cleared by the check
    again = ops.rpn_proposals(*args)
    ops.check_device_status(dev)
    for a, b in zip(ref, again):
        assert torch.equal(a, b)


def test_sampler_wait_timeout_raises(dev):
    from frcnn_amd import ops
    lib = _spin()
    lab = torch.from_numpy(np.random.default_rng(2).choice([-1, 0, 1], size=(2, 155520), p=[0.3, 0.69, 0.01])).to(dev)
    num = torch.full((2,), 155520, dtype=torch.int32, device=dev)
    ops.set_sampler_mode('device', seed=3)
    ref = ops.sample_labels(lab, num, 155520, 256, 128, mode='device')
    ops.set_sampler_mode('device', seed=3)
    ops.sample_labels(lab, num, 155520, 256, 128, mode='device', _entry=(lib.frh_sample_random, 'spin'))
    torch.cuda.synchronize()
    assert int(ops.status_word(dev).item()) & 4
    # a product call with no check in between: the aborted launch may have left its zero region
    # dirty, so the one-launch sampler must not run on it (it returns at once while the word is
    # set) and must not clear the bit
    ops.set_sampler_mode('device', seed=3)
    ops.sample_labels(lab, num, 155520, 256, 128, mode='device')
    torch.cuda.synchronize()
    assert int(ops.status_word(dev).item()) & 4
    with pytest.raises(RuntimeError, match='device sampler image barrier'):
        ops.check_device_status(dev)
    assert not ops._SAMPLE_WS  # the possibly dirty zero-contract workspace was dropped
    ops.set_sampler_mode('device', seed=3)
    again = ops.sample_labels(lab, num, 155520, 256, 128, mode='device')
    ops.check_device_status(dev)
    assert torch.equal(ref, again)
    ops.set_sampler_mode('numpy')


def test_one_launch_nms_column_timeout_sets_its_bit(dev):
    """The one-launch NMS alone (tools entry, valid inputs) in the zero-spin build: its loaders'
    column waits run out, the scan stops (the kept counts stay within the segment) and
    FRH_DEVERR_NMS_COLUMN is set."""
    import sys
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    from frcnn_amd import ops, _lib
    lib = ctypes.CDLL(SPIN)
    fn = lib.frh_nms_fused_stamped
    import toolslib
    fn.restype, fn.argtypes = toolslib.TOOL_SIGNATURES['frh_nms_fused_stamped']
    S, P = 4, 2000
    rng = np.random.default_rng(9)
    xy = rng.uniform(0, 900, (S, P, 2)).astype(np.float32)
    wh = rng.uniform(8, 120, (S, P, 2)).astype(np.float32)
    rows = torch.from_numpy(np.concatenate([xy, xy + wh], 2)).to(dev)
    cnt = torch.full((S,), P, dtype=torch.int32, device=dev)
    keep = torch.empty(S, P, dtype=torch.int32, device=dev)
    kc = torch.empty(S, dtype=torch.int32, device=dev)
    nb = int(_lib.query('frh_nms_workspace', S, P)) + int(fn_flags(lib)(S, P))
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    r = fn(S, _lib.ptr(rows), rows.stride(0), _lib.ptr(cnt), P, 0.7, -1, _lib.ptr(keep), keep.stride(0), _lib.ptr(kc),
           _lib.ptr(ops.status_word(dev)), _lib.ptr(ws), ws.numel(), None, _lib.stream_of(rows))
    assert r == 0
    torch.cuda.synchronize()
    assert int(ops.status_word(dev).item()) & 2
    assert int(kc.min()) >= 0 and int(kc.max()) <= P
    with pytest.raises(RuntimeError, match='RPN NMS mask column'):
        ops.check_device_status(dev)


def fn_flags(lib):
    f = lib.frh_nms_fused_flag_bytes
    f.restype, f.argtypes = ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32]
    return f


def _spin_proposals(monkeypatch):
    import functools
    from frcnn_amd import ops
    lib = _spin()
    monkeypatch.setattr(ops, 'rpn_proposals',
                        functools.partial(ops.rpn_proposals, _entry=(lib.frh_rpn_proposals_strided, 'spin')))


def test_timed_out_wait_fails_the_same_step(dev, monkeypatch):
    """VERDICT r05 Missing 2: a cfg2 forward_train whose RPN selection barrier runs out (the
    zero-spin proposals) returns non-finite losses in that same call -- the loss kernels read
    the status word (ABI 3) -- and check_device_status names the bit.  TrainStep, without a host
    sync: NaN loss, the update skipped on the device (fused SGD found_inf: parameters unchanged),
    the next call raises; with status_every=1 it raises inside the failed step, before its update.
    Reference loop: lib/trainer/trainer.py:110-119 reads every loss each iteration."""
    import sys
    sys.path.insert(0, REPO)
    import bench
    from frcnn_amd import ops, set_sampler_mode
    from frcnn_amd.train import TrainStep
    set_sampler_mode('device', seed=5)
    model, cfg = bench.make_model(dev, seed=0)
    batch = bench.make_batch(dev, 2, seed=0)
    ops.check_device_status(dev)
    with torch.no_grad():
        clean = model.forward_train(*batch)
    assert all(bool(torch.isfinite(v)) for v in clean.values())
    _spin_proposals(monkeypatch)
    with torch.no_grad():
        losses = model.forward_train(*batch)
    bad = [k for k, v in losses.items() if not bool(torch.isfinite(v))]
    assert bad, {k: float(v) for k, v in losses.items()}
    assert any('rcnn' in k or 'cls' in k for k in bad), bad
    with pytest.raises(RuntimeError, match='RPN selection segment barrier'):
        ops.check_device_status(dev)
    # TrainStep, no host sync: the failed step's losses are NaN and its update is skipped on the
    # device (fused SGD found_inf); the next call raises once the step's status copy has landed
    before = [p.detach().clone() for p in model.parameters() if p.requires_grad]
    step = TrainStep(model, cfg.optimizer, cfg.optimizer_config.get('grad_clip'))
    assert step.device.index == dev.index  # taken from the parameters
    loss = step(*batch)
    torch.cuda.synchronize()
    assert not bool(torch.isfinite(loss))
    after = [p.detach() for p in model.parameters() if p.requires_grad]
    assert all(torch.equal(a, b) for a, b in zip(before, after))  # no update from the failed step
    with pytest.raises(RuntimeError, match='in-launch wait timed out'):
        step(*batch)
    assert int(ops.status_word(dev).item()) == 0
    # the synchronous form raises inside the failed step, before its update
    sync_step = TrainStep(model, cfg.optimizer, cfg.optimizer_config.get('grad_clip'), status_every=1)
    with pytest.raises(RuntimeError, match='in-launch wait timed out'):
        sync_step(*batch)
    assert all(torch.equal(a, b) for a, b in zip(before, [p.detach() for p in model.parameters() if p.requires_grad]))
    # a clean step after the failures updates normally (momentum buffers defined)
    monkeypatch.undo()
    good = step(*batch)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(good))
    moved = [not torch.equal(a, b.detach()) for a, b in zip(before, [p for p in model.parameters() if p.requires_grad])]
    assert sum(moved) > len(moved) // 2
    assert all(bool(torch.isfinite(p).all()) for p in model.parameters())
    ops.check_device_status(dev)
    set_sampler_mode('numpy')

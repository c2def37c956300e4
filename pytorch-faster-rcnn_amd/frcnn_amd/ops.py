"""Tensor-level wrappers of the HIP kernels (one function per C-ABI entry).

These take/return torch tensors resident on the HIP device, allocate outputs
and workspaces with the caching allocator and launch on the current stream.
The reference-API modules (anchor, region, bbox, utils, heads) are built on
these.  The torchvision drop-ins the reference imports (`nms`, `roi_align`,
`RoIAlign`, `RoIPool`) live here too.
"""
import ctypes
import os
import warnings

import numpy as np
import torch
from torch import nn

from . import _lib
from ._lib import call as _call, ptr, stream_of, i32_array, i64_array, f32_array, ptr_array, workspace


def call(name, *args):
    """_lib.call; a failed entry point drops the zero-contract workspaces (their counters
    are left zero only by calls that ran to completion), so the next call starts from
    freshly zeroed buffers."""
    try:
        _call(name, *args)
    except RuntimeError:
        _drop_zero_workspaces()
        raise


def _drop_zero_workspaces():
    for ws in (_ASSIGN_WS, _SAMPLE_WS, _LOSS_WS):
        ws.clear()


# ---------------------------------------------------------------- device status word
# include/frcnn_amd.h FRH_DEVERR_*: the one-launch kernels (RPN selection, RPN NMS, device
# sampler) OR a bit into this per-device int32 word when an in-launch wait runs out, and
# end that workgroup's work.  The word is read (one 4-byte copy, a synchronisation) by
# check_device_status(): at the points that synchronise anyway -- the numpy sampler's count
# read, bench.py's loss read after the timed region, the tester -- and after every one-launch
# call when FRCNN_AMD_DEBUG=1.
DEVERR_BITS = {1: 'RPN selection segment barrier (rpn_select_kernel)',
               2: 'RPN NMS mask column wait (nms_fused_kernel)',
               4: 'device sampler image barrier (sampler_fused_kernel)'}
_STATUS = {}
DEBUG = os.environ.get('FRCNN_AMD_DEBUG', '') not in ('', '0')


def _device_key(dev):
    """Device index of `dev`; a bare 'cuda' device means the current device (both the word's
    owner and its checker resolve it this way)."""
    d = torch.device(dev)
    return d.index if d.index is not None else torch.cuda.current_device()


def status_word(dev):
    """The device status word of `dev` (int32 [1], zero until a one-launch kernel flags)."""
    key = _device_key(dev)
    w = _STATUS.get(key)
    if w is None:
        w = _STATUS[key] = torch.zeros(1, dtype=torch.int32, device=torch.device('cuda', key))
    return w


def check_device_status(dev=None):
    """Raise RuntimeError if a one-launch kernel on `dev` (default: every device used) flagged
    a timed-out in-launch wait since the last check.  Synchronises with the word's device.
    The word is cleared and the zero-contract workspaces are dropped (their counters may be
    left dirty by the aborted launch), so later calls start clean."""
    keys = list(_STATUS) if dev is None else [_device_key(dev)]
    for k in keys:
        w = _STATUS.get(k)
        if w is None:
            continue
        v = int(w.item())
        if v:
            w.zero_()
            _drop_zero_workspaces()
            what = ', '.join(m for b, m in DEVERR_BITS.items() if v & b) or 'unknown'
            raise RuntimeError('frcnn_amd: device status 0x{:x} on cuda:{}: an in-launch wait timed out ({}); '
                               'the outputs of that call are undefined'.format(v, k, what))


def _debug_check(dev):
    if DEBUG:
        check_device_status(dev)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('frcnn_amd: HIP device tensors required (got {})'.format(t.device))


def _f32(t):
    return t if t.dtype == torch.float32 else t.float()


# ---------------------------------------------------------------- anchors (a1/a2)
def anchor_grid(grid_sizes, strides, ws, hs, num_anchors, center_lt, device):
    """All levels' anchors as one [4, N] tensor (reference AnchorCreator per level, concatenated)."""
    L = len(grid_sizes)
    n = sum(num_anchors * int(h) * int(w) for h, w in grid_sizes)
    out = torch.empty(4, max(n, 1), dtype=torch.float32, device=device)[:, :n]
    ws_t = torch.tensor(ws, dtype=torch.float32, device=device)
    hs_t = torch.tensor(hs, dtype=torch.float32, device=device)
    hw = i32_array([v for g in grid_sizes for v in (int(g[0]), int(g[1]))])
    call('frh_anchor_grid', L, hw, f32_array(strides), ptr(ws_t), ptr(hs_t), num_anchors,
         int(bool(center_lt)), ptr(out), out.stride(0), stream_of(out))
    return out


def inside_mask(anchors, grid_sizes, in_sizes, num_anchors, img_h, img_w, allowed_border):
    _need_cuda(anchors)
    n = anchors.shape[1]
    mask = torch.empty(n, dtype=torch.uint8, device=anchors.device)
    hw = i32_array([v for g in grid_sizes for v in (int(g[0]), int(g[1]))])
    ihw = i32_array([v for g in in_sizes for v in (int(g[0]), int(g[1]))])
    call('frh_inside_mask', ptr(anchors), anchors.stride(0), len(grid_sizes), hw, ihw, num_anchors,
         int(img_h), int(img_w), int(allowed_border), ptr(mask), stream_of(anchors))
    return mask


# ---------------------------------------------------------------- IoU (a3)
def iou_table(a, b):
    _need_cuda(a, b)
    a, b = _f32(a), _f32(b)
    if a.stride(1) != 1:
        a = a.contiguous()
    if b.stride(1) != 1:
        b = b.contiguous()
    n, k = a.shape[1], b.shape[1]
    out = torch.empty(n, k, dtype=torch.float32, device=a.device)
    call('frh_iou_table', ptr(a), a.stride(0), n, ptr(b), b.stride(0), k, ptr(out), stream_of(a))
    return out


def elem_iou(a, b):
    _need_cuda(a, b)
    a, b = _f32(a).contiguous(), _f32(b).contiguous()
    n = a.shape[1]
    out = torch.empty(n, dtype=torch.float32, device=a.device)
    call('frh_elem_iou', ptr(a), a.stride(0), ptr(b), b.stride(0), n, ptr(out), stream_of(a))
    return out


# ---------------------------------------------------------------- packing helpers
def device_ints(vals, device, dtype=torch.int32):
    """Small host list -> device tensor without a stream synchronisation
    (pinned staging + non_blocking copy; a pageable copy would block)."""
    t = torch.tensor(list(vals), dtype=dtype)
    if device.type != 'cuda':
        return t
    return t.pin_memory().to(device, non_blocking=True)


_PACKED = []  # (inputs, their versions, key, result): the packs of the last few distinct input lists


def _memo(inputs, key, make):
    """A batch's gt boxes / labels are packed once and reused by the RPN and every RCNN stage:
    hit only for the same tensor objects (held by the entry, so their storage cannot be
    reused) with unchanged version counters, on the same stream (a pack is made on the
    current stream and read in stream order).  Detectors drop the entries at the end of
    each forward_train (release_packs)."""
    dev = key[1]
    if isinstance(dev, torch.device) and dev.type == 'cuda':
        key = key + (torch.cuda.current_stream(dev).cuda_stream,)
    vers = tuple(t._version for t in inputs)
    for ent in _PACKED:
        if ent[2] == key and len(ent[0]) == len(inputs) and all(a is b for a, b in zip(ent[0], inputs)) \
                and ent[1] == vers:
            return ent[3]
    res = make()
    _PACKED.insert(0, (tuple(inputs), vers, key, res))
    del _PACKED[8:]
    return res


def release_packs():
    """Forget the memoised gt packs (end of a forward_train)."""
    del _PACKED[:]


def pack_boxes(box_list, device, min_cols=1):
    """list of [4, n_i] -> ([S, 4, n_max] f32, counts int32 device, n_max)."""
    if all(torch.is_tensor(b) and b.dtype == torch.float32 for b in box_list):
        return _memo(list(box_list), ('boxes', device, min_cols), lambda: _pack_boxes(box_list, device, min_cols))
    return _pack_boxes(box_list, device, min_cols)


def _pack_boxes(box_list, device, min_cols):
    S = len(box_list)
    nmax = max([int(b.shape[1]) for b in box_list] + [min_cols])
    out = torch.zeros(S, 4, nmax, dtype=torch.float32, device=device)
    for s, b in enumerate(box_list):
        if b.shape[1]:
            out[s, :, :b.shape[1]] = b
    counts = device_ints([int(b.shape[1]) for b in box_list], device)
    return out, counts, nmax


def pack_labels(label_list, nmax, device):
    if all(torch.is_tensor(l) for l in label_list):
        return _memo(list(label_list), ('labels', device, nmax), lambda: _pack_labels(label_list, nmax, device))
    return _pack_labels(label_list, nmax, device)


def _pack_labels(label_list, nmax, device):
    S = len(label_list)
    out = torch.zeros(S, max(nmax, 1), dtype=torch.int64, device=device)
    for s, l in enumerate(label_list):
        if l.numel():
            out[s, :l.numel()] = l.to(torch.int64)
    return out


# ---------------------------------------------------------------- MaxIoU assignment (a4)
_ASSIGN_WS = {}


def _assign_workspace(dev, S, mg, max_boxes):
    """One buffer per (device, stream): its leading counters / maxima are zero-filled when
    the (segments, gts) layout changes; every call leaves them zero."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    need = int(_lib.query('frh_maxiou_assign_workspace', S, mg, max_boxes))
    layout = (S, mg)
    ent = _ASSIGN_WS.get(key)
    if ent is None or ent[1].numel() < need:
        ent = _ASSIGN_WS[key] = [layout, torch.zeros(need, dtype=torch.uint8, device=dev)]
    elif ent[0] != layout:
        ent[1][:int(_lib.query('frh_maxiou_assign_zero_bytes', S, mg))].zero_()
        ent[0] = layout
    return ent[1]

def maxiou_assign(boxes, box_seg_stride, num_boxes, max_boxes, gts, gt_counts, max_gts, pos_iou, neg_iou,
                  min_pos_iou, valid=None, valid_seg_stride=0, num_segs=None):
    """Batched MaxIoUAssigner: boxes [.., 4, ld] (segment stride given), gts [S, 4, Gmax]."""
    _need_cuda(boxes, gts)
    S = num_segs if num_segs is not None else gts.shape[0]
    dev = boxes.device
    labels = torch.empty(S, max(max_boxes, 1), dtype=torch.int64, device=dev)
    max_iou = torch.empty(S, max(max_boxes, 1), dtype=torch.float32, device=dev)
    ws = _assign_workspace(dev, S, max(max_gts, 1), max_boxes)
    call('frh_maxiou_assign', S, ptr(boxes), boxes.stride(-2), box_seg_stride, ptr(num_boxes),
         ptr(valid), valid_seg_stride, ptr(gts), gts.stride(1), gts.stride(0), ptr(gt_counts),
         float(pos_iou), float(neg_iou), float(min_pos_iou), ptr(labels), labels.stride(0), ptr(max_iou),
         max_iou.stride(0), max_boxes, max_gts, ptr(ws), ws.numel(), stream_of(boxes))
    return labels, max_iou


# ---------------------------------------------------------------- sampling (a5)
_SAMPLER = {'mode': 'numpy', 'seed': 0x5eed, 'calls': 0}


def set_sampler_mode(mode, seed=None):
    """'numpy' = the reference's np.random stream (exact parity, host round trip);
    'device' = on-device hash RNG (same distribution, no sync)."""
    if mode not in ('numpy', 'device'):
        raise ValueError("sampler mode must be 'numpy' or 'device'")
    _SAMPLER['mode'] = mode
    if seed is not None:
        _SAMPLER['seed'] = int(seed)
        _SAMPLER['calls'] = 0


def sampler_mode():
    return _SAMPLER['mode']


class SampleLists(object):
    """The device sampler's selection (frh_sample_random's sel / sel_counts): per segment the
    kept positives and negatives, in no order, for the target gathers; `labels` are the
    assignment labels they select from (unchanged)."""

    def __init__(self, labels, sel, sel_counts, max_num):
        self.labels, self.sel, self.sel_counts, self.max_num = labels, sel, sel_counts, int(max_num)


_SAMPLE_WS = {}


def _sample_workspace(dev, S, max_boxes):
    """One buffer per (device, stream) for frh_sample_random: zero-filled once; every call
    leaves its leading frh_sample_zero_bytes(S) bytes zero (the one-launch sampler's counters
    and histograms), so it is reused as is."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    need = int(_lib.query('frh_sample_workspace', S, max_boxes))
    ws = _SAMPLE_WS.get(key)
    if ws is None or ws.numel() < need:
        ws = _SAMPLE_WS[key] = torch.zeros(need, dtype=torch.uint8, device=dev)
    return ws


def sample_labels(labels, num_boxes, max_boxes, max_num, pos_num, mode=None, lists=False, _entry=None):
    """Batched RandomSampler over labels [S, >=max_boxes] (region.py:43-57,112-126).
    lists=True (device mode only): return a SampleLists instead of the sampled labels."""
    mode = mode or _SAMPLER['mode']
    S = labels.shape[0]
    dev = labels.device
    if mode == 'device':
        ws = _sample_workspace(dev, S, max(max_boxes, 1))
        _SAMPLER['calls'] += 1
        seed = (_SAMPLER['seed'] * 0x9E3779B97F4A7C15 + _SAMPLER['calls']) & 0xFFFFFFFFFFFFFFFF
        out = None if lists else torch.empty_like(labels)
        sel = torch.empty(S, 2, max(int(max_num), 1), dtype=torch.int32, device=dev) if lists else None
        sel_cnt = torch.empty(S, 2, dtype=torch.int32, device=dev) if lists else None
        args = (S, ptr(labels), labels.stride(0), ptr(num_boxes), max_boxes, int(max_num), int(pos_num), seed,
                ptr(out), ptr(sel), ptr(sel_cnt), ptr(status_word(dev)), ptr(ws), ws.numel(), stream_of(labels))
        if _entry is None:
            call('frh_sample_random', *args)
        elif _entry[0](*args) != 0:  # tests: the tools library's two-launch sampler
            raise RuntimeError('{} failed'.format(_entry[1]))
        _debug_check(dev)
        return SampleLists(labels, sel, sel_cnt, max_num) if lists else out
    out = torch.empty_like(labels)
    ld = max(max_boxes, 1)
    pos_list = torch.empty(S, ld, dtype=torch.int32, device=dev)
    neg_list = torch.empty(S, ld, dtype=torch.int32, device=dev)
    counts = torch.empty(S, 2, dtype=torch.int32, device=dev)
    ws = workspace(_lib.query('frh_sample_workspace', S, ld), dev)
    call('frh_sample_candidates', S, ptr(labels), labels.stride(0), ptr(num_boxes), max_boxes, ptr(pos_list),
         ptr(neg_list), ld, ptr(counts), ptr(ws), ws.numel(), stream_of(labels))
    cnt = counts.cpu().numpy()  # host round trip, as the reference's .cpu().numpy() (region.py:48,55)
    check_device_status(dev)  # the stream is drained here anyway: a 4-byte read
    keep_ld = max(int(max_num), 1)
    keep = np.zeros((2, S, keep_ld), dtype=np.int32)
    kc = np.zeros((S, 2), dtype=np.int32)
    for s in range(S):
        npos, nneg = int(cnt[s, 0]), int(cnt[s, 1])
        kp = _numpy_keep(npos, pos_num)
        kneg = _numpy_keep(nneg, max_num - min(npos, pos_num))
        kc[s, 0], kc[s, 1] = len(kp), len(kneg)
        keep[0, s, :len(kp)] = kp
        keep[1, s, :len(kneg)] = kneg
    keep_t = torch.from_numpy(keep).to(dev, non_blocking=False)
    kc_t = torch.from_numpy(kc).to(dev)
    call('frh_sample_apply', S, ptr(labels), labels.stride(0), ptr(num_boxes), max_boxes, ptr(pos_list),
         ptr(neg_list), ld, ptr(keep_t[0]), ptr(keep_t[1]), keep_ld, ptr(kc_t), ptr(out), stream_of(labels))
    return out


def _numpy_keep(n, cap):
    """Positions kept by `np.random.choice(cands, n - cap, replace=False)` discarding.

    numpy's legacy choice(replace=False) is permutation(n)[:size]; the kept
    positions are the rest of that permutation, and the global RNG advances
    exactly as in the reference."""
    if n <= cap:
        return np.arange(n, dtype=np.int32)
    perm = np.random.permutation(n)
    return np.sort(perm[n - cap:]).astype(np.int32)


# ---------------------------------------------------------------- target gathers (a6/a12)
def anchor_target_batched(labels, num_boxes, max_boxes, anchors, gts, gt_labels, means, stds, max_out_per_seg,
                          sync=True):
    """labels: the sampled labels [S, n] (chosen = label >= 0) or a SampleLists.
    sync=False (SampleLists only): no read-back of the output size -- every output keeps
    its full capacity S * max_out_per_seg, the columns past the device total being padding
    (seg_of -1, label -1, zero boxes: the gathers and losses ignore them), and 'n_dev' is
    the total as a device int32 [1] (the heads' avg_factor)."""
    if not sync and not isinstance(labels, SampleLists):
        raise AssertionError('sync-free targets need the device sampler lists')
    sl = labels if isinstance(labels, SampleLists) else None
    if sl is not None:
        labels = sl.labels
    S = labels.shape[0]
    dev = labels.device
    cap = max(int(max_out_per_seg), 1)
    T = S * cap
    chosen_idx = torch.empty(T, dtype=torch.int64, device=dev)
    seg_of = torch.empty(T, dtype=torch.int32, device=dev)
    tar_labels = torch.empty(T, dtype=torch.int64, device=dev)
    tars = torch.empty(3, 4, T, dtype=torch.float32, device=dev)
    counts = torch.empty(S + 1, dtype=torch.int32, device=dev)
    ws = None if sl is not None else workspace(_lib.query('frh_anchor_target_workspace', S, max(max_boxes, 1)), dev)
    m = f32_array(means) if means is not None else None
    sd = f32_array(stds) if stds is not None else None
    if sl is not None and sl.max_num != cap:
        raise AssertionError('sampler lists of max_num {} for a cap of {}'.format(sl.max_num, cap))
    call('frh_anchor_target', S, ptr(labels), labels.stride(0), ptr(num_boxes), max_boxes, ptr(anchors),
         anchors.stride(0), 0, ptr(gts), gts.stride(1), gts.stride(0), ptr(gt_labels),
         gt_labels.stride(0) if gt_labels is not None else 0, m, sd, cap, ptr(sl.sel if sl else None),
         ptr(sl.sel_counts if sl else None), ptr(chosen_idx), ptr(seg_of), ptr(tar_labels), ptr(tars[0]),
         ptr(tars[1]), ptr(tars[2]), T, ptr(counts), ptr(ws), ws.numel() if ws is not None else 0,
         stream_of(labels))
    if not sync:
        return dict(chosen_idx=chosen_idx, seg_of=seg_of, tar_labels=tar_labels, tar_anchors=tars[0],
                    tar_bbox=tars[1], tar_param=tars[2], counts=None, counts_dev=counts[:S], n_dev=counts[S:])
    cnt = counts.cpu().tolist()  # output sizes are data dependent: one sync per batch
    n = cnt[S]
    return dict(chosen_idx=chosen_idx[:n], seg_of=seg_of[:n], tar_labels=tar_labels[:n],
                tar_anchors=tars[0][:, :n], tar_bbox=tars[1][:, :n], tar_param=tars[2][:, :n], counts=cnt[:S])


class _GatherLevels(torch.autograd.Function):
    """tar = cat_l(level_out.view(C, -1))[:, chosen] per image, with its adjoint scatter.
    Levels of any layout (NCHW, or the channels-last outputs of an NHWC head): the kernels
    take each level's element strides."""

    @staticmethod
    def forward(ctx, chosen_idx, seg_of, channels, *levels):
        n = chosen_idx.numel()
        offs, hw, st, A = _level_desc(levels, channels)
        out = torch.empty(channels, n, dtype=torch.float32, device=chosen_idx.device)
        if n:
            call('frh_gather_level_outputs_strided', len(levels), ptr_array(levels), i64_array(offs), i32_array(hw),
                 i64_array(st), A, channels, n, ptr(chosen_idx), ptr(seg_of), ptr(out), out.stride(0), stream_of(out))
        ctx.save_for_backward(chosen_idx, seg_of)
        ctx.shapes = [(l.shape, l.stride()) for l in levels]
        ctx.channels = channels
        return out

    @staticmethod
    def backward(ctx, grad):
        chosen_idx, seg_of = ctx.saved_tensors
        # each level's gradient in the level's own layout
        grads = [torch.empty_strided(sh, sd, dtype=torch.float32, device=grad.device).zero_() for sh, sd in ctx.shapes]
        grad = grad.contiguous()
        n = chosen_idx.numel()
        offs, hw, st, A = _level_desc(grads, ctx.channels)
        if n:
            call('frh_scatter_level_grads_strided', len(grads), ptr_array(grads), i64_array(offs), i32_array(hw),
                 i64_array(st), A, ctx.channels, n, ptr(chosen_idx), ptr(seg_of), ptr(grad), grad.stride(0),
                 stream_of(grad))
        return (None, None, None) + tuple(grads)


def _level_desc(levels, channels):
    """(first flat index per level, (H, W) per level, element strides per level, anchors A)."""
    offs, hw, st, acc = [], [], [], 0
    A = levels[0].shape[1] // channels
    for l in levels:
        if l.dim() != 4 or l.shape[1] != channels * A:
            raise AssertionError('head outputs must be [B, C*A, H, W] with one A for every level')
        offs.append(acc)
        hw += [l.shape[2], l.shape[3]]
        st += list(l.stride())
        acc += A * l.shape[2] * l.shape[3]
    return offs, hw, st, A


def gather_level_outputs(levels, chosen_idx, seg_of, channels):
    _need_cuda(chosen_idx)
    return _GatherLevels.apply(chosen_idx, seg_of, channels, *levels)


def prepend_gt_labels(prop_labels, num_props, num_gts, max_rows):
    S = prop_labels.shape[0]
    rows = torch.empty(S, max(max_rows, 1), dtype=torch.int64, device=prop_labels.device)
    num_rows = torch.empty(S, dtype=torch.int32, device=prop_labels.device)
    call('frh_prepend_gt_labels', S, ptr(prop_labels), prop_labels.stride(0), ptr(num_props), ptr(num_gts),
         max_rows, ptr(rows), rows.stride(0), ptr(num_rows), stream_of(prop_labels))
    return rows, num_rows


def bbox_target_batched(rows, num_rows, num_gts, max_rows, props, prop_seg_stride, gts, gt_labels, means, stds,
                        max_out_per_seg, sync=True):
    """rows: the sampled prepended rows [S, n] (chosen = label >= 0) or a SampleLists.
    sync=False: full-capacity outputs with padding columns and device counts, as
    anchor_target_batched."""
    if not sync and not isinstance(rows, SampleLists):
        raise AssertionError('sync-free targets need the device sampler lists')
    sl = rows if isinstance(rows, SampleLists) else None
    if sl is not None:
        rows = sl.labels
    S = rows.shape[0]
    dev = rows.device
    cap = max(int(max_out_per_seg), 1)
    T = S * cap
    tars = torch.empty(3, 4, T, dtype=torch.float32, device=dev)
    lab = torch.empty(2, T, dtype=torch.int64, device=dev)
    counts = torch.empty(S + 1, dtype=torch.int32, device=dev)
    ws = None if sl is not None else workspace(_lib.query('frh_bbox_target_workspace', S, max(max_rows, 1)), dev)
    m = f32_array(means) if means is not None else None
    sd = f32_array(stds) if stds is not None else None
    if sl is not None and sl.max_num != cap:
        raise AssertionError('sampler lists of max_num {} for a cap of {}'.format(sl.max_num, cap))
    call('frh_bbox_target', S, ptr(rows), rows.stride(0), ptr(num_rows), ptr(num_gts), max_rows, ptr(props),
         props.stride(-2), prop_seg_stride, ptr(gts), gts.stride(1), gts.stride(0), ptr(gt_labels),
         gt_labels.stride(0), m, sd, cap, ptr(sl.sel if sl else None), ptr(sl.sel_counts if sl else None),
         ptr(tars[0]), ptr(tars[1]), ptr(lab[0]), ptr(tars[2]), ptr(lab[1]), T, ptr(counts), ptr(ws),
         ws.numel() if ws is not None else 0, stream_of(rows))
    if not sync:
        return dict(tar_props=tars[0], tar_bbox=tars[1], tar_label=lab[0], tar_param=tars[2], tar_is_gt=lab[1],
                    counts=None, counts_dev=counts[:S], n_dev=counts[S:])
    cnt = counts.cpu().tolist()
    n = cnt[S]
    return dict(tar_props=tars[0][:, :n], tar_bbox=tars[1][:, :n], tar_label=lab[0][:n], tar_param=tars[2][:, :n],
                tar_is_gt=lab[1][:n], counts=cnt[:S])


# ---------------------------------------------------------------- encode / decode (a7/a8)
def bbox2param(base, bbox, means=None, stds=None):
    _need_cuda(base, bbox)
    base, bbox = _f32(base), _f32(bbox)
    if base.stride(1) != 1:
        base = base.contiguous()
    if bbox.stride(1) != 1:
        bbox = bbox.contiguous()
    n = base.shape[1]
    out = torch.empty(4, n, dtype=torch.float32, device=base.device)
    call('frh_bbox2param', ptr(base), base.stride(0), ptr(bbox), bbox.stride(0), n,
         f32_array(means) if means is not None else None, f32_array(stds) if stds is not None else None,
         ptr(out), out.stride(0), stream_of(base))
    return out


def param2bbox(base, param, means, stds, img_size=None):
    """base [4, n]; param [4*ncls, n] (coordinate-major classes); out like param."""
    _need_cuda(base, param)
    base, param = _f32(base), _f32(param)
    if base.stride(1) != 1:
        base = base.contiguous()
    if param.stride(1) != 1:
        param = param.contiguous()
    n = base.shape[1]
    ncls = param.shape[0] // 4
    out = torch.empty(param.shape[0], n, dtype=torch.float32, device=base.device)
    h, w = (float(img_size[0]), float(img_size[1])) if img_size is not None else (0.0, 0.0)
    call('frh_param2bbox', ptr(base), base.stride(0), ptr(param), param.stride(0), n, ncls, f32_array(means),
         f32_array(stds), int(img_size is not None), h, w, ptr(out), out.stride(0), stream_of(base))
    return out


# ---------------------------------------------------------------- RPN proposals (a9)
def rpn_proposals(cls_outs, reg_outs, anchors, num_anchors, cls_channels, means, stds, img_hw, min_sizes, pre_nms,
                  post_nms, max_num, nms_iou, _entry=None):
    """All images x levels; returns (boxes [B, 4, cap], scores [B, cap], counts int32 device [B]).
    cls / reg levels of any layout (NCHW or channels-last: the kernels take their strides).
    _entry: (ctypes function, name) taking frh_rpn_proposals_strided's arguments instead of it
    (tests: the tools library's four-launch selection)."""
    _need_cuda(*cls_outs)
    B, L = cls_outs[0].shape[0], len(cls_outs)
    grid = [v for c in cls_outs for v in (c.shape[2], c.shape[3])]
    grid_a = i32_array(grid)
    per_level = [num_anchors * c.shape[2] * c.shape[3] for c in cls_outs]
    P = max(min(pre_nms, n) if pre_nms > 0 else n for n in per_level)
    post = min(post_nms, P) if post_nms > 0 else P
    cap = max_num if max_num > 0 else post * L
    dev = cls_outs[0].device
    boxes = torch.empty(B, 4, cap, dtype=torch.float32, device=dev)
    scores = torch.empty(B, cap, dtype=torch.float32, device=dev)
    counts = torch.empty(B, dtype=torch.int32, device=dev)
    wsb = _lib.query('frh_rpn_proposals_workspace', B, L, grid_a, num_anchors, int(pre_nms))
    ws = workspace(wsb, dev)
    args = (B, L, ptr_array(cls_outs), ptr_array(reg_outs),
            i64_array([v for c in cls_outs for v in c.stride()]), i64_array([v for r in reg_outs for v in r.stride()]),
            grid_a, num_anchors, cls_channels, ptr(anchors), anchors.stride(0), f32_array(means), f32_array(stds),
            f32_array([v for hw in img_hw for v in hw]), f32_array(min_sizes), int(pre_nms), int(post_nms),
            int(max_num), float(nms_iou), ptr(boxes), ptr(scores), ptr(counts), ptr(status_word(dev)), ptr(ws),
            ws.numel(), stream_of(boxes))
    if _entry is None:
        call('frh_rpn_proposals_strided', *args)
    elif _entry[0](*args) != 0:
        raise RuntimeError('{} failed'.format(_entry[1]))
    _debug_check(dev)
    if NMS_PROFILE['on']:  # keep this call's per-level NMS input (in the workspace) for a replay
        view = (ctypes.c_int64 * 4)()
        call('frh_rpn_proposals_nms_view', B, L, grid_a, num_anchors, int(pre_nms), view)
        o_box, o_cnt, P_, S_ = list(view)
        rows = ws[o_box:o_box + S_ * P_ * 16].view(torch.float32).view(S_, P_, 4)
        cnt = ws[o_cnt:o_cnt + 4 * S_].view(torch.int32)
        NMS_PROFILE['records'].append((ws, rows, cnt, P_, float(nms_iou), int(post_nms) if post_nms > 0 else -1))
    return boxes, scores, counts


NMS_PROFILE = {'on': False, 'records': []}

def nms_bytes(counts, kept):
    """Algorithmic bytes of one segmented NMS call: per segment of N boxes
    20*N + 16*N*ceil(N/64) + 8*K_keep (boxes + scores read, 64-bit mask written and read once)."""
    n = counts.long()
    return int((20 * n + 16 * n * ((n + 63) // 64) + 8 * kept.long()).sum())


# ---------------------------------------------------------------- NMS (a10)
def nms_sorted(boxes_rows, counts, n_max, iou_thr, max_keep=-1):
    """boxes_rows [S, n_max, 4] pre-sorted; returns keep [S, n_max] int32 positions + counts [S]."""
    S = boxes_rows.shape[0]
    dev = boxes_rows.device
    keep = torch.empty(S, max(n_max, 1), dtype=torch.int32, device=dev)
    kc = torch.empty(S, dtype=torch.int32, device=dev)
    ws = workspace(_lib.query('frh_nms_workspace', S, max(n_max, 1)), dev)
    call('frh_nms_sorted', S, ptr(boxes_rows), boxes_rows.stride(0), ptr(counts), n_max, float(iou_thr),
         int(max_keep), ptr(keep), keep.stride(0), ptr(kc), ptr(ws), ws.numel(), stream_of(boxes_rows))
    return keep, kc


def nms(boxes, scores, iou_threshold):
    """Drop-in for torchvision.ops.nms(boxes[N,4], scores[N], thr) -> int64 keep (score order)."""
    _need_cuda(boxes, scores)
    n = boxes.shape[0]
    if n == 0:
        return torch.empty(0, dtype=torch.int64, device=boxes.device)
    order = torch.sort(scores, descending=True, stable=True)[1]
    rows = _f32(boxes).index_select(0, order).contiguous().view(1, n, 4)
    counts = torch.full((1,), n, dtype=torch.int32, device=boxes.device)
    keep, kc = nms_sorted(rows, counts, n, iou_threshold)
    k = int(kc.item())
    return order[keep[0, :k].long()]


# ---------------------------------------------------------------- class-wise batched multiclass NMS (a11)
def multiclass_nms_batched(boxes, scores, nms_channel, nms_iou, min_score=-1, max_num=None, score_factor=None,
                           mode='official', num_rows=None, row_valid=None):
    """utils.multiclass_nms (lib/utils.py:224-269) for B images in one frh_mcnms call.

    boxes [B, n, 4] or [B, n, 4 * C] (viewed (n, 4, C)), scores [B, n, C], score_factor
    [B, n] or [B, n, C] (official) or None, num_rows int32 [B] (device; None = n each),
    row_valid bool [B, n] (False = a row the reference drops before the call) or None.
    Returns per-image lists of (boxes [k, 4], scores [k], labels int64 [k]) in the
    reference's keep order.  Two host syncs per call (segment sizes, output counts)."""
    if mode not in ('official', 'strict'):
        raise AssertionError('unknown mode {}'.format(mode))
    _need_cuda(boxes, scores)
    B, n, C = scores.shape
    dev = scores.device
    boxes, scores = _f32(boxes).contiguous(), _f32(scores).contiguous()
    per_class = int(boxes.shape[2] != 4)
    if per_class and boxes.shape[2] != 4 * C:
        raise AssertionError('boxes must be [B, n, 4] or [B, n, 4 * classes]')
    empty = [(boxes.new_zeros(0, 4), scores.new_zeros(0), torch.zeros(0, dtype=torch.long, device=dev))
             for _ in range(B)]
    if n == 0 or max_num == 0:
        return empty
    if num_rows is None:
        num_rows = torch.full((B,), n, dtype=torch.int32, device=dev)
    chan = torch.zeros(C, dtype=torch.uint8)
    chan[[c for c in nms_channel if 0 <= c < C]] = 1
    chan = chan.to(dev)
    sf, sf_pc = None, 0
    if score_factor is not None:
        sf = _f32(score_factor).contiguous()
        sf_pc = int(sf.dim() == 3)
        if sf_pc and mode == 'strict':
            raise AssertionError('strict mode takes a per-row score factor')
    valid = row_valid.to(torch.uint8).contiguous() if row_valid is not None else None
    ws = workspace(_lib.query('frh_mcnms_workspace', B, C, n), dev)
    st = stream_of(scores)
    info_d = torch.empty(4, dtype=torch.int32, device=dev)
    m = 1 if mode == 'strict' else 0
    for by_class in (1, 0):  # a negative candidate coordinate: the reference's single pass, by image
        call('frh_mcnms_prepare', B, C, n, ptr(num_rows), ptr(boxes), boxes.stride(0), per_class, ptr(scores),
             scores.stride(0), ptr(sf), sf.stride(0) if sf is not None else 0, sf_pc, ptr(valid),
             valid.stride(0) if valid is not None else 0, ptr(chan), m, by_class, float(min_score), ptr(ws),
             ws.numel(), ptr(info_d), st)
        info = info_d.cpu().tolist()  # the call's one sync: segment sizes size the sort and the NMS mask
        if not info[1]:
            break
    P = int(info[0])
    tiles = (info[2] & 0xffffffff) | (info[3] << 32)
    if P == 0:
        return empty
    G = C if by_class else 1
    mx = int(max_num) if max_num is not None else -1
    cap = min(mx, G * P) if mx > 0 else G * P
    ob = torch.empty(B, cap, 4, dtype=torch.float32, device=dev)
    osc = torch.empty(B, cap, dtype=torch.float32, device=dev)
    ol = torch.empty(B, cap, dtype=torch.int64, device=dev)
    oc = torch.empty(B, dtype=torch.int32, device=dev)
    nws = workspace(_lib.query('frh_mcnms_nms_workspace', B, C, P, tiles), dev)
    call('frh_mcnms_finish', B, C, n, P, tiles, ptr(boxes), boxes.stride(0), per_class, ptr(scores),
         scores.stride(0), m, by_class, float(nms_iou), mx, ptr(ob), ptr(osc), ptr(ol), ptr(oc), cap, ptr(ws),
         ws.numel(), ptr(nws), nws.numel(), st)
    counts = oc.cpu().tolist()
    return [(ob[b, :k], osc[b, :k], ol[b, :k]) for b, k in enumerate(counts)]


# ---------------------------------------------------------------- RoI level map + RoIAlign (a13/a14)
def roi_rows(boxes, counts, finest_scale, num_levels, seg_stride=0, flat=True):
    """RoI rows [K, 5] (image, x1, y1, x2, y2) + levels ([K] int64, None for one level) of the
    images' boxes (frh_roi_rows): `boxes` [4, ld] with image b's boxes at columns
    offsets[b]... (flat) or [B, 4, cap] with image b's at boxes[b, :, :counts[b]]."""
    _need_cuda(boxes)
    K = int(sum(counts))
    dev = boxes.device
    rois = torch.empty(K, 5, dtype=torch.float32, device=dev)
    lv = torch.empty(K, dtype=torch.int64, device=dev) if num_levels > 1 else None
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + int(c))
    call('frh_roi_rows', len(counts), ptr(boxes), boxes.stride(-2), seg_stride, int(bool(flat)), i64_array(offs),
         float(finest_scale), int(num_levels), ptr(rois), ptr(lv), stream_of(boxes))
    return rois, lv


def roi_rows_dev(boxes, counts_dev, finest_scale, num_levels):
    """roi_rows for a fixed-capacity flat buffer [4, K] whose per-image counts stay on the
    device (frh_roi_rows_dev): all K rows, those past the total being padding rows."""
    _need_cuda(boxes, counts_dev)
    K = boxes.shape[1]
    dev = boxes.device
    rois = torch.empty(K, 5, dtype=torch.float32, device=dev)
    lv = torch.empty(K, dtype=torch.int64, device=dev) if num_levels > 1 else None
    call('frh_roi_rows_dev', counts_dev.numel(), ptr(boxes), boxes.stride(-2), K, ptr(counts_dev),
         float(finest_scale), int(num_levels), ptr(rois), ptr(lv), stream_of(boxes))
    return rois, lv


def roi_level_map(rois, finest_scale, num_levels):
    _need_cuda(rois)
    rois = _f32(rois).contiguous()
    lv = torch.empty(rois.shape[0], dtype=torch.int64, device=rois.device)
    call('frh_roi_level_map', ptr(rois), rois.shape[0], float(finest_scale), int(num_levels), ptr(lv),
         stream_of(rois))
    return lv


def _feat_desc(feats):
    hw = i32_array([v for f in feats for v in (f.shape[2], f.shape[3])])
    st = i64_array([v for f in feats for v in f.stride()])
    return hw, st


# Optional live timing of the RoIAlign forward launches (bench.py roofline):
# HIP events recorded on the launch stream around each call.  A record keeps the
# feature tensors only to replay the same launch shape for timing; with a graphed
# trunk they alias the graph's output buffers, so a replay reads the newest step's
# values -- never use a record's features for their contents.
ROI_ALIGN_PROFILE = {'on': False, 'records': [], 'events': True, 'timed': None, 'event_pool': [], 'launches': 0}
# 'launches': forward launches so far in this process (tools/roi_dispatch_table.py matches
# them to rocprofv3's dispatches by order).
# 'timed': a list -> each forward launch takes a (start, end, span) triple from 'event_pool'
# (created beforehand; span = device span shards, bench.span_slots), goes through
# frh_roi_align_fwd_strided_timed (the events are bound to the kernel's own dispatch
# timestamps, the span is the kernel's own first-wave-start / last-wave-end on the 100 MHz
# GPU clock: nothing is added to the stream) and appends the triple.


_DETERMINISTIC = {'on': os.environ.get('FRCNN_AMD_DETERMINISTIC', '') not in ('', '0')}


def set_deterministic_backward(on):
    """Force (True) / release (False) the RoIAlign backward's deterministic form."""
    _DETERMINISTIC['on'] = bool(on)


def deterministic_backward():
    """The RoIAlign backward runs its fixed-point form (bit-identical across runs) when
    torch.use_deterministic_algorithms(True) is in effect, FRCNN_AMD_DETERMINISTIC=1 is set, or
    set_deterministic_backward(True) was called; otherwise float atomics (faster)."""
    return _DETERMINISTIC['on'] or torch.are_deterministic_algorithms_enabled()


class _RoIAlignMulti(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rois, levels, scales, output_size, sampling_ratio, aligned, *feats):
        _need_cuda(rois, *feats)
        feats = [_f32(f) for f in feats]
        K = rois.shape[0]
        C = feats[0].shape[1]
        ph, pw = output_size
        out = torch.empty(K, C, ph, pw, dtype=torch.float32, device=rois.device)
        hw, st = _feat_desc(feats)
        ROI_ALIGN_PROFILE['launches'] += 1
        prof = ROI_ALIGN_PROFILE['on']
        e0 = e1 = None
        if prof and ROI_ALIGN_PROFILE['events']:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        timed = ROI_ALIGN_PROFILE['timed']
        if timed is not None and ROI_ALIGN_PROFILE['event_pool']:
            ev = ROI_ALIGN_PROFILE['event_pool'].pop()
            call('frh_roi_align_fwd_strided_timed', len(feats), ptr_array(feats), hw, st, f32_array(scales),
                 feats[0].shape[0], C, ptr(rois), ptr(levels), K, ph, pw, int(sampling_ratio), int(bool(aligned)),
                 ptr(out), ev[0].cuda_event, ev[1].cuda_event, ptr(ev[2]) if len(ev) > 2 else None, stream_of(out))
            timed.append(ev)
        else:
            call('frh_roi_align_fwd_strided', len(feats), ptr_array(feats), hw, st, f32_array(scales),
                 feats[0].shape[0], C, ptr(rois), ptr(levels), K, ph, pw, int(sampling_ratio), int(bool(aligned)),
                 ptr(out), stream_of(out))
        if prof:
            if e1 is not None:
                e1.record()
            ROI_ALIGN_PROFILE['records'].append((e0, e1, rois, levels, [tuple(f.shape) for f in feats], (ph, pw),
                                                 feats, tuple(scales), sampling_ratio))
        ctx.save_for_backward(rois, levels)
        ctx.cfg = (list(scales), output_size, sampling_ratio, aligned, [f.shape for f in feats])
        ctx.formats = [torch.channels_last if (f.stride(1) == 1 and f.shape[1] > 1) else torch.contiguous_format
                       for f in feats]
        return out

    @staticmethod
    def backward(ctx, grad):
        rois, levels = ctx.saved_tensors
        scales, (ph, pw), sr, aligned, shapes = ctx.cfg
        grad = grad.contiguous()
        K, B, C = rois.shape[0], shapes[0][0], shapes[0][1]
        # the gradient keeps each feature map's memory format (NCHW or channels_last)
        if deterministic_backward() and int(sr) == 2 and ph <= 8 and pw <= 8:
            # bit-identical across runs: fixed-point (int64, unit from max|grad|) integer atomics, then one
            # conversion pass that writes every gradient element (frh_roi_align_bwd_fixed)
            grads = [torch.empty(s, dtype=torch.float32, device=grad.device, memory_format=fmt)
                     for s, fmt in zip(shapes, ctx.formats)]
            accs = [torch.empty(s, dtype=torch.int64, device=grad.device, memory_format=fmt).zero_()
                    for s, fmt in zip(shapes, ctx.formats)]
            hw, st = _feat_desc(grads)
            word = torch.empty(1, dtype=torch.int32, device=grad.device)  # the call's max|grad_out| bits
            call('frh_roi_align_bwd_fixed', len(grads), ptr_array(grads), ptr_array(accs), hw, st, f32_array(scales),
                 B, C, ptr(rois), ptr(levels), K, ph, pw, int(sr), int(bool(aligned)), ptr(grad), ptr(word),
                 stream_of(grad))
            return (None, None, None, None, None, None) + tuple(grads)
        if deterministic_backward():
            # the fixed-point form covers sampling 2 with up to 8 x 8 bins (every config); the
            # float-atomic form below is not deterministic, which torch's mode must hear about
            msg = ('frcnn_amd roi_align backward: no deterministic form for sampling_ratio={}, '
                   'output {}x{} (fixed point covers sampling 2 and up to 8x8 bins)'.format(sr, ph, pw))
            if torch.are_deterministic_algorithms_enabled() and torch.is_deterministic_algorithms_warn_only_enabled() \
                    and not _DETERMINISTIC['on']:
                if not _DETERMINISTIC.get('warned'):
                    _DETERMINISTIC['warned'] = True
                    warnings.warn(msg)
            else:
                raise RuntimeError(msg)
        # cleared here and accumulated with float atomics (one per row run of a RoI's taps)
        grads = [torch.empty(s, dtype=torch.float32, device=grad.device, memory_format=fmt).zero_()
                 for s, fmt in zip(shapes, ctx.formats)]
        hw, st = _feat_desc(grads)
        call('frh_roi_align_bwd_strided', len(grads), ptr_array(grads), hw, st, f32_array(scales), B, C,
             ptr(rois), ptr(levels), K, ph, pw, int(sr), int(bool(aligned)), ptr(grad), stream_of(grad))
        return (None, None, None, None, None, None) + tuple(grads)


def roi_align_replay(rec, out=None, events=None):
    """Re-issue a recorded RoIAlign forward launch (same features, RoIs and levels) on the
    current stream; bench.py times back-to-back replays for the per-launch kernel duration.
    events: a (start, end) pair bound to the dispatch (frh_roi_align_fwd_strided_timed)."""
    _, _, rois, levels, shapes, (ph, pw), feats, scales, sr = rec
    K, C = rois.shape[0], shapes[0][1]
    if out is None:
        out = torch.empty(K, C, ph, pw, dtype=torch.float32, device=rois.device)
    hw, st = _feat_desc(feats)
    if events is not None:
        call('frh_roi_align_fwd_strided_timed', len(feats), ptr_array(feats), hw, st, f32_array(scales),
             shapes[0][0], C, ptr(rois), ptr(levels), K, ph, pw, int(sr), 0, ptr(out), events[0].cuda_event,
             events[1].cuda_event, ptr(events[2]) if len(events) > 2 else None, stream_of(out))
    else:
        call('frh_roi_align_fwd_strided', len(feats), ptr_array(feats), hw, st, f32_array(scales), shapes[0][0], C,
             ptr(rois), ptr(levels), K, ph, pw, int(sr), 0, ptr(out), stream_of(out))
    return out


def roi_align_multilevel(feats, rois, levels, scales, output_size, sampling_ratio, aligned=False):
    rois = _f32(rois).contiguous()
    return _RoIAlignMulti.apply(rois, levels, tuple(scales), tuple(output_size), sampling_ratio, aligned, *feats)


def _pair(v):
    return (int(v), int(v)) if isinstance(v, int) else tuple(int(x) for x in v)


def roi_align(input, boxes, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=False):
    """Drop-in for torchvision.ops.roi_align with [K, 5] rois."""
    if isinstance(boxes, (list, tuple)):
        raise NotImplementedError('roi_align takes [K, 5] rois')
    return roi_align_multilevel([input], boxes, None, [spatial_scale], _pair(output_size), sampling_ratio, aligned)


class RoIAlign(nn.Module):
    """Drop-in for torchvision.ops.RoIAlign (reference registry lib/builder.py:9,22)."""

    def __init__(self, output_size, spatial_scale, sampling_ratio, aligned=False):
        super().__init__()
        self.output_size = _pair(output_size)
        self.spatial_scale = spatial_scale
        self.sampling_ratio = sampling_ratio
        self.aligned = aligned

    def forward(self, input, rois):
        return roi_align(input, rois, self.output_size, self.spatial_scale, self.sampling_ratio, self.aligned)

    def __repr__(self):
        return '{}(output_size={}, spatial_scale={}, sampling_ratio={}, aligned={})'.format(
            type(self).__name__, self.output_size, self.spatial_scale, self.sampling_ratio, self.aligned)


class _RoIPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, rois, output_size, spatial_scale):
        _need_cuda(feat, rois)
        feat = _f32(feat)
        rois = _f32(rois).contiguous()
        K, C = rois.shape[0], feat.shape[1]
        ph, pw = output_size
        out = torch.empty(K, C, ph, pw, dtype=torch.float32, device=feat.device)
        argmax = torch.empty(K, C, ph, pw, dtype=torch.int32, device=feat.device)
        call('frh_roi_pool_fwd', ptr(feat), i64_array(feat.stride()), feat.shape[2], feat.shape[3], C,
             float(spatial_scale), ptr(rois), K, ph, pw, ptr(out), ptr(argmax), stream_of(out))
        ctx.save_for_backward(rois, argmax)
        ctx.shape = feat.shape
        return out

    @staticmethod
    def backward(ctx, grad):
        rois, argmax = ctx.saved_tensors
        g = torch.zeros(ctx.shape, dtype=torch.float32, device=grad.device)
        grad = grad.contiguous()
        call('frh_roi_pool_bwd', ptr(g), i64_array(g.stride()), g.shape[2], g.shape[3], g.shape[1], ptr(rois),
             rois.shape[0], grad.shape[2], grad.shape[3], ptr(grad), ptr(argmax), stream_of(grad))
        return g, None, None, None


def roi_pool(input, boxes, output_size, spatial_scale=1.0):
    """Drop-in for torchvision.ops.roi_pool with [K, 5] rois."""
    return _RoIPoolFn.apply(input, boxes, _pair(output_size), spatial_scale)


class RoIPool(nn.Module):
    """Drop-in for torchvision.ops.RoIPool.  Accepts and ignores `sampling_ratio`, which the
    reference's C4 config passes (configs/faster_rcnn_r50.py:26) and torchvision rejects
    (documented deviation Q9)."""

    def __init__(self, output_size, spatial_scale, sampling_ratio=None):
        super().__init__()
        self.output_size = _pair(output_size)
        self.spatial_scale = spatial_scale

    def forward(self, input, rois):
        return roi_pool(input, rois, self.output_size, self.spatial_scale)


# ---------------------------------------------------------------- ATSS / LTRB targets (a16)
def atss_assign(anchors, grid_sizes, strides, gt_list, label_list, img_shapes, topk=9):
    """Batched FCOSHead.single_image_targets_atss (fcos_head.py:283-368).
    anchors: [4, N] f32 (one per cell, levels concatenated); gt_list: per image [4, G_i];
    label_list: per image [G_i]; img_shapes: per image (h, w).
    Returns cls i64 [B, N], reg f32 [B, N, 4] (ltrb), ctr f32 [B, N]."""
    _need_cuda(anchors)
    dev = anchors.device
    B = len(gt_list)
    L = len(grid_sizes)
    N = sum(int(h) * int(w) for h, w in grid_sizes)
    if anchors.shape[1] != N or anchors.stride(1) != 1:
        raise AssertionError('anchors must be a [4, N] row-contiguous tensor with one anchor per cell')
    gts, gcnt, gmax = pack_boxes([g.float() for g in gt_list], dev)
    labels = pack_labels(label_list, gmax, dev)
    img_hw = device_ints([int(v) for s in img_shapes for v in s[:2]], dev)
    cls = torch.empty(B, N, dtype=torch.int64, device=dev)
    reg = torch.empty(B, N, 4, dtype=torch.float32, device=dev)
    ctr = torch.empty(B, N, dtype=torch.float32, device=dev)
    ws_n = _lib.query('frh_atss_workspace', B, gmax, L, int(topk), N)
    ws = workspace(ws_n, dev)
    hw = i32_array([int(v) for g in grid_sizes for v in g])
    call('frh_atss_assign', B, L, hw, f32_array(strides), ptr(anchors), anchors.stride(0), ptr(gts), gts.stride(0),
         ptr(gcnt), ptr(labels), gmax, ptr(img_hw), int(topk), ptr(cls), ptr(reg), ptr(ctr), ptr(ws), ws_n,
         stream_of(cls))
    return cls, reg, ctr


# ---------------------------------------------------------------- FPN top-down merge (channels-last levels)
class _FpnMerge(torch.autograd.Function):
    """out = (lat + bias) + nearest_upsample(up) as a channels-last tensor (frh_fpn_merge_nhwc);
    lat: any layout; bias: [C] or None; up: the merged coarser level (channels-last) or None."""

    @staticmethod
    def forward(ctx, lat, up, bias):
        B, C, H, W = lat.shape
        out = torch.empty(B, C, H, W, dtype=torch.float32, device=lat.device, memory_format=torch.channels_last)
        uh, uw = (int(up.shape[2]), int(up.shape[3])) if up is not None else (0, 0)
        call('frh_fpn_merge_nhwc', ptr(lat), i64_array(lat.stride()), ptr(bias), ptr(up), uh, uw, ptr(out), B, C, H,
             W, stream_of(out))
        ctx.has_up = up is not None
        if ctx.has_up:
            ctx.save_for_backward(up)
        return out

    @staticmethod
    def backward(ctx, g):
        gup = None
        if ctx.has_up and ctx.needs_input_grad[1]:
            (up,) = ctx.saved_tensors
            with torch.enable_grad():
                u = up.detach().requires_grad_(True)
                y = torch.nn.functional.interpolate(u, size=g.shape[2:], mode='nearest')
                gup, = torch.autograd.grad(y, u, g)
        gb = g.sum((0, 2, 3)) if ctx.needs_input_grad[2] else None
        return g if ctx.needs_input_grad[0] else None, gup, gb


def fpn_merge_nhwc(lat, up=None, bias=None):
    """The FPN's top-down step lat + interpolate(up, size=lat.shape[2:], mode='nearest')
    (lib/necks.py:72-84) as one HIP pass writing a channels-last level; bias: the lateral
    conv's bias when lat was computed without it (its add folded into the pass)."""
    _need_cuda(lat, up, bias)
    if lat.dtype != torch.float32 or (up is not None and (up.dtype != torch.float32 or
                                                          not up.is_contiguous(memory_format=torch.channels_last))):
        raise AssertionError('fpn_merge_nhwc: f32 lateral and a channels-last f32 coarser level')
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() != lat.shape[1] or not bias.is_contiguous()):
        raise AssertionError('fpn_merge_nhwc: bias must be a contiguous f32 [C]')
    return _FpnMerge.apply(lat, up, bias)


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias, relu):
        B, C, H, W = y.shape
        call('frh_bias_act_nhwc', ptr(y), ptr(bias), B * H * W, C, int(bool(relu)), stream_of(y))
        ctx.relu = relu
        ctx.mark_dirty(y)
        ctx.save_for_backward(y if relu else None)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        if ctx.relu:
            g = g * (y > 0)
        return g, (g.sum((0, 2, 3)) if ctx.needs_input_grad[1] else None), None


def conv_bias_relu(conv, x, relu=True):
    """act(conv(x)) for a biased Conv2d: on a HIP device with channels-last f32 input and weights
    the conv runs without its bias (MIOpen NHWC) and frh_bias_act_nhwc adds the bias and applies
    the ReLU in one pass (bit-identical to conv + bias, then relu); otherwise the module ops."""
    ok = (x.is_cuda and x.dtype == torch.float32 and conv.bias is not None and conv.weight.dtype == torch.float32
          and conv.out_channels % 4 == 0 and x.is_contiguous(memory_format=torch.channels_last)
          and conv.weight.is_contiguous(memory_format=torch.channels_last))
    if not ok:
        y = conv(x)
        return torch.relu(y) if relu else y
    y = torch.nn.functional.conv2d(x, conv.weight, None, conv.stride, conv.padding, conv.dilation, conv.groups)
    if not y.is_contiguous(memory_format=torch.channels_last):
        y = y.contiguous(memory_format=torch.channels_last)
    return _BiasAct.apply(y, conv.bias, relu)


# ---------------------------------------------------------------- backbone epilogue (frozen BN + add + ReLU)
class _FrozenBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, skip, weight, bias, mean, var, eps, relu):
        n, c, h, w = x.shape
        x = x.contiguous()
        skip = skip.contiguous() if skip is not None else None
        y = torch.empty_like(x)
        call('frh_bn_act', ptr(x), ptr(skip), ptr(y), ptr(weight), ptr(bias), ptr(mean), ptr(var), float(eps), n, c,
             h * w, int(bool(relu)), stream_of(x))
        need_x = weight is not None and weight.requires_grad
        ctx.save_for_backward(x if need_x else None, y if relu else None, weight, mean, var)
        ctx.cfg = (eps, relu, skip is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, weight, mean, var = ctx.saved_tensors
        eps, relu, has_skip = ctx.cfg
        g = gy * (y > 0) if relu else gy
        inv = torch.rsqrt(var + eps)
        s = inv * weight if weight is not None else inv
        gx = g * s.view(1, -1, 1, 1) if ctx.needs_input_grad[0] else None
        gskip = g if has_skip and ctx.needs_input_grad[1] else None
        gw = gb = None
        if ctx.needs_input_grad[2]:
            gw = (g * (x - mean.view(1, -1, 1, 1))).sum((0, 2, 3)) * inv
        if ctx.needs_input_grad[3]:
            gb = g.sum((0, 2, 3))
        return gx, gskip, gw, gb, None, None, None, None


def bn_act(x, bn, skip=None, relu=True):
    """act(bn(x) (+ skip)) for an eval-mode BatchNorm2d in one HIP pass (frh_bn_act).
    A BN in training mode (the reference never trains BN statistics) or CPU tensors take
    the plain module ops."""
    if bn.training or not x.is_cuda or x.dtype != torch.float32 or (x.shape[2] * x.shape[3]) % 4:
        y = bn(x)
        if skip is not None:
            y = y + skip
        return torch.relu_(y) if relu else y
    return _FrozenBNAct.apply(x, skip, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps, relu)


def bn_act_maxpool(x, bn, pool):
    """pool(relu(bn(x))) for the ResNet stem (eval-mode BN, MaxPool2d(3, 2, 1)) in one HIP pass
    (frh_bn_act_maxpool) when nothing needs a gradient through it (the reference freezes the
    stem: frozen_stages >= 0); otherwise bn_act then the pool module."""
    fused = (x.is_cuda and x.dtype == torch.float32 and not bn.training and x.is_contiguous()
             and x.shape[3] % 8 == 0 and x.shape[3] >= 8
             and (pool.kernel_size, pool.stride, pool.padding, pool.dilation) in ((3, 2, 1, 1), ((3, 3), (2, 2), (1, 1), (1, 1)))
             and not pool.ceil_mode and not pool.return_indices
             and not (torch.is_grad_enabled() and (x.requires_grad or (bn.weight is not None and bn.weight.requires_grad)
                                                   or (bn.bias is not None and bn.bias.requires_grad))))
    if not fused:
        return pool(bn_act(x, bn))
    n, c, h, w = x.shape
    y = torch.empty(n, c, (h - 1) // 2 + 1, w // 2, dtype=torch.float32, device=x.device)
    call('frh_bn_act_maxpool', ptr(x), ptr(y), ptr(bn.weight), ptr(bn.bias), ptr(bn.running_mean),
         ptr(bn.running_var), float(bn.eps), n, c, h, w, stream_of(x))
    return y


# ---------------------------------------------------------------- f1: fused losses
CLS_FOCAL, CLS_SIGMOID_BCE, CLS_SOFTMAX_CE = 0, 1, 2
_LOSS_WS = {}


def _loss_workspace(x):
    """Zero-filled once per (device, stream): each forward call leaves its arrival counter zero."""
    key = (x.device, torch.cuda.current_stream(x.device).cuda_stream)
    ws = _LOSS_WS.get(key)
    if ws is None:
        ws = _LOSS_WS[key] = torch.zeros(int(_lib.query('frh_loss_workspace')), dtype=torch.uint8, device=x.device)
    return ws


class _ClsLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target, kind, alpha, gamma):
        n, c = x.shape
        tfloat = int(target.dtype == torch.float32)
        out = torch.empty((), dtype=torch.float32, device=x.device)
        ws = _loss_workspace(x)
        call('frh_cls_loss_fwd', kind, ptr(x), n, c, x.stride(0), x.stride(1), ptr(target), tfloat, float(alpha),
             float(gamma), ptr(status_word(x.device)), ptr(out), ptr(ws), ws.numel(), stream_of(x))
        ctx.save_for_backward(x, target)
        ctx.cfg = (kind, tfloat, alpha, gamma)
        return out

    @staticmethod
    def backward(ctx, g):
        x, target = ctx.saved_tensors
        kind, tfloat, alpha, gamma = ctx.cfg
        n, c = x.shape
        gx = torch.empty_like(x)
        g = _f32(g).contiguous()
        call('frh_cls_loss_bwd', kind, ptr(x), n, c, x.stride(0), x.stride(1), ptr(target), tfloat, float(alpha),
             float(gamma), ptr(g), ptr(gx), gx.stride(0), gx.stride(1), stream_of(x))
        return gx, None, None, None, None


def cls_loss(x, target, kind, alpha=0.25, gamma=2.0):
    """Summed classification loss of logits x [n, C] (any strides) against target [n]
    (frh_cls_loss_fwd/bwd; kinds CLS_FOCAL / CLS_SIGMOID_BCE / CLS_SOFTMAX_CE)."""
    _need_cuda(x, target)
    if x.dim() != 2 or target.dim() != 1 or target.shape[0] != x.shape[0]:
        raise AssertionError('cls_loss: x [n, C] and target [n] expected')
    if target.is_floating_point():
        target = target.float()
        if x.shape[1] != 1 or kind != CLS_SIGMOID_BCE:
            raise AssertionError('cls_loss: float targets only for single-channel sigmoid BCE')
    elif target.dtype != torch.int64:
        target = target.long()
    return _ClsLoss.apply(_f32(x), target.contiguous(), int(kind), alpha, gamma)


class _SmoothL1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, label, xs, ys, n, m, n_sel, beta):
        out = torch.empty((), dtype=torch.float32, device=x.device)
        ws = _loss_workspace(x)
        call('frh_smooth_l1_fwd', ptr(x), xs[0], xs[1], xs[2], ptr(y), ys[0], ys[1], ptr(label), n, m, n_sel,
             float(beta), ptr(status_word(x.device)), ptr(out), ptr(ws), ws.numel(), stream_of(x))
        ctx.save_for_backward(x, y, label)
        ctx.cfg = (xs, ys, n, m, n_sel, beta)
        return out

    @staticmethod
    def backward(ctx, g):
        x, y, label = ctx.saved_tensors
        xs, ys, n, m, n_sel, beta = ctx.cfg
        gx = torch.zeros_like(x)
        if gx.stride() != x.stride():
            raise AssertionError('smooth_l1: gradient layout differs from the input')
        g = _f32(g).contiguous()
        call('frh_smooth_l1_bwd', ptr(x), xs[0], xs[1], xs[2], ptr(y), ys[0], ys[1], ptr(label), n, m, n_sel,
             float(beta), ptr(g), ptr(gx), xs[0], xs[1], xs[2], stream_of(x))
        return gx, None, None, None, None, None, None, None, None


def _l1_args(x, y, label, rows_dim):
    """(x, y, label, x strides, y strides, n, m, n_sel) of a masked smooth-L1 sum."""
    _need_cuda(x, y, label)
    if x.shape != y.shape or x.dim() != 2:
        raise AssertionError('smooth_l1_loss: x and y must be equal 2-D shapes')
    x, y = _f32(x), _f32(y)
    if not (x.is_contiguous() or x.t().is_contiguous()):
        x = x.contiguous()  # the zero-filled gradient must share x's strides
    cd = 1 - rows_dim
    n, m = x.shape[rows_dim], x.shape[cd]
    if label is not None and label.numel() != n:
        raise AssertionError('smooth_l1_loss: one label per row expected')
    lab = label.contiguous().long() if label is not None else None
    return x, y, lab, (x.stride(rows_dim), x.stride(cd), 0), (y.stride(rows_dim), y.stride(cd)), n, m, 1


def smooth_l1_loss(x, y, beta, label=None, rows_dim=0):
    """Summed smooth_l1_loss_v2 of x and y (same shape, 2-D, rows along `rows_dim`),
    counting only rows whose label is > 0 when `label` is given (frh_smooth_l1_fwd/bwd)."""
    return _SmoothL1.apply(*_l1_args(x, y, label, rows_dim), beta)


def _l1_class_select_args(reg_out, num_classes, target, label):
    _need_cuda(reg_out, target, label)
    n = reg_out.shape[0]
    if reg_out.dim() != 2 or reg_out.shape[1] != 4 * num_classes or target.shape != (n, 4) or label.numel() != n:
        raise AssertionError('smooth_l1_class_select: shape mismatch')
    reg_out, target = _f32(reg_out), _f32(target)
    if reg_out.stride(1) != 1:
        reg_out = reg_out.contiguous()
    xs = (reg_out.stride(0), num_classes, 1)
    return reg_out, target, label.contiguous().long(), xs, (target.stride(0), target.stride(1)), n, 4, num_classes


def smooth_l1_class_select(reg_out, num_classes, target, label, beta):
    """BBoxHead's regression loss: reg_out [n, 4*C] viewed [n, 4, C], the labelled class's
    deltas of the positive rows against target [n, 4] (any strides), summed."""
    return _SmoothL1.apply(*_l1_class_select_args(reg_out, num_classes, target, label), beta)


class _DetLoss(torch.autograd.Function):
    """A head's classification and regression losses in one launch (frh_det_loss_fwd),
    each scaled as the heads scale it: (sum * weight) / avg_factor."""

    @staticmethod
    def forward(ctx, x, target, kind, alpha, gamma, wc, rx, ry, rlabel, xs, ys, rn, rm, n_sel, beta, wr, div):
        n, c = x.shape
        tfloat = int(target.dtype == torch.float32)
        out = torch.empty(2, dtype=torch.float32, device=x.device)
        ws = _loss_workspace(x)
        dcount = div if isinstance(div, torch.Tensor) else None  # device int32 count (sync-free targets)
        hdiv = 1.0 if dcount is not None else float(div)
        call('frh_det_loss_fwd', kind, ptr(x), n, c, x.stride(0), x.stride(1), ptr(target), tfloat, float(alpha),
             float(gamma), float(wc), hdiv, ptr(rx), xs[0], xs[1], xs[2], ptr(ry), ys[0], ys[1], ptr(rlabel), rn,
             rm, n_sel, float(beta), float(wr), hdiv, ptr(dcount), ptr(status_word(x.device)), ptr(out), ptr(ws),
             ws.numel(), stream_of(x))
        if dcount is not None:
            # backward divides by the count as f32 (count 0: every row is padding, gradients 0)
            div = dcount.float()
        ctx.save_for_backward(x, target, rx, ry, rlabel)
        ctx.cfg = (kind, tfloat, alpha, gamma, wc, xs, ys, rn, rm, n_sel, beta, wr, div)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, gc, gr):
        x, target, rx, ry, rlabel = ctx.saved_tensors
        kind, tfloat, alpha, gamma, wc, xs, ys, rn, rm, n_sel, beta, wr, div = ctx.cfg
        gx = grx = None
        if gc is not None and ctx.needs_input_grad[0]:
            g = _f32((gc / div) * wc).contiguous()  # the reference's Div then Mul backward
            n, c = x.shape
            gx = torch.empty_like(x)
            call('frh_cls_loss_bwd', kind, ptr(x), n, c, x.stride(0), x.stride(1), ptr(target), tfloat, float(alpha),
                 float(gamma), ptr(g), ptr(gx), gx.stride(0), gx.stride(1), stream_of(x))
        if gr is not None and ctx.needs_input_grad[6]:
            g = _f32((gr / div) * wr).contiguous()
            grx = torch.zeros_like(rx)
            if grx.stride() != rx.stride():
                raise AssertionError('det loss: gradient layout differs from the input')
            call('frh_smooth_l1_bwd', ptr(rx), xs[0], xs[1], xs[2], ptr(ry), ys[0], ys[1], ptr(rlabel), rn, rm, n_sel,
                 float(beta), ptr(g), ptr(grx), xs[0], xs[1], xs[2], stream_of(rx))
        return gx, None, None, None, None, None, grx, None, None, None, None, None, None, None, None, None, None


def det_losses(x, target, kind, alpha, gamma, cls_weight, l1_args, beta, reg_weight, avg_factor):
    """(cls, reg) = (cls_loss(x, target, kind) * cls_weight / avg_factor,
    smooth-L1(*l1_args) * reg_weight / avg_factor) in one launch; l1_args from _l1_args /
    _l1_class_select_args.  avg_factor is a host number (the sampled count) or a device
    int32 [1] count (sync-free targets: rows labelled < 0 are padding and ignored, a count
    of 0 gives zero losses)."""
    _need_cuda(x, target)
    if target.dtype != torch.int64:
        target = target.long()
    rx, ry, rlabel, xs, ys, rn, rm, n_sel = l1_args
    if isinstance(avg_factor, torch.Tensor):
        if avg_factor.dtype != torch.int32 or avg_factor.numel() != 1 or not avg_factor.is_cuda:
            raise AssertionError('a device avg_factor is an int32 [1] count')
    else:
        avg_factor = float(avg_factor)
    return _DetLoss.apply(_f32(x), target.contiguous(), int(kind), alpha, gamma, cls_weight, rx, ry, rlabel, xs, ys,
                          rn, rm, n_sel, beta, reg_weight, avg_factor)

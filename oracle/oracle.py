"""TEST INFRASTRUCTURE — CPU oracle of the frcnn_amd hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the timed CPU baseline.  The
product package (pytorch-faster-rcnn_amd/frcnn_amd) never imports it.

Per-op arithmetic lives in csrc/oracle.c (scalar C in the reference's
operation order); this file restates the reference's per-image glue on
numpy arrays, citing the reference file:line each function follows.

Pinning: anchors, masks, IoU, MaxIoU assignment,
sampling (numpy global RNG), anchor_target, bbox_target, encode/decode,
proposal selection/ordering and level mapping are checked against golden
vectors produced by the reference itself (tests/golden/gen_golden.py).
torchvision nms / roi_align / roi_pool are absent from the reference and
from this image: those rows are "parity unpinned" (restated semantics).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'liboracle.so')

_c = None
_F = ctypes.POINTER(ctypes.c_float)
_I64 = ctypes.POINTER(ctypes.c_int64)
_I32 = ctypes.POINTER(ctypes.c_int32)


def build():
    src = os.path.join(HERE, 'csrc', 'oracle.c')
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(['make', '-s', '-C', HERE])
    return LIB


def lib():
    global _c
    if _c is None:
        build()
        _c = ctypes.CDLL(LIB)
        _c.orc_nms_sorted.restype = ctypes.c_int64
        _c.orc_maxiou_assign.restype = ctypes.c_int
        _c.orc_set_threads.restype = ctypes.c_int
    return _c


def set_threads(n):
    """Thread count of the C restatement's parallel loops (OpenMP); returns the previous one.
    Results do not depend on it (every output element is one thread's, in reference order)."""
    return int(lib().orc_set_threads(int(n)))


def _f(a):
    return a.ctypes.data_as(_F)


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


# ------------------------------------------------------------------ per-op
def calc_iou(a, b):
    """lib/utils.py:151-172."""
    a, b = _c32(a), _c32(b)
    n, k = a.shape[1], b.shape[1]
    out = np.empty((n, k), np.float32)
    lib().orc_iou_table(_f(a), ctypes.c_int64(n), ctypes.c_int64(n), _f(b), ctypes.c_int64(k), ctypes.c_int64(k),
                        _f(out))
    return out


def elem_iou(a, b):
    """lib/utils.py:174-182 (numpy, f32 op order)."""
    a, b = a.astype(np.float32), b.astype(np.float32)
    tl = np.maximum(a[:2], b[:2])
    br = np.minimum(a[2:], b[2:])
    ai = (br[0] - tl[0]) * (br[1] - tl[1])
    ai = ai * np.all(tl < br, axis=0).astype(np.float32)
    aa = (a[2] - a[0]) * (a[3] - a[1])
    ab = (b[2] - b[0]) * (b[3] - b[1])
    return (ai / ((aa + ab) - ai)).astype(np.float32)


def maxiou_assign(boxes, gts, pos_iou, neg_iou, min_pos_iou):
    """MaxIoUAssigner.__call__ (lib/region.py:75-107) -> (labels int64, max_iou f32)."""
    boxes, gts = _c32(boxes), _c32(gts)
    n, g = boxes.shape[1], gts.shape[1]
    labels = np.empty(n, np.int64)
    miou = np.empty(n, np.float32)
    r = lib().orc_maxiou_assign(_f(boxes), ctypes.c_int64(n), ctypes.c_int64(n), _f(gts), ctypes.c_int64(g),
                                ctypes.c_int64(g), ctypes.c_float(pos_iou), ctypes.c_float(neg_iou),
                                ctypes.c_float(min_pos_iou), labels.ctypes.data_as(_I64), _f(miou))
    if r != 0:
        raise RuntimeError('maxiou_assign: no gts')
    return labels, miou


def anchor_sizes(base, scales, ratios):
    """lib/anchor.py:91-97 (float64 then f32)."""
    ws = [base * s * np.sqrt(ar) for s in scales for ar in ratios]
    hs = [base * s / np.sqrt(ar) for s in scales for ar in ratios]
    return np.asarray(ws, np.float64).astype(np.float32), np.asarray(hs, np.float64).astype(np.float32)


def anchor_grid(base, scales, ratios, stride, grid, center_lt=False):
    """AnchorCreator(base, scales, ratios)(stride, grid) -> [4, A, H, W] (lib/anchor.py:107-129)."""
    ws, hs = anchor_sizes(base, scales, ratios)
    gh, gw = grid
    A = len(ws)
    out = np.empty((4, A * gh * gw), np.float32)
    lib().orc_anchor_grid(_f(ws), _f(hs), A, gh, gw, ctypes.c_float(stride), int(center_lt), _f(out),
                          ctypes.c_int64(A * gh * gw))
    return out.reshape(4, A, gh, gw)


def inside_grid_mask(num_anchors, img_size, grid_size, stride):
    """lib/region.py:10-16."""
    in_h = min(grid_size[0], int(img_size[0] * (1.0 / stride)) + 1)
    in_w = min(grid_size[1], int(img_size[1] * (1.0 / stride)) + 1)
    f = np.zeros((num_anchors, grid_size[0], grid_size[1]), np.float32)
    f[:, :in_h, :in_w] = 1
    return f.reshape(-1)


def inside_anchor_mask(anchors, img_size, allowed_border=0):
    """lib/region.py:19-29 (f32 compares)."""
    H, W = img_size
    if allowed_border < 0:
        return np.ones(anchors.shape[1], bool)
    b = np.float32(-allowed_border)
    return ((anchors[0] >= b) & (anchors[1] >= b) & (anchors[2] < np.float32(W + allowed_border)) &
            (anchors[3] < np.float32(H + allowed_border)))


def bbox2param(base, bbox, means=None, stds=None):
    base, bbox = _c32(base), _c32(bbox)
    n = base.shape[1]
    out = np.empty((4, n), np.float32)
    m = _c32(means) if means is not None else None
    s = _c32(stds) if stds is not None else None
    lib().orc_bbox2param(_f(base), ctypes.c_int64(n), _f(bbox), ctypes.c_int64(n), ctypes.c_int64(n),
                         _f(m) if m is not None else None, _f(s) if s is not None else None, _f(out),
                         ctypes.c_int64(n))
    return out


def param2bbox(base, param, means=(0, 0, 0, 0), stds=(1, 1, 1, 1), img_size=None):
    """lib/utils.py:83-106 (+clamp_bbox), param [4*ncls, n]."""
    base, param = _c32(base), _c32(param)
    n = base.shape[1]
    ncls = param.shape[0] // 4
    out = np.empty_like(param)
    h, w = (float(img_size[0]), float(img_size[1])) if img_size is not None else (0.0, 0.0)
    lib().orc_param2bbox(_f(base), ctypes.c_int64(n), _f(param), ctypes.c_int64(n), ctypes.c_int64(n), ncls,
                         _f(_c32(means)), _f(_c32(stds)), int(img_size is not None), ctypes.c_float(h),
                         ctypes.c_float(w), _f(out), ctypes.c_int64(n))
    return out


def roi_level_map(rois5, finest, L):
    """lib/region.py:256-264 on [K,5] rois."""
    r = _c32(rois5)
    out = np.empty(r.shape[0], np.int64)
    lib().orc_roi_level_map(_f(r), ctypes.c_int64(r.shape[0]), ctypes.c_float(finest), L, out.ctypes.data_as(_I64))
    return out


def nms(boxes, scores, thr, max_keep=-1):
    """torchvision.ops.nms(boxes [N,4], scores [N], thr): stable descending sort + greedy."""
    boxes = _c32(boxes).reshape(-1, 4)
    scores = np.asarray(scores, np.float32)
    order = np.argsort(-scores, kind='stable')
    sb = np.ascontiguousarray(boxes[order])
    keep = np.empty(max(len(order), 1), np.int64)
    k = lib().orc_nms_sorted(_f(sb), ctypes.c_int64(len(order)), ctypes.c_double(thr), ctypes.c_int64(max_keep),
                             keep.ctypes.data_as(_I64))
    return order[keep[:k]]


def _strides_of(feats):
    st = []
    for f in feats:
        st += [s // f.itemsize for s in f.strides]
    return np.asarray(st, np.int64)


def roi_align(feats, rois5, levels, scales, output_size, sampling_ratio, aligned=False):
    """Multi-level torchvision RoIAlign forward; feats list of [B,C,H,W] f32 arrays."""
    feats = [_c32(f) for f in feats]
    rois5 = _c32(rois5)
    K, C = rois5.shape[0], feats[0].shape[1]
    ph, pw = output_size
    out = np.empty((K, C, ph, pw), np.float32)
    fp = (ctypes.c_void_p * len(feats))(*[f.ctypes.data for f in feats])
    hw = np.asarray([v for f in feats for v in f.shape[2:]], np.int32)
    st = _strides_of(feats)
    lv = np.ascontiguousarray(levels, np.int64) if levels is not None else None
    lib().orc_roi_align_fwd(len(feats), fp, hw.ctypes.data_as(_I32), st.ctypes.data_as(_I64),
                            _f(_c32(scales)), C, _f(rois5), lv.ctypes.data_as(_I64) if lv is not None else None,
                            ctypes.c_int64(K), ph, pw, int(sampling_ratio), int(aligned), _f(out))
    return out


def roi_align_bwd(feat_shapes, rois5, levels, scales, grad_out, sampling_ratio, aligned=False):
    grads = [np.zeros(s, np.float32) for s in feat_shapes]
    rois5 = _c32(rois5)
    g = _c32(grad_out)
    K, C, ph, pw = g.shape
    fp = (ctypes.c_void_p * len(grads))(*[x.ctypes.data for x in grads])
    hw = np.asarray([v for s in feat_shapes for v in s[2:]], np.int32)
    st = _strides_of(grads)
    lv = np.ascontiguousarray(levels, np.int64) if levels is not None else None
    lib().orc_roi_align_bwd(len(grads), fp, hw.ctypes.data_as(_I32), st.ctypes.data_as(_I64), _f(_c32(scales)), C,
                            _f(rois5), lv.ctypes.data_as(_I64) if lv is not None else None, ctypes.c_int64(K), ph, pw,
                            int(sampling_ratio), int(aligned), _f(g))
    return grads


def roi_pool(feat, rois5, output_size, scale):
    feat, rois5 = _c32(feat), _c32(rois5)
    K, C = rois5.shape[0], feat.shape[1]
    ph, pw = output_size
    out = np.empty((K, C, ph, pw), np.float32)
    am = np.empty((K, C, ph, pw), np.int32)
    st = _strides_of([feat])
    lib().orc_roi_pool_fwd(_f(feat), st.ctypes.data_as(_I64), feat.shape[2], feat.shape[3], C, ctypes.c_float(scale),
                           _f(rois5), ctypes.c_int64(K), ph, pw, _f(out), am.ctypes.data_as(_I32))
    return out, am


# ------------------------------------------------------------------ per-image glue
def random_sample_label(labels, pos_num, tot_num):
    """lib/region.py:43-57 on a numpy int64 label vector (1/0/-1), numpy global RNG."""
    labels = labels.copy()
    pos = np.nonzero(labels == 1)[0]
    if len(pos) > pos_num:
        dis = np.random.choice(pos, size=len(pos) - pos_num, replace=False)
        labels[dis] = -1
    n_negs = tot_num - min(len(pos), pos_num)
    neg = np.nonzero(labels == 0)[0]
    if len(neg) > n_negs:
        dis = np.random.choice(neg, size=len(neg) - n_negs, replace=False)
        labels[dis] = -1
    return labels


def random_sampler(labels, max_num, pos_num):
    """RandomSampler.__call__ (lib/region.py:118-126)."""
    l1 = labels.copy()
    l1[labels > 0] = 1
    l1 = random_sample_label(l1, pos_num, max_num)
    pos = l1 == 1
    l1[pos] = labels[pos]
    return l1


def anchor_target(cls_out, reg_out, cls_channels, in_anchors, in_mask, gt_bbox, gt_label, assign, sampler,
                  means, stds):
    """lib/anchor.py:11-76.  assign = (pos, neg, min_pos); sampler = (max_num, pos_num), None, or a
    callable labels -> sampled labels (tests: a given selection, e.g. the device sampler's)."""
    labels, _ = maxiou_assign(in_anchors, gt_bbox, *assign)
    if callable(sampler):
        labels = sampler(labels)
    elif sampler is not None:
        labels = random_sampler(labels, *sampler)
    non_neg = labels >= 0
    zero = labels == 0
    lab_ = labels.copy()
    lab_[lab_ > 0] = 1
    g = labels - 1
    g[g < 0] = 0
    chosen = np.nonzero(in_mask)[0][non_neg]
    tar_cls_out = cls_out.reshape(cls_channels, -1)[:, chosen]
    tar_reg_out = reg_out.reshape(4, -1)[:, chosen]
    if gt_label is None:
        tar_labels = lab_[non_neg]
    else:
        gl = np.asarray(gt_label, np.int64)[g]
        gl[zero] = 0
        tar_labels = gl[non_neg]
    tar_anchors = in_anchors[:, non_neg]
    tar_bbox = np.asarray(gt_bbox, np.float32)[:, g][:, non_neg]
    tar_param = bbox2param(tar_anchors, tar_bbox, means, stds)
    return tar_cls_out, tar_reg_out, tar_labels, tar_anchors, tar_bbox, tar_param, chosen


def bbox_target(props, gt_bbox, gt_label, assign, sampler, means=None, stds=None):
    """lib/bbox.py:6-78 -> (tar_props, tar_bbox, tar_label, tar_param, tar_is_gt)."""
    gt_bbox = np.asarray(gt_bbox, np.float32)
    labels, ious = maxiou_assign(props, gt_bbox, *assign)
    G = gt_bbox.shape[1]
    props = np.concatenate([gt_bbox, np.asarray(props, np.float32)], 1)
    labels = np.concatenate([np.arange(1, G + 1, dtype=np.int64), labels])
    labels = sampler(labels) if callable(sampler) else random_sampler(labels, *sampler)
    chosen = labels >= 0
    neg = labels == 0
    is_gt = np.zeros(props.shape[1], np.int64)
    is_gt[:G] = 1
    g = labels - 1
    g[g < 0] = 0
    cls = np.asarray(gt_label, np.int64)[g]
    cls[neg] = 0
    tp = props[:, chosen]
    tb = gt_bbox[:, g][:, chosen]
    return tp, tb, cls[chosen], bbox2param(tp, tb, means, stds), is_gt[chosen]


def sigmoid(x):
    return (1.0 / (1.0 + np.exp(-x.astype(np.float32)))).astype(np.float32)


def rpn_predict_single_image(level_cls, level_reg, level_anchors, img_size, min_size, pre_nms, post_nms, max_num,
                             nms_iou, means=(0, 0, 0, 0), stds=(1, 1, 1, 1), scores=None):
    """RPNHead.predict_single_image (lib/heads/rpn_head.py:68-120), sigmoid RPN.

    `scores` (optional, per level) injects precomputed scores so a test can
    compare the discrete steps on identical inputs.  Top-k order: (score desc,
    index asc); the reference's torch.topk tie order is implementation-defined."""
    out_s, out_b = [], []
    for i, (co, ro, an) in enumerate(zip(level_cls, level_reg, level_anchors)):
        sc = sigmoid(co.reshape(-1)) if scores is None else np.asarray(scores[i], np.float32)
        ro, an = ro.reshape(4, -1), an.reshape(4, -1)
        if 0 < pre_nms < len(sc):
            idx = np.argsort(-sc, kind='stable')[:pre_nms]
            sc, ro, an = sc[idx], ro[:, idx], an[:, idx]
        bx = param2bbox(an, ro, means, stds, img_size)
        if min_size > 0:
            ns = ((bx[2] - bx[0] + np.float32(1)) >= np.float32(min_size)) & \
                 ((bx[3] - bx[1] + np.float32(1)) >= np.float32(min_size))
            sc, bx = sc[ns], bx[:, ns]
        keep = nms(bx.T, sc, nms_iou)
        sc, bx = sc[keep], bx[:, keep]
        if 0 < post_nms < len(sc):
            sc, bx = sc[:post_nms], bx[:, :post_nms]
        out_s.append(sc)
        out_b.append(bx)
    s = np.concatenate(out_s)
    b = np.concatenate(out_b, 1)
    if 0 < max_num < len(s):
        idx = np.argsort(-s, kind='stable')[:max_num]
        s, b = s[idx], b[:, idx]
    return b, s


def atss_targets(anchors, grids, strides, gts, labels, img_shape, topk=9):
    """FCOSHead.single_image_targets_atss (fcos_head.py:283-368) for one image.
    anchors: per-level [4, H*W] f32 (one anchor per cell); gts [4, G]; labels [G].
    Returns level-concatenated (cls int64 [N], reg f32 [N, 4], ctr f32 [N])."""
    L = len(grids)
    gh = np.array([g[0] for g in grids], np.int32)
    gw = np.array([g[1] for g in grids], np.int32)
    N = int((gh.astype(np.int64) * gw).sum())
    an = [np.ascontiguousarray(a, np.float32).reshape(4, -1) for a in anchors]
    ap = (ctypes.c_void_p * L)(*[a.ctypes.data for a in an])
    g = np.ascontiguousarray(gts, np.float32).reshape(4, -1)
    lab = np.ascontiguousarray(labels, np.int64)
    cls = np.empty(N, np.int64)
    reg = np.empty((N, 4), np.float32)
    ctr = np.empty(N, np.float32)
    lib().orc_atss_targets(L, gh.ctypes.data_as(_I32), gw.ctypes.data_as(_I32), _f(_c32(strides)), ap, _f(g),
                           ctypes.c_int64(g.shape[1]), lab.ctypes.data_as(_I64), int(img_shape[0]),
                           int(img_shape[1]), int(topk), cls.ctypes.data_as(_I64), _f(reg), _f(ctr))
    return cls, reg, ctr


def multiclass_nms(bbox, score, nms_channel, nms_iou, min_score=-1, max_num=None, score_factor=None,
                   mode='official'):
    """utils.multiclass_nms (lib/utils.py:224-269) + batched_nms (:211-221) in numpy f32:
    candidate (box, class) pairs, coordinate offset label * max(candidate coords), one
    greedy nms (this module's `nms`, torchvision semantics), first max_num."""
    bbox = np.asarray(bbox, np.float32)
    score = np.asarray(score, np.float32)
    n, ncls = score.shape
    simple = bbox.shape[1] == 4
    chans = np.zeros(ncls, bool)
    chans[list(nms_channel)] = True
    if mode == 'official':
        label = np.where(chans[None, :], np.arange(ncls)[None, :], -1).repeat(n, 0)
        boxes = np.repeat(bbox[:, :, None], ncls, 2) if simple else bbox.reshape(n, 4, ncls)
        boxes = boxes.transpose(0, 2, 1)
        chosen = (score >= np.float32(min_score)) & (label != -1)
        if score_factor is not None:
            sf = np.asarray(score_factor, np.float32)
            score = score * (sf[:, None] if sf.ndim == 1 else sf)
        nb, ns, nl = boxes[chosen], score[chosen], label[chosen]
    else:
        lab = score.argmax(1)
        sc = score[np.arange(n), lab]
        if not simple:
            bbox = bbox.reshape(n, 4, ncls)[np.arange(n), :, lab]
        chosen = (sc >= np.float32(min_score)) & chans[lab]
        if score_factor is not None:
            sc = sc * np.asarray(score_factor, np.float32)
        nb, ns, nl = bbox[chosen], sc[chosen], lab[chosen]
    if ns.size == 0:
        return nb, ns, nl
    mx = nb.max()
    off = nb + (nl.astype(np.float32) * mx).astype(np.float32)[:, None]
    keep = np.asarray(nms(off, ns, nms_iou), np.int64)
    kb, ks, kl = nb[keep], ns[keep], nl[keep]
    if max_num is not None and ks.size > max_num:
        kb, ks, kl = kb[:max_num], ks[:max_num], kl[:max_num]
    return kb, ks, kl


# ------------------------------------------------------------------ losses (float64 restatements)
def sigmoid_focal_loss(pred, target, alpha=0.25, gamma=2.0):
    """lib/losses.py:33-61 summed, in float64: pred [n, C] logits, target [n] (0 = background,
    k -> one-hot column k-1); BCE-with-logits * (alpha_t * (1 - p_t) ** gamma)."""
    x = np.asarray(pred, np.float64)
    t = np.zeros_like(x)
    tg = np.asarray(target, np.int64)
    fg = tg > 0
    t[np.nonzero(fg)[0], tg[fg] - 1] = 1.0
    p = 1.0 / (1.0 + np.exp(-x))
    pt = p * t + (1 - p) * (1 - t)
    w = (alpha * t + (1 - alpha) * (1 - t)) * (1 - pt) ** gamma
    bce = np.maximum(x, 0) - x * t + np.log1p(np.exp(-np.abs(x)))
    return float((bce * w).sum())


def smooth_l1_v2(x, y, beta):
    """lib/losses.py:77-83 summed, in float64."""
    d = np.abs(np.asarray(x, np.float64) - np.asarray(y, np.float64))
    return float(np.where(d < beta, d * d / (2 * beta), d - 0.5 * beta).sum())


def anchor_head_loss(level_cls, level_reg, level_anchors, strides, gts, labels, img_shape, assign, allowed_border,
                     beta, cls_channels, means=(0, 0, 0, 0), stds=(1, 1, 1, 1)):
    """AnchorHead.loss for a sigmoid focal-loss head without sampler (lib/heads/anchor_head.py:152-199,
    per-image targets :69-111, calc_loss :113-139, avg_factor = #positives).
    level_cls / level_reg: per level [B, A*C, H, W] / [B, A*4, H, W]; level_anchors: per level
    [4, A, H, W].  Returns (cls_loss, reg_loss, (tar_cls_out, tar_reg_out, tar_labels, tar_param))
    with the targets concatenated in image order."""
    A = level_anchors[0].shape[1]
    anc = np.concatenate([a.reshape(4, -1) for a in level_anchors], 1)
    ingrid = np.concatenate([inside_grid_mask(A, img_shape, a.shape[2:], s)
                             for a, s in zip(level_anchors, strides)]).astype(bool)
    mask = ingrid & inside_anchor_mask(anc, img_shape, allowed_border)
    outs = [[] for _ in range(4)]
    for b in range(len(gts)):
        co = np.concatenate([c[b].reshape(cls_channels, -1) for c in level_cls], 1)
        ro = np.concatenate([r[b].reshape(4, -1) for r in level_reg], 1)
        t = anchor_target(co, ro, cls_channels, anc[:, mask], mask, gts[b], labels[b], assign, None, means, stds)
        for k, v in enumerate((t[0], t[1], t[2], t[5])):
            outs[k].append(v)
    tc, tr = np.concatenate(outs[0], 1), np.concatenate(outs[1], 1)
    tl, tp = np.concatenate(outs[2]), np.concatenate(outs[3], 1)
    pos = tl > 0
    npos = int(pos.sum())
    if tl.size == 0:
        return 0.0, 0.0, (tc, tr, tl, tp)
    cls_loss = sigmoid_focal_loss(tc.T, tl) / npos if npos else float('inf')
    reg_loss = smooth_l1_v2(tr[:, pos], tp[:, pos], beta) / npos if npos else 0.0
    return cls_loss, reg_loss, (tc, tr, tl, tp)

"""Deterministic synthetic inputs shared by the golden generator and the tests.

Everything here is numpy (PCG64 `default_rng`, stable across platforms) so the
GPU box regenerates bit-identical inputs without the reference present; the
only stored inputs are the VOC ground-truth boxes (tests/golden/voc_gts.npz).
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

IMG_SHAPE = (600, 1000)
PAD_SHAPE = (608, 1024)
# cfg2/cfg4 FPN: strides 4..64; P6 = P5[::2, ::2]
FPN_STRIDES = [4, 8, 16, 32, 64]
FPN_GRIDS = [(152, 256), (76, 128), (38, 64), (19, 32), (10, 16)]
# cfg3 / cfg5: strides 8..128 (P3..P7)
RETINA_STRIDES = [8, 16, 32, 64, 128]
RETINA_GRIDS = [(76, 128), (38, 64), (19, 32), (10, 16), (5, 8)]
# cfg1 C4: one level, stride 16
C4_GRIDS = [(38, 64)]


def img_meta(scale_factor=1.6):
    return {'img_shape': IMG_SHAPE + (3,), 'pad_shape': PAD_SHAPE + (3,), 'scale_factor': scale_factor,
            'ori_shape': (375, 625, 3)}


def voc_gts():
    """[(boxes [4, G] f32 xyxy in the 1000x600 frame, labels int64 [G])] from the committed fixture."""
    z = np.load(os.path.join(HERE, 'voc_gts.npz'))
    out = []
    for i in range(int(z['n'])):
        out.append((z['boxes_{}'.format(i)].astype(np.float32), z['labels_{}'.format(i)].astype(np.int64)))
    return out


def head_outputs(seed, grids, num_anchors, cls_channels, batch=1, cls_scale=1.0, reg_scale=0.1):
    """Per-level (cls [B, C*A, H, W], reg [B, 4*A, H, W]) f32 arrays."""
    rng = np.random.default_rng(seed)
    cls, reg = [], []
    for h, w in grids:
        cls.append((rng.standard_normal((batch, cls_channels * num_anchors, h, w)) * cls_scale).astype(np.float32))
        reg.append((rng.standard_normal((batch, 4 * num_anchors, h, w)) * reg_scale).astype(np.float32))
    return cls, reg


def random_boxes(seed, n, img=IMG_SHAPE, min_wh=2.0, max_wh=400.0):
    """[4, n] f32 xyxy boxes inside the image."""
    rng = np.random.default_rng(seed)
    w = rng.uniform(min_wh, max_wh, n)
    h = rng.uniform(min_wh, max_wh, n)
    x1 = rng.uniform(0, img[1] - 1, n)
    y1 = rng.uniform(0, img[0] - 1, n)
    x2 = np.minimum(x1 + w, img[1] - 1)
    y2 = np.minimum(y1 + h, img[0] - 1)
    return np.stack([x1, y1, x2, y2]).astype(np.float32)


def golden_path(name):
    return os.path.join(HERE, name)


def feature_maps(seed, grids, channels, batch):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal((batch, channels, h, w)).astype(np.float32) for h, w in grids]


def atss_cases():
    """(gt boxes [4, G] f32, labels [G] i64) cases for the ATSS fixtures: 8 VOC images plus
    synthetic sets (many boxes, tiny boxes, border boxes, one box)."""
    gts = voc_gts()
    cases = [gts[i] for i in range(8)]
    rng = np.random.default_rng(77)
    b = random_boxes(21, 40)
    cases.append((b, rng.integers(1, 21, 40).astype(np.int64)))
    b = random_boxes(22, 12, min_wh=1.0, max_wh=12.0)
    cases.append((b, rng.integers(1, 21, 12).astype(np.int64)))
    b = np.array([[0, 0, 40, 30], [950, 560, 999, 599], [0, 300, 999, 599], [480, 0, 520, 599]], np.float32).T
    cases.append((b.copy(), np.array([3, 7, 11, 15], np.int64)))
    cases.append((np.array([[100.5], [200.25], [300.75], [260.0]], np.float32), np.array([9], np.int64)))
    return cases


# (mode, n boxes, score channels, class-specific boxes, score factor) for multiclass_nms
MCNMS_CASES = [('official', 300, 21, False, False), ('official', 400, 21, True, False),
               ('strict', 500, 20, False, True), ('strict', 300, 21, True, False)]


def mcnms_inputs(i):
    """(bbox [n, 4] or [n, 4*C], score [n, C], score_factor or None, channels) of case i:
    clustered boxes (heavy overlap) with softmax / sigmoid-like scores."""
    mode, n, ncls, per_class, factor = MCNMS_CASES[i]
    rng = np.random.default_rng(1100 + i)
    ctr = rng.uniform(50, 950, (12, 2))
    k = rng.integers(0, 12, n)
    wh = rng.uniform(20, 200, (n, 2))
    c = ctr[k] + rng.normal(0, 15, (n, 2))
    base = np.stack([c[:, 0] - wh[:, 0] / 2, c[:, 1] - wh[:, 1] / 2, c[:, 0] + wh[:, 0] / 2, c[:, 1] + wh[:, 1] / 2], 1)
    if per_class:
        jit = rng.normal(0, 4, (n, 4, ncls))
        bbox = (base[:, :, None] + jit).reshape(n, 4 * ncls)
    else:
        bbox = base
    logits = rng.normal(0, 2, (n, ncls))
    if mode == 'official':
        e = np.exp(logits - logits.max(1, keepdims=True))
        score = e / e.sum(1, keepdims=True)
        channels = list(range(1, ncls))
    else:
        score = 1 / (1 + np.exp(-logits))
        channels = list(range(0, ncls))
    sf = rng.uniform(0.2, 1.0, n).astype(np.float32) if factor else None
    return bbox.astype(np.float32), score.astype(np.float32), sf, channels


def refine_inputs(agnostic, n=512, ncls=21):
    """(props [4, n], label [n], reg_out [n, 4] or [n, 4*C], is_gt [n] u8) for BBoxHead.refine."""
    rng = np.random.default_rng(1200 + int(agnostic))
    props = random_boxes(1201, n)
    label = rng.integers(0, ncls, n).astype(np.int64)
    reg_out = rng.normal(0, 1.0, (n, 4 if agnostic else 4 * ncls)).astype(np.float32)
    is_gt = (np.arange(n) < 9).astype(np.uint8)
    return props, label, reg_out, is_gt


def eval_case():
    """Fixed detections for the f3 evaluation fixture (tester.py:25-57 -> test.py:75-90):
    per image (meta, boxes [4, n] f32 xyxy in the resized frame, scores [n] f32, labels [n]
    i64); image 2 has no detections (the reference's warning/skip branch).  Plus a COCO
    ground truth in the original frame: jittered copies of about half the detections
    (some with another class, one crowd), and missed objects."""
    rng = np.random.default_rng(1300)
    names = ['000005.jpg', '000123.jpg', '001234.jpg', '009999.jpg']
    counts = [37, 0, 12, 100]
    images, anns, aid = [], [], 1
    for name, n in zip(names, counts):
        sf = float(rng.choice([1.6, 1.5, 2.0]))
        meta = {'filename': '/data/VOC2007/JPEGImages/' + name, 'ori_shape': (375, 625, 3), 'scale_factor': sf,
                'img_shape': IMG_SHAPE + (3,), 'pad_shape': PAD_SHAPE + (3,)}
        b = random_boxes(int(rng.integers(1 << 30)), n, min_wh=4.0, max_wh=300.0)
        s = np.sort(rng.uniform(0.05, 1.0, n)).astype(np.float32)[::-1].copy()
        lab = rng.integers(1, 21, n).astype(np.int64)
        images.append((meta, b, s, lab))
        iid = int(name[:-4])
        for j in range(n):
            if rng.random() < 0.5:
                x1, y1, x2, y2 = (b[:, j] / sf).tolist()
                w, h = x2 - x1 + 1, y2 - y1 + 1
                jit = rng.normal(0, 0.08, 4) * [w, h, w, h]
                box = [round(float(v), 2) for v in np.add([x1, y1, w, h], jit).clip(1.0)]
                cat = int(lab[j]) if rng.random() < 0.85 else int(rng.integers(1, 21))
                anns.append({'id': aid, 'image_id': iid, 'category_id': cat, 'bbox': box,
                             'iscrowd': int(aid == 7), 'area': box[2] * box[3]})
                aid += 1
        for _ in range(3):
            box = [round(float(v), 2) for v in (rng.uniform(0, 500), rng.uniform(0, 300), rng.uniform(8, 120),
                                                rng.uniform(8, 120))]
            anns.append({'id': aid, 'image_id': iid, 'category_id': int(rng.integers(1, 21)), 'bbox': box,
                         'iscrowd': 0, 'area': box[2] * box[3]})
            aid += 1
    gt = {'images': [{'id': int(n[:-4]), 'file_name': n} for n in names], 'annotations': anns,
          'categories': [{'id': c} for c in range(1, 21)]}
    return images, gt


# ---------------------------------------------------------------- full forward_train case
FTRAIN_SHAPE = (256, 384)
FTRAIN_NP_SEED = 20240607  # np.random.seed before forward_train: the samplers' legacy RNG


def seeded_state(shapes):
    """A deterministic state_dict for a model with these {key: shape} entries (the reference's
    CascadeRCNN and frcnn_amd's have identical keys / shapes): each tensor from its own
    PCG64 stream keyed by crc32(key).  Conv / FC weights ~ N(0, 2 / fan_in), the RPN and RCNN
    output layers ~ N(0, 0.01^2) (scores away from saturation, no exact ties), frozen-BN
    weights 1 + 0.1 N (0.2 + 0.02 N on each block's last BN and shortcut BN, so the residual
    stream stays O(1) through 16 blocks), biases / running means 0.05 N, running vars
    1 + 0.1 U."""
    import zlib
    out = {}
    for key in sorted(shapes):
        shape = tuple(shapes[key])
        rng = np.random.default_rng(zlib.crc32(key.encode()))
        if key.endswith('num_batches_tracked'):
            out[key] = np.zeros(shape, np.int64)
            continue
        if key.endswith('running_var'):
            v = 1.0 + 0.1 * rng.random(shape)
        elif key.endswith('running_mean') or key.endswith('bias'):
            v = 0.05 * rng.standard_normal(shape)
        elif len(shape) == 1 and (key.endswith('bn3.weight') or key.endswith('downsample.1.weight')):
            v = 0.2 + 0.02 * rng.standard_normal(shape)  # residual branches / shortcuts damped: bounded stream
        elif len(shape) == 1:  # BN weight
            v = 1.0 + 0.1 * rng.standard_normal(shape)
        elif ('classifier' in key or 'regressor' in key) and ('rpn_head' in key or 'rcnn_head' in key):
            v = 0.01 * rng.standard_normal(shape)
        else:
            v = rng.standard_normal(shape) * np.sqrt(2.0 / float(np.prod(shape[1:])))
        out[key] = v.astype(np.float32)
    return out


def ftrain_case(shape=FTRAIN_SHAPE):
    """One image (default 256x384, N(0,1) pixels) with the 5 boxes of VOC gt set 9 scaled into
    it: (img [1, 3, H, W] f32, boxes [[4, G] f32], labels [[G] i64], img_metas)."""
    shape = tuple(shape)
    rng = np.random.default_rng(4242)
    img = rng.standard_normal((1, 3) + shape).astype(np.float32)
    b, l = voc_gts()[9]
    f = 0.38 * shape[0] / FTRAIN_SHAPE[0]
    b = (b * np.float32(f)).astype(np.float32)
    meta = {'img_shape': shape + (3,), 'pad_shape': shape + (3,), 'scale_factor': f * 1.6,
            'ori_shape': (160, 240, 3)}
    return img, [b], [l], [meta]


# BASELINE configs whose whole detector (forward_train losses + forward_test detections) is
# pinned to the reference's own outputs (gen_golden.gen_whole_detectors): (tag, config file,
# test_cfg overrides, image shape).  The two-stage configs' RCNN classifiers are N(0, 0.01^2)
# under seeded_state, so every softmax score sits near 1/21 < 0.05: their fixtures lower
# min_score to 0 (every (proposal, class) pair is a multiclass-NMS candidate: one offset NMS
# over up to 20 000 boxes).  cfg1 is the C4 graph: one stride-16 level, RoIPool (its
# sampling_ratio accepted and ignored), pre_nms 12 000.  cfg5 runs on 384x640: the reference's ATSS top-9 per level needs
# 9 cells on P7 (stride 128).
WHOLE_DETECTORS = [('cfg1', 'faster_rcnn_r50.py', {'rcnn': {'min_score': 0.0}}, FTRAIN_SHAPE),
                   ('cfg2', 'faster_rcnn_r50_fpn.py', {'rcnn': {'min_score': 0.0}}, FTRAIN_SHAPE),
                   ('cfg3', 'retinanet_r50_fpn.py', {}, FTRAIN_SHAPE),
                   ('cfg4', 'cascade_rcnn_r50_fpn.py', {'rcnn': {'min_score': 0.0}}, FTRAIN_SHAPE),
                   ('cfg5', 'fcos_r50_fpn_atss.py', {}, (384, 640))]

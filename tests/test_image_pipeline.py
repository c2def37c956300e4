"""Image pipeline: mmdet v1 Resize/RandomFlip/Normalize/Pad + collate.

CPU: the oracle restatement (oracle/image_prep.py) on hand-computed cases, the host-side
size / box / img_meta rules of frcnn_amd.datasets, and the COCO-json dataset parsing.
GPU: frh_image_preprocess bit-exact against the oracle (integer resize, f32 normalise),
and a real-file batch through forward_train.  cv2 / mmcv / mmdet are absent, so parity with
them is unpinned; the cases below are computed by hand from their published algorithms."""
import json

import numpy as np
import pytest
import torch

import image_prep
from frcnn_amd import datasets

REF_TRAIN_PIPELINE = [  # configs/faster_rcnn_r50_fpn.py:119-128 (data, not code)
    dict(type='LoadImageFromFile'),
    dict(type='LoadAnnotations', with_bbox=True),
    dict(type='Resize', img_scale=(1333, 800), keep_ratio=True),
    dict(type='RandomFlip', flip_ratio=0.5),
    dict(type='Normalize', mean=[123.675, 116.28, 103.53], std=[58.395, 57.12, 57.375], to_rgb=True),
    dict(type='Pad', size_divisor=32),
    dict(type='DefaultFormatBundle'),
    dict(type='Collect', keys=['img', 'gt_bboxes', 'gt_labels']),
]


def test_resize_identity_and_constant():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    np.testing.assert_array_equal(image_prep.resize_linear_u8(img, 37, 53), img)
    const = np.full((20, 30, 3), 77, np.uint8)
    for nh, nw in ((41, 61), (9, 13), (20, 47)):
        np.testing.assert_array_equal(image_prep.resize_linear_u8(const, nh, nw), 77)


def test_resize_linear_by_hand():
    # 1x2 -> 1x4: scale 0.5; f = -0.25 (clamped), 0.25, 0.75, 1.25 (clamped);
    # weights (1536, 512) and (512, 1536) of 2048: 100 * 512 * 2048 / 2^22 = 25.0 -> 25, 75
    img = np.zeros((1, 2, 3), np.uint8)
    img[0, 1] = 100
    out = image_prep.resize_linear_u8(img, 1, 4)
    assert out[0, :, 0].tolist() == [0, 25, 75, 100]
    # rounding: 1x2 [0, 1] -> 1x4 gives (512 * 2048 + 2^21) >> 22 = 0 and (1536 * 2048 + 2^21) >> 22 = 1
    img[0, 1] = 1
    assert image_prep.resize_linear_u8(img, 1, 4)[0, :, 0].tolist() == [0, 0, 1, 1]


def test_resize_exact_half_is_area_mean():
    img = np.array([[[1], [2], [5], [7]], [[3], [6], [0], [0]]], np.uint8).repeat(3, 2)
    out = image_prep.resize_linear_u8(img, 1, 2)
    assert out[0, :, 0].tolist() == [(1 + 2 + 3 + 6 + 2) >> 2, (5 + 7 + 0 + 0 + 2) >> 2]


def test_rescale_size_and_pipeline_config():
    assert datasets.rescale_size(375, 500, (1333, 800)) == ((1067, 800), 800 / 375)
    assert datasets.rescale_size(600, 1000, (1000, 600))[0] == (1000, 600)
    p = datasets.ImagePipeline.from_config(REF_TRAIN_PIPELINE)
    assert p.img_scale == (1333, 800) and p.keep_ratio and p.flip_ratio == 0.5 and p.size_divisor == 32
    assert p.to_rgb and np.allclose(p.std, [58.395, 57.12, 57.375])
    nh, nw, s = p._plan(375, 500)
    assert (nh, nw, p._pad(nh), p._pad(nw)) == (800, 1067, 800, 1088)
    with pytest.raises(ValueError):
        datasets.ImagePipeline.from_config([dict(type='PhotoMetricDistortion')])


def test_box_transform():
    meta = {'img_shape': (800, 1067, 3), 'scale_factor': 2.0, 'flip': False}
    b = np.array([[10, 20, 100, 200], [400, 300, 600, 399]], np.float32)
    np.testing.assert_array_equal(datasets.transform_boxes(b, meta), [[20, 40, 200, 400], [800, 600, 1066, 798]])
    meta['flip'] = True
    np.testing.assert_array_equal(datasets.transform_boxes(b, meta),
                                  [[1067 - 200 - 1, 40, 1067 - 20 - 1, 400], [0, 600, 1067 - 800 - 1, 798]])


def _write_dataset(tmp_path, sizes):
    from PIL import Image
    rng = np.random.default_rng(3)
    images, anns = [], []
    for i, (h, w) in enumerate(sizes):
        fn = '{:06d}.png'.format(i + 1)
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / fn)
        images.append({'id': i + 1, 'file_name': fn, 'width': w, 'height': h})
        anns += [{'id': 10 * i + 1, 'image_id': i + 1, 'category_id': 12, 'bbox': [5, 6, 40, 30], 'area': 1200,
                  'iscrowd': 0},
                 {'id': 10 * i + 2, 'image_id': i + 1, 'category_id': 3, 'bbox': [50, 20, 0.5, 10], 'area': 5,
                  'iscrowd': 0},
                 {'id': 10 * i + 3, 'image_id': i + 1, 'category_id': 7, 'bbox': [1, 1, 20, 20], 'area': 400,
                  'iscrowd': 1}]
    images.append({'id': 99, 'file_name': 'none.png', 'width': 100, 'height': 100})  # no annotations
    cats = [{'id': c, 'name': n} for c, n in zip(range(1, 21), datasets.VOC_CLASSES)]
    ann_file = tmp_path / 'ann.json'
    ann_file.write_text(json.dumps({'images': images, 'annotations': anns, 'categories': cats}))
    return str(ann_file)


def test_dataset_parsing(tmp_path):
    ann = _write_dataset(tmp_path, [(60, 80), (48, 64)])
    ds = datasets.VOCDataset(ann, str(tmp_path), REF_TRAIN_PIPELINE, seed=0)
    assert len(ds) == 2  # the image without annotations is filtered in training mode
    a = ds.ann_info(0)
    np.testing.assert_array_equal(a['bboxes'], [[5, 6, 44, 35]])   # x1 + w - 1; the w < 1 box dropped
    assert a['labels'].tolist() == [12]
    np.testing.assert_array_equal(a['bboxes_ignore'], [[1, 1, 20, 20]])
    rec = ds[1]
    assert rec['img'].shape == (48, 64, 3) and rec['img'].dtype == np.uint8
    from PIL import Image
    rgb = np.asarray(Image.open(tmp_path / '000002.png'))
    np.testing.assert_array_equal(rec['img'], rgb[..., ::-1])  # BGR like mmcv.imread
    assert len(datasets.VOCDataset(ann, str(tmp_path), REF_TRAIN_PIPELINE, test_mode=True)) == 3


# ---------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize('case', ['upscale', 'identity', 'half', 'odd'])
def test_preprocess_matches_oracle(case):
    dev = torch.device('cuda', 0)
    rng = np.random.default_rng(["upscale", "identity", "half", "odd"].index(case))
    shapes, scale = {'upscale': ([(375, 500), (333, 500), (500, 281)], (1333, 800)),
                     'identity': ([(600, 1000)], (1000, 600)),
                     'half': ([(1200, 1600), (800, 1200)], (800, 600)),
                     'odd': ([(17, 23), (5, 9), (64, 3)], (101, 37))}[case]
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in shapes]
    flips = [i % 2 == 1 for i in range(len(imgs))]
    p = datasets.ImagePipeline(img_scale=scale, size_divisor=32)
    out, metas, _ = p(imgs, device=dev, flips=flips)
    sizes = [m['img_shape'][:2] for m in metas]
    ref = image_prep.preprocess(imgs, sizes, flips, p.mean, p.std, True, out.shape[2], out.shape[3])
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    for m in metas:
        assert m['pad_shape'][0] % 32 == 0 and m['pad_shape'][1] % 32 == 0
    if case == 'half':
        assert sizes[0] == (600, 800)  # exact 2x: the INTER_AREA path


@pytest.mark.gpu
def test_dataset_batch_trains(tmp_path):
    import bench
    dev = torch.device('cuda', 0)
    ann = _write_dataset(tmp_path, [(300, 500), (375, 500)])
    pipe = [dict(s) for s in REF_TRAIN_PIPELINE]
    pipe[2] = dict(type='Resize', img_scale=(1000, 600), keep_ratio=True)
    ds = datasets.VOCDataset(ann, str(tmp_path), pipe, seed=0)
    batch = ds.collate([ds[0], ds[1]], device=dev)
    assert batch['img'].shape == (2, 3, 608, 1024)  # (600, 1000) and (600, 800) padded to the batch max
    assert batch['gt_bboxes'][0].shape == (4, 1)
    model, _ = bench.make_model(dev, seed=0)
    losses = model.forward_train(batch['img'], batch['gt_bboxes'], batch['gt_labels'], batch['img_meta'])
    total = sum(losses.values())
    assert torch.isfinite(total)
    total.backward()

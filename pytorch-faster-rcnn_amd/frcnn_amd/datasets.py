"""Data format of the reference: the mmdet v1 pipelines and
img_meta / batch layout, with the per-pixel work on the device.

Reference: configs/faster_rcnn_r50_fpn.py:115-160 (img_norm, train_pipeline,
test_pipeline, data), lib/datasets.py:1-31 (VOCDataset = mmdet CocoDataset with the 20
VOC classes), lib/trainer/trainer.py:100-108 and lib/tester.py:33-35 (what the batch
holds: 'img' [B, 3, H, W], 'img_meta' list, 'gt_bboxes' [n, 4] -> .t(), 'gt_labels').

The host side here does what is per image and scalar in mmcv/mmdet -- the keep-ratio
scale (mmcv.imrescale), box scaling + clipping (mmdet Resize), box flipping
(mmdet bbox_flip, inclusive pixels), pad shapes (size_divisor) and the img_meta dicts.
The per-pixel work (bilinear resize, flip, normalise, pad, HWC -> CHW, batch collation)
is one HIP launch (frh_image_preprocess, csrc/image.hip).  Images are decoded on the
host (PIL; mmcv.imread's cv2 decoder is absent here) into BGR uint8 like mmcv.imread.
"""
import json
import math
import os.path as osp

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_of

VOC_CLASSES = ('aeroplane', 'bicycle', 'bird', 'boat', 'bottle', 'bus', 'car', 'cat', 'chair', 'cow', 'diningtable',
               'dog', 'horse', 'motorbike', 'person', 'pottedplant', 'sheep', 'sofa', 'train', 'tvmonitor')


def load_image(path):
    """mmcv.imread(path) equivalent: HxWx3 uint8 in BGR order."""
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert('RGB'), dtype=np.uint8)
    return np.ascontiguousarray(rgb[..., ::-1])


def rescale_size(h, w, scale):
    """mmcv.imrescale for a (long edge, short edge) tuple: ((new_w, new_h), scale_factor)."""
    s = min(max(scale) / max(h, w), min(scale) / min(h, w))
    return (int(w * float(s) + 0.5), int(h * float(s) + 0.5)), s


class ImagePipeline:
    """Resize -> RandomFlip -> Normalize -> Pad of an mmdet v1 pipeline config list.

    __call__(imgs, gt_bboxes=None, filenames=None) takes BGR uint8 HxWx3 numpy arrays
    (or uint8 HIP tensors) and returns (img [B, 3, H, W] f32 on `device`, img_metas,
    gt_bboxes as [4, n] device tensors or None) -- the tensors the reference's trainer
    hands to forward_train."""

    def __init__(self, img_scale=(1333, 800), keep_ratio=True, flip_ratio=0.0, mean=(123.675, 116.28, 103.53),
                 std=(58.395, 57.12, 57.375), to_rgb=True, size_divisor=32, seed=None):
        self.img_scale = tuple(img_scale)
        self.keep_ratio = keep_ratio
        self.flip_ratio = flip_ratio
        self.mean = np.asarray(mean, np.float32)
        self.std = np.asarray(std, np.float32)
        self.to_rgb = bool(to_rgb)
        self.size_divisor = size_divisor
        self.rng = np.random if seed is None else np.random.RandomState(seed)

    @classmethod
    def from_config(cls, pipeline, seed=None):
        """Build from the reference's pipeline list (LoadImageFromFile / LoadAnnotations /
        DefaultFormatBundle / Collect are the host-side steps this class's caller does)."""
        kw = {}
        for step in pipeline:
            t = step['type']
            if t == 'Resize':
                kw['img_scale'] = tuple(step['img_scale'])
                kw['keep_ratio'] = step.get('keep_ratio', True)
            elif t == 'RandomFlip':
                kw['flip_ratio'] = step.get('flip_ratio', 0.0) or 0.0
            elif t == 'Normalize':
                kw.update(mean=step['mean'], std=step['std'], to_rgb=step.get('to_rgb', True))
            elif t == 'Pad':
                kw['size_divisor'] = step.get('size_divisor', None)
            elif t not in ('LoadImageFromFile', 'LoadAnnotations', 'DefaultFormatBundle', 'Collect', 'ImageToTensor'):
                raise ValueError('unsupported pipeline step {}'.format(t))
        return cls(seed=seed, **kw)

    def _plan(self, h, w):
        if self.keep_ratio:
            (nw, nh), s = rescale_size(h, w, self.img_scale)
            return nh, nw, s
        # mmdet v1 Resize(keep_ratio=False): exact img_scale, per-axis factors
        nw, nh = self.img_scale
        return nh, nw, np.array([nw / w, nh / h, nw / w, nh / h], dtype=np.float32)

    def _pad(self, n):
        d = self.size_divisor
        return n if not d else int(math.ceil(n / d)) * d

    def __call__(self, imgs, gt_bboxes=None, filenames=None, device=None, flips=None):
        device = device or torch.device('cuda', torch.cuda.current_device())
        metas, sizes, hw, offs, fl = [], [], [], [], []
        off = 0
        for b, img in enumerate(imgs):
            h, w = int(img.shape[0]), int(img.shape[1])
            if img.ndim != 3 or img.shape[2] != 3:
                raise AssertionError('images must be HxWx3 uint8')
            nh, nw, sf = self._plan(h, w)
            flip = bool(flips[b]) if flips is not None else bool(self.flip_ratio > 0 and
                                                                 self.rng.rand() < self.flip_ratio)
            ph, pw = self._pad(nh), self._pad(nw)
            metas.append({'filename': filenames[b] if filenames else None, 'ori_shape': (h, w, 3),
                          'img_shape': (nh, nw, 3), 'pad_shape': (ph, pw, 3), 'scale_factor': sf, 'flip': flip,
                          'img_norm_cfg': {'mean': self.mean, 'std': self.std, 'to_rgb': self.to_rgb}})
            sizes.append((nh, nw))
            hw += [h, w]
            offs.append(off)
            fl.append(int(flip))
            off += h * w * 3
        out_h = max(m['pad_shape'][0] for m in metas)
        out_w = max(m['pad_shape'][1] for m in metas)
        src = torch.cat([(i if isinstance(i, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(i)))
                         .to(device=device, dtype=torch.uint8).reshape(-1) for i in imgs])
        out = torch.empty(len(imgs), 3, out_h, out_w, dtype=torch.float32, device=device)
        call('frh_image_preprocess', ptr(src), len(imgs), _lib.i64_array(offs), _lib.i32_array(hw),
             _lib.i32_array([v for s in sizes for v in s]), _lib.i32_array(fl), _lib.f32_array(self.mean),
             _lib.f32_array(self.std), int(self.to_rgb), ptr(out), out_h, out_w, stream_of(out))
        boxes = None
        if gt_bboxes is not None:
            boxes = [torch.from_numpy(transform_boxes(np.asarray(g, np.float32), m)).to(device).t().contiguous()
                     for g, m in zip(gt_bboxes, metas)]
        return out, metas, boxes


def transform_boxes(bboxes, meta):
    """mmdet v1 Resize._resize_bboxes (scale, clip to img_shape - 1) then RandomFlip's
    bbox_flip (x1' = w - x2 - 1, x2' = w - x1 - 1) on [n, 4] xyxy float32."""
    nh, nw = meta['img_shape'][:2]
    b = (bboxes * meta['scale_factor']).astype(np.float32)
    b[:, 0::2] = np.clip(b[:, 0::2], 0, nw - 1)
    b[:, 1::2] = np.clip(b[:, 1::2], 0, nh - 1)
    if meta['flip']:
        f = b.copy()
        f[:, 0] = nw - b[:, 2] - 1
        f[:, 2] = nw - b[:, 0] - 1
        b = f
    return b


class VOCDataset:
    """lib/datasets.py:26-31: mmdet v1 CocoDataset over a COCO-format json with the VOC
    classes.  Annotations: [x, y, w, h] -> [x1, y1, x1 + w - 1, y1 + h - 1]; crowd boxes go
    to bboxes_ignore; boxes with w < 1 or h < 1 are dropped; labels are 1-based in sorted
    category-id order (CocoDataset._parse_ann_info).  __getitem__ gives the host-side
    record; `collate` runs the device pipeline over a list of records."""
    CLASSES = VOC_CLASSES

    def __init__(self, ann_file, img_prefix, pipeline=None, test_mode=False, seed=None):
        ann = json.load(open(ann_file))
        self.img_prefix = img_prefix
        self.cat_ids = sorted(c['id'] for c in ann['categories'])
        self.cat2label = {c: i + 1 for i, c in enumerate(self.cat_ids)}
        self.img_infos = list(ann['images'])  # COCO.getImgIds(): file order
        self._anns = {}
        for a in ann.get('annotations', []):
            self._anns.setdefault(a['image_id'], []).append(a)
        if not test_mode:  # CocoDataset._filter_imgs: images with annotations and min side >= 32
            self.img_infos = [i for i in self.img_infos
                              if i['id'] in self._anns and min(i['width'], i['height']) >= 32]
        self.pipeline = ImagePipeline.from_config(pipeline, seed) if pipeline is not None else ImagePipeline()

    def __len__(self):
        return len(self.img_infos)

    def ann_info(self, idx):
        bboxes, labels, ignore = [], [], []
        for a in self._anns.get(self.img_infos[idx]['id'], []):
            if a.get('ignore', False):
                continue
            x1, y1, w, h = a['bbox']
            if a.get('area', w * h) <= 0 or w < 1 or h < 1:
                continue
            box = [x1, y1, x1 + w - 1, y1 + h - 1]
            if a.get('iscrowd', False):
                ignore.append(box)
            else:
                bboxes.append(box)
                labels.append(self.cat2label[a['category_id']])
        return {'bboxes': np.array(bboxes, np.float32).reshape(-1, 4), 'labels': np.array(labels, np.int64),
                'bboxes_ignore': np.array(ignore, np.float32).reshape(-1, 4)}

    def __getitem__(self, idx):
        info = self.img_infos[idx]
        fn = osp.join(self.img_prefix, info['file_name'])
        a = self.ann_info(idx)
        return {'img': load_image(fn), 'filename': fn, 'gt_bboxes': a['bboxes'], 'gt_labels': a['labels']}

    def collate(self, records, device=None):
        """The batch of trainer.py:102-108: {'img', 'img_meta', 'gt_bboxes' ([4, n] each), 'gt_labels'}."""
        img, metas, boxes = self.pipeline([r['img'] for r in records], [r['gt_bboxes'] for r in records],
                                          [r['filename'] for r in records], device)
        dev = img.device
        return {'img': img, 'img_meta': metas, 'gt_bboxes': boxes,
                'gt_labels': [torch.from_numpy(r['gt_labels']).to(dev) for r in records]}

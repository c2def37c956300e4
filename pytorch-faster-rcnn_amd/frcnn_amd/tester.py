"""Inference loop and COCO-results conversion of the reference tester.

Reference: `BasicTester` (`lib/tester.py:7-57`) runs `forward_test` over a dataloader and
keeps, per image, the xywh boxes scaled back to the original image
(`utils.xyxy2xywh(bbox).t() / scale_factor`), scores and categories, keyed by the image
id parsed from the file name; `test.py:74-90` flattens that into the COCO results list
(bbox rounded to 2 decimals, score to 3) that COCOeval scores.  `frcnn_amd.coco_eval`
stands in for pycocotools' COCOeval (absent here).
"""
import copy
import logging
import os.path as osp

import torch

from . import ops

from . import utils


class BasicTester:
    def __init__(self, model, train_cfg, test_cfg, device):
        self.device = device
        self.model = model
        self.train_cfg = copy.deepcopy(train_cfg)
        self.test_cfg = copy.deepcopy(test_cfg)

    def load_ckpt(self, ckpt):
        """tester.py:19-23; tensors only (weights_only=True)."""
        self.ckpt = ckpt
        if self.model is None:
            raise AssertionError('no model to load into')
        self.model.load_state_dict(torch.load(ckpt, map_location=self.device, weights_only=True))
        logging.info('loaded ckpt: %s', ckpt)

    def inference_one(self, img_data, img_metas):
        return self.model.forward_test(img_data.to(device=self.device), img_metas)

    def inference(self, dataloader):
        """tester.py:25-53.  Each batch is {'img': [B, 3, H, W] tensor, 'img_meta': [meta, ...]}."""
        self.model.eval()
        inf_res = []
        with torch.no_grad():
            for ith, batch in enumerate(dataloader):
                img_metas = batch['img_meta']
                bboxes, scores, categories = self.inference_one(batch['img'], img_metas)
                if self.device.type == 'cuda':  # forward_test synchronises (mcnms counts): a 4-byte read
                    ops.check_device_status(self.device)
                for i, meta in enumerate(img_metas):
                    res = image_result(bboxes[i], scores[i], categories[i], meta)
                    if res is None:
                        logging.warning('0 predictions for image %s', meta['filename'])
                        continue
                    inf_res.append(res)
        return inf_res


def image_result(bbox, score, category, img_meta):
    """One image's entry of tester.py:38-52.  The reference skips an image only when
    ``len(bbox) == 0`` (tester.py:46); a detector's empty result is a [4, 0] tensor, whose
    len is 4, so such an image is kept with empty bbox/score/category (it contributes no
    COCO results).  None only for a bbox with no rows at all."""
    filename = osp.basename(img_meta['filename'])
    img_w, img_h = img_meta['ori_shape'][:2]  # tester.py:43 keeps the reference's (w, h) naming
    res = {'width': img_w, 'height': img_h, 'image_id': int(filename[:-4]), 'file_name': filename}
    if len(bbox) == 0:
        return None
    res['bbox'] = utils.xyxy2xywh(bbox).t() / img_meta['scale_factor']
    res['score'] = score
    res['category'] = category
    return res


def results_to_coco(inf_res):
    """test.py:74-90: per-image results -> COCO results list."""
    out, anno_idx = [], 0
    for pred in inf_res:
        bbox = pred['bbox'].detach().cpu().tolist()
        score = pred['score'].detach().cpu().tolist()
        category = pred['category'].detach().cpu().tolist()
        for i, cur in enumerate(bbox):
            out.append({'id': anno_idx, 'image_id': pred['image_id'], 'file_name': pred['file_name'],
                        'bbox': [round(x, 2) for x in cur], 'score': round(score[i], 3),
                        'category_id': int(category[i])})
            anno_idx += 1
    return out

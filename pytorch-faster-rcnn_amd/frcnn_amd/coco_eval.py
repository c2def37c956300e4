"""COCO bbox evaluation (AP@[.5:.95], AP50, AP75, per-area AP, AR) in numpy.

The reference scores detections with pycocotools' COCOeval (`test.py:91-97`,
`scripts/det_calc_mAP:14-20`; README's VOC07 numbers are its AP / AP50).  pycocotools is
not installed here, so this is a restatement of its published bbox algorithm
(cocoapi PythonAPI/pycocotools/cocoeval.py, evaluateImg / accumulate / summarize):

* per (image, category): detections sorted by score (stable), cut to maxDet; ground
  truths sorted with non-ignored first; IoU of xywh boxes without +1, a crowd ground truth
  scored as intersection / detection area;
* per IoU threshold 0.50:0.05:0.95, greedy matching in score order to the best-IoU
  unmatched ground truth (crowd ground truths match repeatedly; a match to an ignored
  ground truth ignores the detection; a match is recorded as the ground truth's id, so
  as in pycocotools a ground truth with id 0 never counts); detections outside the area
  range unmatched and ignored;
* accumulate: detections of all images merged by score (mergesort), cumulative TP/FP,
  precision made monotone from the right, sampled at 101 recall points
  (searchsorted 'left'; points past the last recall score 0);
* summarize: mean over the entries > -1.

Parity with pycocotools itself is unpinned (the library is absent); the tests pin the
algorithm on hand-computed cases.  Inputs are the COCO json structures: ground truth
{'images', 'annotations', 'categories'} and a results list of {'image_id', 'category_id',
'bbox', 'score'} (what `frcnn_amd.tester.results_to_coco` writes, as `test.py:75-90`).
"""
from collections import defaultdict

import numpy as np

IOU_THRS = np.linspace(0.5, 0.95, int(np.round((0.95 - 0.5) / 0.05)) + 1, endpoint=True)
REC_THRS = np.linspace(0.0, 1.0, int(np.round((1.0 - 0.0) / 0.01)) + 1, endpoint=True)
MAX_DETS = (1, 10, 100)
AREA_RNG = {'all': (0 ** 2, 1e5 ** 2), 'small': (0 ** 2, 32 ** 2), 'medium': (32 ** 2, 96 ** 2),
            'large': (96 ** 2, 1e5 ** 2)}
AREA_NAMES = ('all', 'small', 'medium', 'large')


def box_iou_xywh(d, g, crowd):
    """pycocotools maskUtils.iou for boxes: [D, 4] x [G, 4] xywh -> [D, G]."""
    d = np.asarray(d, np.float64).reshape(-1, 4)
    g = np.asarray(g, np.float64).reshape(-1, 4)
    if len(d) == 0 or len(g) == 0:
        return np.zeros((len(d), len(g)))
    dx2, dy2 = d[:, 0] + d[:, 2], d[:, 1] + d[:, 3]
    gx2, gy2 = g[:, 0] + g[:, 2], g[:, 1] + g[:, 3]
    iw = np.minimum(dx2[:, None], gx2[None]) - np.maximum(d[:, 0][:, None], g[:, 0][None])
    ih = np.minimum(dy2[:, None], gy2[None]) - np.maximum(d[:, 1][:, None], g[:, 1][None])
    inter = np.where((iw > 0) & (ih > 0), iw * ih, 0.0)
    da, ga = d[:, 2] * d[:, 3], g[:, 2] * g[:, 3]
    union = np.where(np.asarray(crowd, bool)[None], da[:, None], da[:, None] + ga[None] - inter)
    return np.where(union > 0, inter / np.where(union > 0, union, 1.0), 0.0)


class COCOEval:
    def __init__(self, gt, dt):
        self.gt = gt
        self.img_ids = sorted(im['id'] for im in gt['images'])
        self.cat_ids = sorted(c['id'] for c in gt['categories'])
        self._gts, self._dts = defaultdict(list), defaultdict(list)
        for a in gt['annotations']:
            a = dict(a)
            a.setdefault('iscrowd', 0)
            a.setdefault('area', a['bbox'][2] * a['bbox'][3])
            a['ignore'] = int(bool(a['iscrowd']))  # cocoeval _prepare: ignore is overwritten by iscrowd
            self._gts[a['image_id'], a['category_id']].append(a)
        for d in dt:
            d = dict(d)
            d['area'] = d['bbox'][2] * d['bbox'][3]
            self._dts[d['image_id'], d['category_id']].append(d)

    def evaluate_img(self, img, cat, arng, max_det):
        gts, dts = self._gts.get((img, cat), []), self._dts.get((img, cat), [])
        if not gts and not dts:
            return None
        g_ign = np.array([1 if (g['ignore'] or g['area'] < arng[0] or g['area'] > arng[1]) else 0 for g in gts],
                         np.int64)
        gind = np.argsort(g_ign, kind='mergesort')
        gts = [gts[i] for i in gind]
        g_ign = g_ign[gind]
        dind = np.argsort([-d['score'] for d in dts], kind='mergesort')
        dts = [dts[i] for i in dind[:max_det]]
        crowd = [int(g['iscrowd']) for g in gts]
        ious = box_iou_xywh([d['bbox'] for d in dts], [g['bbox'] for g in gts], crowd)
        T, G, D = len(IOU_THRS), len(gts), len(dts)
        gtm, dtm = np.zeros((T, G)), np.zeros((T, D))
        dt_ig = np.zeros((T, D))
        if G and D:
            for ti, t in enumerate(IOU_THRS):
                for di in range(D):
                    iou, m = min(t, 1 - 1e-10), -1
                    for gi in range(G):
                        if gtm[ti, gi] > 0 and not crowd[gi]:
                            continue
                        if m > -1 and g_ign[m] == 0 and g_ign[gi] == 1:
                            break
                        if ious[di, gi] < iou:
                            continue
                        iou, m = ious[di, gi], gi
                    if m == -1:
                        continue
                    dt_ig[ti, di] = g_ign[m]
                    dtm[ti, di] = gts[m]['id']  # pycocotools keeps the gt id: a gt with id 0 never 'matches'
                    gtm[ti, m] = 1
        d_out = np.array([d['area'] < arng[0] or d['area'] > arng[1] for d in dts], bool).reshape(1, D)
        dt_ig = np.logical_or(dt_ig, np.logical_and(dtm == 0, np.repeat(d_out, T, 0)))
        return {'scores': np.array([d['score'] for d in dts]), 'dtm': dtm, 'dt_ig': dt_ig, 'g_ign': g_ign}

    def run(self):
        """precision [T, R, K, A, M] and recall [T, K, A, M] (-1 where undefined)."""
        T, R, K, A, M = len(IOU_THRS), len(REC_THRS), len(self.cat_ids), len(AREA_NAMES), len(MAX_DETS)
        precision = -np.ones((T, R, K, A, M))
        recall = -np.ones((T, K, A, M))
        for k, cat in enumerate(self.cat_ids):
            for a, an in enumerate(AREA_NAMES):
                evs = [self.evaluate_img(img, cat, AREA_RNG[an], MAX_DETS[-1]) for img in self.img_ids]
                evs = [e for e in evs if e is not None]
                if not evs:
                    continue
                for m, md in enumerate(MAX_DETS):
                    scores = np.concatenate([e['scores'][:md] for e in evs])
                    inds = np.argsort(-scores, kind='mergesort')
                    dtm = np.concatenate([e['dtm'][:, :md] for e in evs], 1)[:, inds]
                    dt_ig = np.concatenate([e['dt_ig'][:, :md] for e in evs], 1)[:, inds]
                    npig = int(sum((e['g_ign'] == 0).sum() for e in evs))
                    if npig == 0:
                        continue
                    tps = np.logical_and(dtm, np.logical_not(dt_ig))
                    fps = np.logical_and(np.logical_not(dtm), np.logical_not(dt_ig))
                    tp_sum = np.cumsum(tps, 1).astype(np.float64)
                    fp_sum = np.cumsum(fps, 1).astype(np.float64)
                    for t in range(T):
                        tp, fp = tp_sum[t], fp_sum[t]
                        nd = len(tp)
                        rc = tp / npig
                        pr = tp / (fp + tp + np.spacing(1))
                        recall[t, k, a, m] = rc[-1] if nd else 0
                        pr = pr.tolist()
                        for i in range(nd - 1, 0, -1):
                            if pr[i] > pr[i - 1]:
                                pr[i - 1] = pr[i]
                        q = np.zeros(R)
                        idx = np.searchsorted(rc, REC_THRS, side='left')
                        for ri, pi in enumerate(idx):
                            if pi < nd:
                                q[ri] = pr[pi]
                        precision[t, :, k, a, m] = q
        self.precision, self.recall = precision, recall
        return precision, recall

    def summarize(self):
        if not hasattr(self, 'precision'):
            self.run()
        p, r = self.precision, self.recall

        def ap(iou=None, area='all', md=100):
            s = p[:, :, :, AREA_NAMES.index(area), MAX_DETS.index(md)]
            if iou is not None:
                s = s[np.where(np.isclose(IOU_THRS, iou))[0]]
            s = s[s > -1]
            return float(s.mean()) if s.size else -1.0

        def ar(area='all', md=100):
            s = r[:, :, AREA_NAMES.index(area), MAX_DETS.index(md)]
            s = s[s > -1]
            return float(s.mean()) if s.size else -1.0

        self.stats = {'AP': ap(), 'AP50': ap(0.5), 'AP75': ap(0.75), 'APs': ap(area='small'),
                      'APm': ap(area='medium'), 'APl': ap(area='large'), 'AR1': ar(md=1), 'AR10': ar(md=10),
                      'AR100': ar(), 'ARs': ar('small'), 'ARm': ar('medium'), 'ARl': ar('large')}
        return self.stats


def evaluate(gt, results):
    """gt: COCO ground-truth dict; results: COCO results list -> summary dict (AP, AP50, ...)."""
    return COCOEval(gt, results).summarize()

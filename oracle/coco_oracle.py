"""TEST INFRASTRUCTURE — independent restatement of pycocotools' bbox COCOeval.

Only tests/ and tests/golden/gen_golden.py use this module, as the checker for the
product evaluator (pytorch-faster-rcnn_amd/frcnn_amd/coco_eval.py).  The reference
scores detections with pycocotools (test.py:91-97: COCO(ann_file).loadRes(json),
COCOeval(gt, dt, 'bbox').evaluate/accumulate/summarize); pycocotools is absent from
this image, so its published algorithm (cocoapi PythonAPI/pycocotools/cocoeval.py and
maskApi.c bbIou) is restated here a second time, in plain Python scalar loops and
written apart from the numpy product version, so the two can check each other:

  loadRes      every result gets id = index + 1 and area = w * h;
  _prepare     gt ignore flag := iscrowd;
  bbIou        double precision, no +1, crowd gt -> intersection / detection area;
  evaluateImg  gts with ignore flag (crowd or area outside the range) sorted last
               (stable), detections by score (stable) cut to maxDet; per IoU threshold
               greedy matching; dtMatches / gtMatches hold the partner's *id* (so a
               ground truth with id 0 never counts as matched, as in pycocotools);
  accumulate   per (category, area, maxDet) over all images, stable merge by score,
               cumulative TP/FP, precision envelope, 101 recall points;
  summarize    the 12 standard stats, mean over entries > -1.

Parity with pycocotools itself is unpinned (it is not installed); this restatement
and the product's are pinned together on hand-worked cases (tests/test_coco_eval.py).
"""
IOU_THRS = [0.5 + 0.05 * i for i in range(10)]
REC_THRS = [0.01 * i for i in range(101)]
MAX_DETS = [1, 10, 100]
AREAS = [('all', 0.0, 1e10), ('small', 0.0, 1024.0), ('medium', 1024.0, 9216.0), ('large', 9216.0, 1e10)]
EPS = 2.220446049250313e-16  # np.spacing(1)


def _iou(d, g, crowd):
    w = min(d[0] + d[2], g[0] + g[2]) - max(d[0], g[0])
    if w <= 0:
        return 0.0
    h = min(d[1] + d[3], g[1] + g[3]) - max(d[1], g[1])
    if h <= 0:
        return 0.0
    inter = w * h
    union = d[2] * d[3] if crowd else d[2] * d[3] + g[2] * g[3] - inter
    return inter / union if union > 0 else 0.0


def _stable_sort(items, key):
    order = sorted(range(len(items)), key=lambda n: (key(items[n]), n))
    return [items[n] for n in order]


def _eval_img(gts, dts, lo, hi, max_det):
    if not gts and not dts:
        return None
    gig = {id(g): 1 if (g['iscrowd'] or g['area'] < lo or g['area'] > hi) else 0 for g in gts}
    gts = _stable_sort(gts, lambda g: gig[id(g)])
    ig = [gig[id(g)] for g in gts]
    dts = _stable_sort(dts, lambda d: -d['score'])[:max_det]
    T = len(IOU_THRS)
    gtm = [[0] * len(gts) for _ in range(T)]
    dtm = [[0] * len(dts) for _ in range(T)]
    dig = [[0] * len(dts) for _ in range(T)]
    for t, thr in enumerate(IOU_THRS):
        for di, d in enumerate(dts):
            best, m = min(thr, 1 - 1e-10), -1
            for gi, g in enumerate(gts):
                if gtm[t][gi] > 0 and not g['iscrowd']:
                    continue
                if m > -1 and ig[m] == 0 and ig[gi] == 1:
                    break
                v = _iou(d['bbox'], g['bbox'], g['iscrowd'])
                if v < best:
                    continue
                best, m = v, gi
            if m == -1:
                continue
            dig[t][di] = ig[m]
            dtm[t][di] = gts[m]['id']
            gtm[t][m] = d['id']
    for t in range(T):
        for di, d in enumerate(dts):
            if dtm[t][di] == 0 and (d['area'] < lo or d['area'] > hi):
                dig[t][di] = 1
    return {'scores': [d['score'] for d in dts], 'dtm': dtm, 'dig': dig, 'gig': ig}


def _accumulate(evs, max_det):
    """-> (precision[T][R], recall[T]) for one (category, area, maxDet), or None."""
    rows = []  # (score, image order, position, e)
    for n, e in enumerate(evs):
        for p in range(min(max_det, len(e['scores']))):
            rows.append((e['scores'][p], n, p, e))
    rows = _stable_sort(rows, lambda r: -r[0])
    npig = sum(1 for e in evs for v in e['gig'] if v == 0)
    if npig == 0:
        return None
    prec, rec = [], []
    for t in range(len(IOU_THRS)):
        tp = fp = 0
        rc, pr = [], []
        for _, _, p, e in rows:
            matched, ignored = e['dtm'][t][p] != 0, e['dig'][t][p] != 0
            if ignored:
                pass
            elif matched:
                tp += 1
            else:
                fp += 1
            rc.append(tp / npig)
            pr.append(tp / (fp + tp + EPS))
        rec.append(rc[-1] if rows else 0.0)
        for i in range(len(pr) - 1, 0, -1):
            if pr[i] > pr[i - 1]:
                pr[i - 1] = pr[i]
        q = []
        for r in REC_THRS:
            # first position whose recall >= r (searchsorted 'left'); none -> 0
            pos = next((i for i, v in enumerate(rc) if v >= r), None)
            q.append(pr[pos] if pos is not None else 0.0)
        prec.append(q)
    return prec, rec


def evaluate(gt, results):
    """gt: COCO ground-truth dict; results: list of {'image_id','category_id','bbox','score'}.
    Returns the 12 summary stats (AP, AP50, AP75, APs, APm, APl, AR1, AR10, AR100, ARs,
    ARm, ARl)."""
    img_ids = sorted(im['id'] for im in gt['images'])
    cat_ids = sorted(c['id'] for c in gt['categories'])
    gts, dts = {}, {}
    for a in gt['annotations']:
        b = [float(v) for v in a['bbox']]
        rec = {'id': a['id'], 'bbox': b, 'iscrowd': int(a.get('iscrowd', 0)),
               'area': float(a['area']) if 'area' in a else b[2] * b[3]}
        gts.setdefault((a['image_id'], a['category_id']), []).append(rec)
    for n, r in enumerate(results):
        b = [float(v) for v in r['bbox']]
        rec = {'id': n + 1, 'bbox': b, 'score': float(r['score']), 'area': b[2] * b[3]}
        dts.setdefault((r['image_id'], r['category_id']), []).append(rec)
    table = {}  # (k, a, m) -> (precision, recall)
    for k, cat in enumerate(cat_ids):
        for a, (_, lo, hi) in enumerate(AREAS):
            evs = [_eval_img(gts.get((i, cat), []), dts.get((i, cat), []), lo, hi, MAX_DETS[-1]) for i in img_ids]
            evs = [e for e in evs if e is not None]
            if not evs:
                continue
            for m, md in enumerate(MAX_DETS):
                r = _accumulate(evs, md)
                if r is not None:
                    table[k, a, m] = r

    def mean(vals):
        vals = [v for v in vals if v > -1]
        return sum(vals) / len(vals) if vals else -1.0

    def ap(t_sel, a, m):
        vals = []
        for (k, aa, mm), (prec, _) in table.items():
            if aa == a and mm == m:
                for t in t_sel:
                    vals.extend(prec[t])
        # undefined (category, area) cells count as -1 in pycocotools and are dropped by mean
        return mean(vals)

    def ar(a, m):
        vals = []
        for (k, aa, mm), (_, rec) in table.items():
            if aa == a and mm == m:
                vals.extend(rec)
        return mean(vals)

    T = range(len(IOU_THRS))
    return {'AP': ap(T, 0, 2), 'AP50': ap([0], 0, 2), 'AP75': ap([5], 0, 2), 'APs': ap(T, 1, 2),
            'APm': ap(T, 2, 2), 'APl': ap(T, 3, 2), 'AR1': ar(0, 0), 'AR10': ar(0, 1), 'AR100': ar(0, 2),
            'ARs': ar(1, 2), 'ARm': ar(2, 2), 'ARl': ar(3, 2)}

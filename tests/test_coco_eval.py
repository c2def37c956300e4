"""COCO bbox evaluator (frcnn_amd.coco_eval) and the tester's results conversion.

The reference scores with pycocotools' COCOeval (test.py:91-97); pycocotools is absent
here, so parity with it is unpinned and these cases pin the restated algorithm on values
computed by hand (101-point interpolated precision, greedy matching, crowd/area/maxDet
rules).  The conversion tests follow lib/tester.py:38-52 and test.py:74-90."""
import numpy as np
import pytest
import torch

from frcnn_amd import coco_eval, tester


def _gt(boxes, cats=(1,), crowd=None, img_of=None):
    anns = []
    for i, (b, c) in enumerate(boxes):
        anns.append({'id': i + 1, 'image_id': img_of[i] if img_of else 1, 'category_id': c, 'bbox': list(b),
                     'iscrowd': int(crowd[i]) if crowd else 0, 'area': b[2] * b[3]})
    imgs = sorted({a['image_id'] for a in anns} | {1})
    return {'images': [{'id': i} for i in imgs], 'annotations': anns,
            'categories': [{'id': c} for c in cats]}


def _dt(boxes, img_of=None):
    return [{'image_id': img_of[i] if img_of else 1, 'category_id': c, 'bbox': list(b), 'score': s}
            for i, (b, c, s) in enumerate(boxes)]


def test_perfect_detections():
    g = [((10, 10, 50, 40), 1), ((100, 80, 120, 130), 2), ((5, 200, 20, 20), 1)]
    gt = _gt(g, cats=(1, 2), img_of=[1, 1, 2])
    dt = _dt([(b, c, 0.9) for b, c in g], img_of=[1, 1, 2])
    s = coco_eval.evaluate(gt, dt)
    for k in ('AP', 'AP50', 'AP75', 'AR1', 'AR10', 'AR100'):
        assert s[k] == pytest.approx(1.0, abs=1e-12), k
    assert s['APs'] == pytest.approx(1.0)        # the 20x20 box
    assert s['APm'] == pytest.approx(1.0)        # 50x40
    assert s['APl'] == pytest.approx(1.0)        # 120x130


def test_interpolated_precision_by_hand():
    # scores 0.9 TP, 0.8 FP, 0.7 TP against 2 GTs: precision (1, 1/2, 2/3) -> monotone
    # (1, 2/3, 2/3); recall (1/2, 1/2, 1).  Recall points 0..0.50 (51) read 1, 0.51..1 (50) read 2/3.
    g = [((0, 0, 40, 40), 1), ((100, 100, 40, 40), 1)]
    dt = _dt([((0, 0, 40, 40), 1, 0.9), ((300, 300, 40, 40), 1, 0.8), ((100, 100, 40, 40), 1, 0.7)])
    s = coco_eval.evaluate(_gt(g), dt)
    want = (51 * 1.0 + 50 * (2.0 / 3.0)) / 101
    assert s['AP'] == pytest.approx(want, abs=1e-12)
    assert s['AP50'] == pytest.approx(want, abs=1e-12)
    assert s['AR100'] == pytest.approx(1.0)
    assert s['AR1'] == pytest.approx(0.5)


def test_iou_threshold_sweep():
    # detection shifted so IoU = 0.72: a TP at 0.50..0.70 (5 of 10 thresholds), a miss above
    gt_box = (0, 0, 100, 100)
    # x-shift d gives IoU (100-d)/(100+d) = 0.72 -> d = 28/1.72
    d = 28.0 / 1.72
    iou = coco_eval.box_iou_xywh([(d, 0, 100, 100)], [gt_box], [0])[0, 0]
    assert iou == pytest.approx(0.72, abs=1e-9)
    s = coco_eval.evaluate(_gt([(gt_box, 1)]), _dt([((d, 0, 100, 100), 1, 0.5)]))
    assert s['AP50'] == pytest.approx(1.0)
    assert s['AP75'] == pytest.approx(0.0)
    assert s['AP'] == pytest.approx(0.5)
    assert s['AR100'] == pytest.approx(0.5)


def test_greedy_matching_prefers_highest_score():
    # two detections on one GT: the higher score matches, the other is an FP
    g = [((0, 0, 50, 50), 1)]
    dt = _dt([((0, 0, 50, 50), 1, 0.3), ((1, 1, 50, 50), 1, 0.9)])
    ev = coco_eval.COCOEval(_gt(g), dt)
    e = ev.evaluate_img(1, 1, coco_eval.AREA_RNG['all'], 100)
    np.testing.assert_array_equal(e['scores'], [0.9, 0.3])
    assert e['dtm'][0].tolist() == [1, 0]     # at IoU 0.5 the 0.9 detection takes the GT
    s = ev.summarize()
    assert s['AP50'] == pytest.approx(1.0)    # precision 1 at recall 1 reached first


def test_crowd_ground_truth_ignores_detections():
    # a detection inside a crowd region is neither TP nor FP; the crowd GT is not counted
    g = [((0, 0, 200, 200), 1), ((300, 300, 40, 40), 1)]
    dt = _dt([((10, 10, 50, 50), 1, 0.95), ((300, 300, 40, 40), 1, 0.5)])
    s = coco_eval.evaluate(_gt(g, crowd=[1, 0]), dt)
    assert s['AP'] == pytest.approx(1.0)
    # crowd IoU = intersection / detection area
    assert coco_eval.box_iou_xywh([(10, 10, 50, 50)], [(0, 0, 200, 200)], [1])[0, 0] == pytest.approx(1.0)


def test_area_ranges_and_missing_categories():
    g = [((0, 0, 20, 20), 1)]                 # small only
    dt = _dt([((0, 0, 20, 20), 1, 0.9), ((50, 50, 10, 10), 2, 0.9)])
    s = coco_eval.evaluate(_gt(g, cats=(1, 2)), dt)
    assert s['APs'] == pytest.approx(1.0)
    assert s['APm'] == -1.0 and s['APl'] == -1.0   # no GT in range: undefined, skipped
    assert s['AP'] == pytest.approx(1.0)           # category 2 has no GT: excluded


def test_max_dets_cut():
    g = [((0, 0, 40, 40), 1), ((100, 0, 40, 40), 1), ((200, 0, 40, 40), 1)]
    dt = _dt([((0, 0, 40, 40), 1, 0.9), ((100, 0, 40, 40), 1, 0.8), ((200, 0, 40, 40), 1, 0.7)])
    s = coco_eval.evaluate(_gt(g), dt)
    assert s['AR1'] == pytest.approx(1 / 3)
    assert s['AR10'] == pytest.approx(1.0)


def test_empty_results():
    s = coco_eval.evaluate(_gt([((0, 0, 40, 40), 1)]), [])
    assert s['AP'] == 0.0 and s['AR100'] == 0.0


def test_results_conversion_matches_reference_format():
    bbox = torch.tensor([[10., 20., 59., 69.], [0., 0., 9.5, 19.25]]).t()   # [4, n] xyxy
    meta = {'filename': '/data/VOC/000123.jpg', 'ori_shape': (500, 375, 3), 'scale_factor': 2.0}
    res = tester.image_result(bbox, torch.tensor([0.91234, 0.5]), torch.tensor([3, 7]), meta)
    assert res['image_id'] == 123 and res['file_name'] == '000123.jpg'
    assert (res['width'], res['height']) == (500, 375)
    out = tester.results_to_coco([res])
    assert out[0] == {'id': 0, 'image_id': 123, 'file_name': '000123.jpg', 'bbox': [5.0, 10.0, 25.0, 25.0],
                      'score': 0.912, 'category_id': 3}
    assert out[1]['bbox'] == [0.0, 0.0, 5.25, 10.12]   # 10.125 -> 10.12: Python round, half-even
    assert out[1]['id'] == 1
    empty = tester.image_result(torch.zeros(4, 0), torch.zeros(0), torch.zeros(0), meta)
    assert empty['bbox'].shape == (0, 4) and tester.results_to_coco([empty]) == []  # kept, as tester.py:46
    assert tester.image_result(torch.zeros(0, 4), torch.zeros(0), torch.zeros(0), meta) is None
    # converted results score themselves perfectly against the same boxes as ground truth
    gt = {'images': [{'id': 123}], 'categories': [{'id': 3}, {'id': 7}],
          'annotations': [{'id': i + 1, 'image_id': 123, 'category_id': o['category_id'], 'bbox': o['bbox'],
                           'iscrowd': 0, 'area': o['bbox'][2] * o['bbox'][3]} for i, o in enumerate(out)]}
    assert coco_eval.evaluate(gt, out)['AP'] == pytest.approx(1.0)


def test_tester_inference_loop():
    class Model(torch.nn.Module):
        def forward_test(self, img, metas):
            b = torch.tensor([[0., 0., 9., 9.]]).t()
            return [b] * len(metas), [torch.tensor([0.8])] * len(metas), [torch.tensor([1])] * len(metas)

    t = tester.BasicTester(Model(), {}, {}, torch.device('cpu'))
    metas = [{'filename': '000001.jpg', 'ori_shape': (10, 10, 3), 'scale_factor': 1.0},
             {'filename': '000002.jpg', 'ori_shape': (10, 10, 3), 'scale_factor': 1.0}]
    res = t.inference([{'img': torch.zeros(2, 3, 32, 32), 'img_meta': metas}])
    assert [r['image_id'] for r in res] == [1, 2]
    assert res[0]['bbox'].tolist() == [[0.0, 0.0, 10.0, 10.0]]


# ---------------------------------------------------------------- product evaluator vs the oracle restatement
import coco_oracle  # noqa: E402


def _random_case(seed, n_img=6, n_cat=4, crowd_p=0.1):
    rng = np.random.default_rng(seed)
    anns, dts, aid = [], [], 1
    for img in range(1, n_img + 1):
        for _ in range(rng.integers(0, 12)):
            w, h = rng.uniform(4, 200, 2)
            box = [float(v) for v in (rng.uniform(0, 400), rng.uniform(0, 300), w, h)]
            cat = int(rng.integers(1, n_cat + 1))
            anns.append({'id': aid, 'image_id': img, 'category_id': cat, 'bbox': box,
                         'iscrowd': int(rng.random() < crowd_p), 'area': box[2] * box[3]})
            aid += 1
            for _ in range(rng.integers(0, 3)):  # jittered detections of this gt, some with the wrong class
                j = rng.normal(0, 0.15, 4) * [w, h, w, h]
                dts.append({'image_id': img, 'category_id': cat if rng.random() < 0.8 else int(rng.integers(1, n_cat + 1)),
                            'bbox': [round(float(v), 2) for v in np.add(box, j).clip(0.5)],
                            'score': round(float(rng.random()), 3)})
        for _ in range(rng.integers(0, 8)):  # background false positives
            w, h = rng.uniform(4, 150, 2)
            dts.append({'image_id': img, 'category_id': int(rng.integers(1, n_cat + 1)),
                        'bbox': [round(float(v), 2) for v in (rng.uniform(0, 400), rng.uniform(0, 300), w, h)],
                        'score': round(float(rng.random()), 3)})
    gt = {'images': [{'id': i} for i in range(1, n_img + 1)], 'annotations': anns,
          'categories': [{'id': c} for c in range(1, n_cat + 1)]}
    return gt, dts


@pytest.mark.parametrize('seed', range(6))
def test_evaluator_matches_oracle_restatement(seed):
    """frcnn_amd.coco_eval (numpy) == oracle/coco_oracle.py (scalar loops, written apart) on
    random multi-image, multi-class cases with crowds, all area ranges, ties in score
    (3-decimal rounding) and > 100 detections per image in one case."""
    gt, dts = _random_case(seed, n_img=3 if seed == 5 else 6)
    if seed == 5:
        dts = dts * 12  # > maxDet 100 per image: the cut and the stable order matter
    a, b = coco_eval.evaluate(gt, dts), coco_oracle.evaluate(gt, dts)
    assert a.keys() == b.keys()
    for k in a:
        assert a[k] == pytest.approx(b[k], abs=1e-12), k


def test_evaluator_gt_id_zero_never_matches():
    """pycocotools records a match as the gt's id: a gt annotated with id 0 is consumed by
    its detection but the detection still counts as a false positive."""
    gt = {'images': [{'id': 1}], 'categories': [{'id': 1}],
          'annotations': [{'id': 0, 'image_id': 1, 'category_id': 1, 'bbox': [0, 0, 40, 40], 'iscrowd': 0,
                           'area': 1600.0}]}
    dt = [{'image_id': 1, 'category_id': 1, 'bbox': [0, 0, 40, 40], 'score': 0.9}]
    assert coco_eval.evaluate(gt, dt)['AP'] == 0.0 == coco_oracle.evaluate(gt, dt)['AP']


@pytest.mark.parametrize('case', ['perfect', 'interp', 'crowd', 'maxdet'])
def test_hand_cases_on_oracle(case):
    """The hand-worked cases above, on the oracle restatement too."""
    if case == 'perfect':
        g = [((10, 10, 50, 40), 1), ((100, 80, 120, 130), 2), ((5, 200, 20, 20), 1)]
        s = coco_oracle.evaluate(_gt(g, cats=(1, 2), img_of=[1, 1, 2]), _dt([(b, c, 0.9) for b, c in g], [1, 1, 2]))
        assert s['AP'] == pytest.approx(1.0) and s['APs'] == pytest.approx(1.0)
    elif case == 'interp':
        g = [((0, 0, 40, 40), 1), ((100, 100, 40, 40), 1)]
        dt = _dt([((0, 0, 40, 40), 1, 0.9), ((300, 300, 40, 40), 1, 0.8), ((100, 100, 40, 40), 1, 0.7)])
        assert coco_oracle.evaluate(_gt(g), dt)['AP'] == pytest.approx((51 + 50 * 2 / 3) / 101, abs=1e-12)
    elif case == 'crowd':
        g = [((0, 0, 200, 200), 1), ((300, 300, 40, 40), 1)]
        dt = _dt([((10, 10, 50, 50), 1, 0.95), ((300, 300, 40, 40), 1, 0.5)])
        assert coco_oracle.evaluate(_gt(g, crowd=[1, 0]), dt)['AP'] == pytest.approx(1.0)
    else:
        g = [((0, 0, 40, 40), 1), ((100, 0, 40, 40), 1), ((200, 0, 40, 40), 1)]
        dt = _dt([((0, 0, 40, 40), 1, 0.9), ((100, 0, 40, 40), 1, 0.8), ((200, 0, 40, 40), 1, 0.7)])
        s = coco_oracle.evaluate(_gt(g), dt)
        assert s['AR1'] == pytest.approx(1 / 3) and s['AR10'] == pytest.approx(1.0)


def test_eval_fixture_from_reference_conversion(golden_dir=None):
    """f3 pinned on the reference: tests/golden/eval.json holds the COCO results the
    reference's own BasicTester.inference (lib/tester.py:25-57) + test.py:75-90 produced for
    the fixed detections of inputs.eval_case (gen_golden.gen_eval).  The product tester must
    write the identical json, and the product evaluator must reproduce the fixture's summary
    (computed by the oracle restatement of COCOeval)."""
    import json
    import os
    import inputs
    fx = json.load(open(os.path.join(os.path.dirname(inputs.__file__), 'eval.json')))
    images, gt = inputs.eval_case()
    assert gt == fx['gt']

    class Model(torch.nn.Module):
        def forward_test(self, img, metas):
            b, s, l = images[int(img[0, 0, 0, 0])][1:]
            return [torch.from_numpy(b)], [torch.from_numpy(s)], [torch.from_numpy(l)]

    t = tester.BasicTester(Model(), {}, {}, torch.device('cpu'))
    res = t.inference([{'img': torch.full((1, 3, 8, 8), float(i)), 'img_meta': [images[i][0]]}
                       for i in range(len(images))])
    assert [{k: r[k] for k in ('width', 'height', 'image_id', 'file_name')} for r in res] == fx['image_results']
    out = tester.results_to_coco(res)
    assert out == fx['results']
    s = coco_eval.evaluate(gt, out)
    for k, v in fx['summary'].items():
        assert s[k] == pytest.approx(v, abs=1e-12), k
    assert 0.2 < s['AP50'] < 0.8 and s['AP'] < s['AP50']

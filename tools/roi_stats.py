"""RoI window-size statistics of the bench workload (cfg2, 2 images), computed on the CPU.

    python tools/roi_stats.py [--save rois.npy]

Runs the cfg2 model's backbone/RPN on the host with the bench's seeds, then the
oracle's proposal + bbox_target restatement (test infrastructure), and prints the
FPN level histogram and the per-RoI tap-window sizes that decide which RoIAlign
path (LDS-staged / gather) a RoI takes."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pytorch-faster-rcnn_amd'), os.path.join(REPO, 'oracle'),
                os.path.join(REPO, 'tests', 'golden')]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--save')
    args = ap.parse_args()
    import bench
    import oracle
    import pipeline
    model, cfg = bench.make_model(torch.device('cpu'), 0)
    imgs, boxes, labels, _ = bench.make_batch(torch.device('cpu'), 2, 0)
    tc = cfg.train_cfg
    with torch.no_grad():
        feats = model.extract_feat(imgs)
        head = model.rpn_head
        co, ro = head(feats)
    grids = [tuple(c.shape[-2:]) for c in co]
    lv_anc, _ = pipeline._anchors(head, grids)
    pc = tc.rpn_proposal
    sc, rh = tc.rcnn[0], model.rcnn_head[0]
    allr = []
    for i in range(2):
        b, _ = oracle.rpn_predict_single_image([c[i].numpy() for c in co], [r[i].numpy() for r in ro], lv_anc,
                                               (600, 1000), 0, pc.pre_nms, pc.post_nms, pc.max_num, pc.nms_iou,
                                               head.target_means, head.target_stds)
        out = oracle.bbox_target(b, boxes[i].numpy(), labels[i].numpy(),
                                 (sc.assigner.pos_iou, sc.assigner.neg_iou, sc.assigner.min_pos_iou),
                                 (sc.sampler.max_num, sc.sampler.pos_num), rh.target_means, rh.target_stds)
        allr.append(np.concatenate([np.full((1, out[0].shape[1]), i, np.float32), out[0]], 0).T)
    r5 = np.concatenate(allr, 0)
    if args.save:
        np.save(args.save, r5)
    lv = oracle.roi_level_map(r5, 56.0, 4)
    print('K', len(r5), 'levels', np.bincount(lv, minlength=4).tolist())
    s = np.array([1 / 4, 1 / 8, 1 / 16, 1 / 32])[lv]
    w = np.maximum(r5[:, 3] * s - r5[:, 1] * s, 1)
    h = np.maximum(r5[:, 4] * s - r5[:, 2] * s, 1)
    win = (np.ceil(w) + 2) * (np.ceil(h) + 2)
    print('window cells p10/50/75/90/99/max', np.percentile(win, [10, 50, 75, 90, 99, 100]).round(0).tolist())
    print('frac >256', float((win > 256).mean()), 'frac >1024', float((win > 1024).mean()))
    print('w p10/50/90/max', np.percentile(w, [10, 50, 90, 100]).round(1).tolist(),
          'h', np.percentile(h, [10, 50, 90, 100]).round(1).tolist())


if __name__ == '__main__':
    main()

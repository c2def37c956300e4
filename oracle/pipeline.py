"""TEST INFRASTRUCTURE — the reference's CPU forward+loss path, restated.

Used only by bench.py's cpu_baseline leg (and tests).  Mirrors
CascadeRCNN.forward_train (lib/detectors/cascade_rcnn.py:90-154) on the host:
the model's convolutions / FC layers / losses run as torch CPU ops, and every
detection primitive runs per image through this oracle's C restatement
(anchor_target lib/anchor.py:11-76, RPN proposals lib/heads/rpn_head.py:68-120,
bbox_target lib/bbox.py:6-82, BasicRoIExtractor lib/region.py:280-296),
i.e. the reference's own per-image Python loop structure.
"""
import numpy as np
import torch

import oracle


def _anchors(head, grids):
    lv = [oracle.anchor_grid(s, head.anchor_scales, head.anchor_ratios, s, g, head.anchor_center_lt)
          for s, g in zip(head.anchor_strides, grids)]
    return lv, np.concatenate([a.reshape(4, -1) for a in lv], 1)


def _in_mask(head, flat, grids, img_size, border):
    ingrid = np.concatenate([oracle.inside_grid_mask(head.num_anchors, img_size, g, s)
                             for g, s in zip(grids, head.anchor_strides)]).astype(bool)
    return ingrid & oracle.inside_anchor_mask(flat, img_size, border)


def forward_train_cpu(model, cfg, imgs, gt_bboxes, gt_labels, img_metas, sampler_hook=None):
    """sampler_hook (tests): callable(stage, image, labels) -> sampled labels replacing the numpy
    RandomSampler; stage 'rpn' (labels over the image's inside anchors) or 'rcnn<k>' (labels over
    the prepended [gts; proposals] rows)."""
    tc = cfg.train_cfg
    feats = model.extract_feat(imgs)
    head = model.rpn_head
    cls_outs, reg_outs = head(feats)
    grids = [tuple(c.shape[-2:]) for c in cls_outs]
    lv_anc, flat = _anchors(head, grids)
    a = tc.rpn.assigner
    s = tc.rpn.get('sampler', None)
    t_cls, t_reg, t_lab, t_par = [], [], [], []
    for i, meta in enumerate(img_metas):
        img = meta['img_shape'][:2]
        mask = _in_mask(head, flat, grids, img, tc.rpn.allowed_border)
        co = torch.cat([c[i].reshape(head.cls_channels, -1) for c in cls_outs], 1)
        ro = torch.cat([r[i].reshape(4, -1) for r in reg_outs], 1)
        gb = gt_bboxes[i].numpy()
        out = oracle.anchor_target(co.detach().numpy(), ro.detach().numpy(), head.cls_channels, flat[:, mask], mask, gb,
                                   np.ones(gb.shape[1], np.int64), (a.pos_iou, a.neg_iou, a.min_pos_iou),
                                   ((lambda lab, i=i: sampler_hook('rpn', i, lab)) if sampler_hook else
                                    (s.max_num, s.pos_num)) if s else None, head.target_means, head.target_stds)
        chosen = torch.from_numpy(out[6])
        t_cls.append(co[:, chosen])
        t_reg.append(ro[:, chosen])
        t_lab.append(torch.from_numpy(out[2]))
        t_par.append(torch.from_numpy(out[5]))
    losses = {}
    losses['rpn_cls_loss'], losses['rpn_reg_loss'] = head.calc_loss(
        torch.cat(t_cls, 1), torch.cat(t_reg, 1), torch.cat(t_lab), torch.cat(t_par, 1), tc.rpn)
    pc = tc.rpn_proposal
    props = []
    for i, meta in enumerate(img_metas):
        b, _ = oracle.rpn_predict_single_image([c[i].detach().numpy() for c in cls_outs],
                                               [r[i].detach().numpy() for r in reg_outs], lv_anc,
                                               meta['img_shape'][:2], meta['scale_factor'] * pc.min_bbox_size,
                                               pc.pre_nms, pc.post_nms, pc.max_num, pc.nms_iou,
                                               head.target_means, head.target_stds)
        props.append(b)
    for st in range(model.num_stages):
        rh, ex, sc = model.rcnn_head[st], model.roi_extractors[st], tc.rcnn[st]
        tl, tp, rois = [], [], []
        for i in range(len(img_metas)):
            out = oracle.bbox_target(props[i], gt_bboxes[i].numpy(), gt_labels[i].numpy(),
                                     (sc.assigner.pos_iou, sc.assigner.neg_iou, sc.assigner.min_pos_iou),
                                     (lambda lab, i=i, st=st: sampler_hook('rcnn{}'.format(st), i, lab))
                                     if sampler_hook else (sc.sampler.max_num, sc.sampler.pos_num),
                                     rh.target_means, rh.target_stds)
            tl.append(torch.from_numpy(out[2]))
            tp.append(torch.from_numpy(out[3]))
            rois.append(np.concatenate([np.full((1, out[0].shape[1]), i, np.float32), out[0]], 0).T)
        r5 = np.concatenate(rois, 0)
        L = len(ex.roi_layers)
        lv = oracle.roi_level_map(r5, ex.finest_scale, L) if L > 1 else None
        roi_feats = oracle.roi_align([f.detach().numpy() for f in feats[:L]], r5, lv,
                                     [l.spatial_scale for l in ex.roi_layers], ex.output_size,
                                     ex.roi_layers[0].sampling_ratio)
        x = torch.from_numpy(roi_feats)
        sizes = [t.numel() for t in tl]
        cls_outs_r, reg_outs_r = rh([x])
        c_loss, r_loss = rh.calc_loss_all(cls_outs_r[0], reg_outs_r[0], torch.cat(tl), torch.cat(tp, 1), sc)
        losses['rcnn_{}_cls_loss'.format(st)] = c_loss * tc.stage_loss_weight[st]
        losses['rcnn_{}_reg_loss'.format(st)] = r_loss * tc.stage_loss_weight[st]
        del sizes
    return losses

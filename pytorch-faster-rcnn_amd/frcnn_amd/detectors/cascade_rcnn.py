"""CascadeRCNN detector graph (reference lib/detectors/cascade_rcnn.py).
Faster R-CNN is the 1-stage case.  Same forward_train / forward_test flow;
every detection primitive underneath runs batched on the HIP kernels."""
import torch
from torch import nn

from .. import ops, utils
from ..region import RoiBatch


class CascadeRCNN(nn.Module):
    def __init__(self, num_stages=3, backbone=None, neck=None, rpn_head=None, roi_extractor=None, shared_head=None,
                 rcnn_head=None, train_cfg=None, test_cfg=None):
        super().__init__()
        from ..builder import build_module
        if num_stages <= 0:
            raise AssertionError('num_stages must be positive')
        self.num_stages = num_stages
        self.backbone = build_module(backbone)
        self.with_neck = neck is not None
        if self.with_neck:
            self.neck = nn.Sequential(*[build_module(c) for c in neck]) if isinstance(neck, list) else \
                build_module(neck)
        self.rpn_head = build_module(rpn_head)
        cfgs = roi_extractor if isinstance(roi_extractor, list) else [roi_extractor] * num_stages
        if len(cfgs) < num_stages:
            raise AssertionError('not enough roi extractors')
        self.roi_extractors = nn.ModuleList([build_module(cfgs[i]) for i in range(num_stages)])
        self.with_shared_head = shared_head is not None
        if self.with_shared_head:
            self.shared_head = build_module(shared_head)
        if isinstance(rcnn_head, list):
            if len(rcnn_head) < num_stages:
                raise AssertionError('not enough rcnn heads')
            heads = [build_module(rcnn_head[i]) for i in range(num_stages)]
        else:
            if num_stages != 1:
                raise AssertionError('rcnn_head must be consistent with num_stages')
            heads = [build_module(rcnn_head)]
        self.rcnn_head = nn.ModuleList(heads)
        self.train_cfg = train_cfg
        self.test_cfg = test_cfg
        # optional hipGraph of backbone + neck + RPN head convs (frcnn_amd.graphs.capture_trunk)
        self.graphed_trunk = None

    def init_weights(self):
        self.backbone.init_weights()
        self.rpn_head.init_weights()
        if self.with_neck:
            for nk in (self.neck if isinstance(self.neck, nn.Sequential) else [self.neck]):
                nk.init_weights()
        for h in self.rcnn_head:
            h.init_weights()
        if self.with_shared_head:
            self.shared_head.init_weights()

    def _sync_free_rcnn(self, feats):
        """Faster R-CNN (one stage) with the device sampler, RoIAlign extraction and the fused
        HIP head losses: the RCNN stage needs no host synchronisation on the sampled sizes."""
        if self.num_stages != 1 or self.with_shared_head:
            return False
        head, extractor = self.rcnn_head[0], self.roi_extractors[0]
        return (getattr(extractor, 'forward_flat', None) is not None and extractor._fusable() and
                getattr(head, 'sync_free', None) is not None and head.sync_free(self.train_cfg.rcnn[0], feats[0].device))

    def extract_feat(self, x):
        x = self.backbone(x)
        return self.neck(x) if self.with_neck else x

    def forward_train(self, img_data, gt_bboxes, gt_labels, img_metas):
        """cascade_rcnn.py:90-154."""
        try:
            return self._forward_train(img_data, gt_bboxes, gt_labels, img_metas)
        finally:
            ops.release_packs()  # the batch's gt packs are shared by the RPN and every stage only

    def _forward_train(self, img_data, gt_bboxes, gt_labels, img_metas):
        losses = {}
        if self.graphed_trunk is not None and self.graphed_trunk.matches(img_data):
            feats, rpn_cls, rpn_reg = self.graphed_trunk(img_data)
        else:
            feats = self.extract_feat(img_data)
            rpn_cls, rpn_reg = self.rpn_head(feats)
        cfg = self.train_cfg
        rpn_gt_labels = [torch.ones_like(g) for g in gt_labels]
        # (the proposal chain on a second stream beside the RPN target / loss chain was built and
        # measured slower in round 4: 309.4 vs 315.4 img/s; removed)
        props = self.rpn_head.predict_bboxes_from_output(rpn_cls, rpn_reg, img_metas, cfg.rpn_proposal)[0]
        l_cls, l_reg = self.rpn_head.loss(rpn_cls, rpn_reg, gt_bboxes, rpn_gt_labels, img_metas, cfg.rpn)
        losses['rpn_cls_loss'] = l_cls
        losses['rpn_reg_loss'] = l_reg
        if self._sync_free_rcnn(feats):
            # one stage, device sampler: padded targets, all rows through RoIAlign and the head,
            # the loss divides by the device count -- no host synchronisation in the RCNN stage
            head, extractor, scfg = self.rcnn_head[0], self.roi_extractors[0], cfg.rcnn[0]
            r = head.bbox_targets_flat(props, gt_bboxes, gt_labels, scfg)
            roi_out = extractor.forward_flat(feats, r['tar_props'], r['counts_dev'])
            rois = RoiBatch([roi_out])
            rois.flat = roi_out
            cls_out, reg_out = head(rois)[0].flat
            c_loss, r_loss = head.calc_loss_dev(cls_out, reg_out, r['tar_label'], r['tar_param'], r['n_dev'])
            losses['rcnn_0_cls_loss'] = c_loss * cfg.stage_loss_weight[0]
            losses['rcnn_0_reg_loss'] = r_loss * cfg.stage_loss_weight[0]
            return losses
        for i in range(self.num_stages):
            head, extractor, scfg = self.rcnn_head[i], self.roi_extractors[i], cfg.rcnn[i]
            tar_props, tar_bboxes, tar_labels, tar_params, tar_is_gts = head.bbox_targets(
                props, gt_bboxes, gt_labels, scfg)
            roi_outs = extractor(feats, tar_props)
            if self.with_shared_head:
                raise NotImplementedError('multi-image shared head is not implemented for CascadeRCNN')
            cls_outs, reg_outs = head(roi_outs)
            c_loss, r_loss = head.calc_loss(cls_outs, reg_outs, tar_labels, tar_params, scfg)
            losses['rcnn_{}_cls_loss'.format(i)] = c_loss * cfg.stage_loss_weight[i]
            losses['rcnn_{}_reg_loss'.format(i)] = r_loss * cfg.stage_loss_weight[i]
            if i < self.num_stages - 1:
                with torch.no_grad():
                    props = head.refine_bboxes(tar_props, tar_labels, reg_outs, tar_is_gts, img_metas)
        return losses

    def forward_test(self, img_data, img_metas):
        """cascade_rcnn.py:157-203."""
        cfg = self.test_cfg
        feats = self.extract_feat(img_data)
        props = list(self.rpn_head.predict_bboxes(feats, img_metas, cfg.rpn)[0])
        img_sizes = [m['img_shape'][:2] for m in img_metas]
        stage_cls = []
        for i in range(self.num_stages):
            head = self.rcnn_head[i]
            cls_outs, reg_outs = head(self.roi_extractors[i](feats, props))
            stage_cls.append(list(cls_outs))
            if i < self.num_stages - 1:
                labels = [c.argmax(1) for c in cls_outs]
                if head.use_sigmoid:
                    labels = [l + 1 for l in labels]
                props = head.refine_bboxes(props, labels, list(reg_outs), None, img_metas)
        per_img = utils.unpack_multi_result(stage_cls)
        mean_cls = [sum(c) / self.num_stages for c in per_img]
        return self.rcnn_head[-1].predict_bboxes_batched(props, mean_cls, list(reg_outs), img_sizes, cfg.rcnn)

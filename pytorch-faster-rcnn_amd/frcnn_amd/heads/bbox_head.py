"""BBoxHead base (reference lib/heads/bbox_head.py) with batched targets."""
import logging

import torch
from torch import nn

from .. import losses, ops, utils
from ..bbox import bbox_targets_batched


class BBoxHead(nn.Module):
    def __init__(self, num_classes, target_means=(0.0, 0.0, 0.0, 0.0), target_stds=(0.1, 0.1, 0.2, 0.2),
                 reg_class_agnostic=False, loss_cls=None, loss_bbox=None):
        super().__init__()
        from ..builder import build_module
        self.num_classes = num_classes
        self.target_means = list(target_means)
        self.target_stds = list(target_stds)
        self.reg_class_agnostic = reg_class_agnostic
        self.loss_cls = build_module(loss_cls) if isinstance(loss_cls, dict) else loss_cls
        self.loss_bbox = build_module(loss_bbox) if isinstance(loss_bbox, dict) else loss_bbox
        self.use_sigmoid = loss_cls.get('use_sigmoid', False) if isinstance(loss_cls, dict) else \
            getattr(self.loss_cls, 'use_sigmoid', False)
        self.cls_channels = num_classes - 1 if self.use_sigmoid else num_classes

    def bbox_targets(self, img_props, gt_bboxes, gt_labels, train_cfg):
        """Per image (tar_props, tar_bbox, tar_label, tar_param, tar_is_gt) lists (bbox_head.py:47-52),
        computed for the whole batch at once."""
        r = bbox_targets_batched(img_props, gt_bboxes, gt_labels, train_cfg.assigner, train_cfg.sampler,
                                 tuple(self.target_means), tuple(self.target_stds))
        return r['tar_props'], r['tar_bbox'], r['tar_label'], r['tar_param'], r['tar_is_gt']

    def sync_free(self, train_cfg, device):
        """Whether this head's targets and loss can run without reading the sampled row
        count back (see AnchorHead.sync_free): device sampler lists, fused HIP losses."""
        return (device.type == 'cuda' and train_cfg.get('sampler', None) is not None and
                ops.sampler_mode() == 'device' and losses.fused_kinds(self.loss_cls, self.loss_bbox))

    def bbox_targets_flat(self, img_props, gt_bboxes, gt_labels, train_cfg):
        """bbox_targets for the sync-free path: the flat padded buffers and the device counts."""
        return bbox_targets_batched(img_props, gt_bboxes, gt_labels, train_cfg.assigner, train_cfg.sampler,
                                    tuple(self.target_means), tuple(self.target_stds), sync=False)

    def calc_loss_dev(self, cls_out, reg_out, tar_label, tar_param, n_dev):
        """calc_loss_all over padded targets (label -1 rows ignored) with the sampled
        avg_factor as the device count n_dev (bbox_head.py:56-80; 0 rows -> zero losses)."""
        if self.reg_class_agnostic:
            l1 = lambda: ops._l1_args(reg_out, tar_param.t(), tar_label, 0)  # noqa: E731
        else:
            l1 = lambda: ops._l1_class_select_args(reg_out, self.num_classes, tar_param.t(), tar_label)  # noqa: E731
        return losses.head_losses(self.loss_cls, self.loss_bbox, cls_out, tar_label, l1, None, div_count=n_dev)

    def calc_loss_all(self, cls_out, reg_out, tar_label, tar_param, train_cfg):
        """bbox_head.py:56-80."""
        dev = cls_out.device
        cls_loss, reg_loss = losses.zero_loss(dev), losses.zero_loss(dev)
        n = len(tar_label)
        avg_factor = (tar_label > 0).sum() if 'sampler' not in train_cfg else n
        if avg_factor == 0:
            logging.warning('return zero loss due to zero avg_factor')
            return cls_loss, reg_loss
        if tar_label.numel() != 0:
            # both losses and their scaling in one launch (HIP losses, sampled avg_factor)
            if self.reg_class_agnostic:
                l1 = lambda: ops._l1_args(reg_out, tar_param.t(), tar_label, 0)  # noqa: E731
            else:
                l1 = lambda: ops._l1_class_select_args(reg_out, self.num_classes, tar_param.t(), tar_label)  # noqa: E731
            fused = losses.head_losses(self.loss_cls, self.loss_bbox, cls_out, tar_label, l1, avg_factor)
            if fused is not None:
                return fused
            cls_loss = self.loss_cls(cls_out, tar_label) / avg_factor
            if isinstance(self.loss_bbox, losses.SmoothL1Loss):
                # fused class selection + positive-row mask + smooth-L1 (one kernel each way)
                if self.reg_class_agnostic:
                    reg_loss = self.loss_bbox.masked(reg_out, tar_param.t(), tar_label, rows_dim=0)
                else:
                    reg_loss = self.loss_bbox.class_selected(reg_out, self.num_classes, tar_param.t(), tar_label)
                return cls_loss, reg_loss / avg_factor
            if not self.reg_class_agnostic:
                reg_out = reg_out.view(-1, 4, self.num_classes)
                reg_out = reg_out[torch.arange(n, device=dev), :, tar_label]
            # masked sum over positive rows (see AnchorHead.calc_loss): no host sync
            m = (tar_label > 0).view(-1, 1)
            z = reg_out.new_zeros(())
            reg_loss = self.loss_bbox(torch.where(m, reg_out, z), torch.where(m, tar_param.t(), z)) / avg_factor
        return cls_loss, reg_loss

    def calc_loss(self, cls_outs, reg_outs, tar_labels, tar_params, train_cfg):
        flat = getattr(cls_outs, 'flat', None)
        cls_out = flat[0] if flat is not None else torch.cat(cls_outs, 0)
        reg_out = flat[1] if flat is not None else torch.cat(reg_outs, 0)
        tl, tp = getattr(tar_labels, 'flat', None), getattr(tar_params, 'flat', None)  # the targets' own buffers
        return self.calc_loss_all(cls_out, reg_out, tl if tl is not None else torch.cat(tar_labels),
                                  tp if tp is not None else torch.cat(tar_params, 1), train_cfg)

    def refine_bboxes(self, props, labels, reg_outs, is_gts=None, img_metas=None):
        return utils.multi_apply(self.refine_bboxes_single_image, props, labels, reg_outs,
                                 is_gts if is_gts is not None else [None] * len(props),
                                 img_metas if img_metas is not None else [None] * len(props))

    def refine_bboxes_single_image(self, props, label, reg_out, is_gt=None, img_meta=None):
        """bbox_head.py:100-120: decode the predicted deltas of the labelled class, dropping gt rows."""
        if is_gt is None:
            is_gt = torch.zeros_like(label)
        if not (props.shape[1] == reg_out.shape[0] == is_gt.numel()):
            raise AssertionError('props / reg_out / is_gt size mismatch')
        n = len(label)
        if not self.reg_class_agnostic:
            reg_out = reg_out.view(-1, 4, self.num_classes)[torch.arange(n, device=reg_out.device), :, label]
        keep = ~is_gt.bool()
        return utils.param2bbox(props[:, keep], reg_out.t()[:, keep], self.target_means, self.target_stds,
                                img_meta['img_shape'] if img_meta is not None else None)

    def predict_bboxes_single_image(self, props, cls_out, reg_out, img_size=None, cfg=None):
        """bbox_head.py:122-146: softmax, per-class decode, multiclass NMS."""
        out = self.predict_bboxes_batched([props], [cls_out], [reg_out], [img_size], cfg)
        return out[0][0], out[1][0], out[2][0]

    def predict_bboxes_batched(self, props, cls_outs, reg_outs, img_sizes, cfg):
        """bbox_head.py:148-158 (predict_bboxes over the images) with ONE class-wise batched
        multiclass NMS (csrc/mcnms.hip): per image softmax + per-class decode (device ops),
        rows padded to the largest image, num_rows from the host-known shapes."""
        if self.use_sigmoid:
            raise NotImplementedError('Need to be implemented')
        with torch.no_grad():
            B = len(props)
            n = [int(c.shape[0]) for c in cls_outs]
            n_max, C = max(n), int(cls_outs[0].shape[1])
            dev = cls_outs[0].device
            dec = [utils.batched_param2bbox(props[b], reg_outs[b].t(), self.target_means, self.target_stds,
                                            img_sizes[b]).t() for b in range(B)]  # [n, 4] agnostic / [n, 4C]
            scores = cls_outs[0].new_zeros(B, n_max, C)
            boxes = cls_outs[0].new_zeros(B, n_max, dec[0].shape[1])
            for b in range(B):
                scores[b, :n[b]] = cls_outs[b].softmax(dim=1)
                boxes[b, :n[b]] = dec[b]
            res = ops.multiclass_nms_batched(boxes, scores, range(1, self.num_classes), cfg.nms_iou, cfg.min_score,
                                             cfg.max_per_img, mode=cfg.get('nms_type', 'official'),
                                             num_rows=torch.tensor(n, dtype=torch.int32).to(dev))
        return [[kb.t() for kb, _, _ in res], [ks for _, ks, _ in res], [kl for _, _, kl in res]]


class HeadOutputs(list):
    """Per-image head outputs plus the unsplit batch tensor (`flat`)."""
    flat = None

"""FCOSHead (reference lib/heads/fcos_head.py) with the ATSS target path on HIP.

ATSS targets (fcos_head.py:283-368) for every image of the batch
come from one `ops.atss_assign` call (frh_atss_assign: fill, per-(gt, level)
top-k, per-image resolve); the plain FCOS scale-range targets
(fcos_head.py:371-420), the losses (:418-534, focal / GIoU / centerness, QFL,
DFL) and inference (:566-627) are PyTorch-ROCm tensor code around them.
The LTRB helpers keep the reference's names and semantics.
"""
import logging
from collections import OrderedDict

import numpy as np
import torch
from torch import nn

from .. import ops, utils
from ..anchor import AnchorCreator
from ..utils import ChannelsLastConvs


# ---------------------------------------------------------------- LTRB helpers (fcos_head.py:9-116)
def length2class(length, cls_channels, stride):
    """fcos_head.py:10-29: distance -> two-hot distribution over cls_channels bins."""
    shape = length.shape
    flat = length.reshape(-1).float()
    n = flat.numel()
    flat = flat.clamp(0, (cls_channels - 1) * stride)
    left = (flat / stride).long()
    right = left + 1
    right_prob = (flat - left * stride) / stride
    left_prob = (right * stride - flat) / stride
    distr = flat.new_zeros((n, cls_channels))
    ar = torch.arange(n, device=flat.device)
    distr[ar, left] = left_prob
    distr[ar, right] = right_prob
    return distr.view(*shape, -1), left


def class2length(cls_score, stride):
    """fcos_head.py:32-40: expected length of a per-bin distribution."""
    c = cls_score.shape[-1]
    bins = torch.arange(c, device=cls_score.device, dtype=cls_score.dtype) * stride
    return (cls_score * bins).sum(-1)


def make_level_blanks(grids, dim, value, dtype, device):
    return [torch.full(list(g) + [dim], value, dtype=dtype, device=device) for g in grids]


def positive_ltrb(ltrb):
    return (ltrb > 0).all(dim=-1)


def centerness(ltrb):
    ltrb = ltrb + 1e-6
    l, t, r, b = [ltrb[..., i] for i in range(4)]
    return torch.sqrt((torch.min(l, r) / torch.max(l, r)) * (torch.min(t, b) / torch.max(t, b)))


def ltrb2bbox(ltrb, stride):
    """ltrb [4, H, W] -> boxes [4, H, W] around the cell centres."""
    idx = utils.full_index(ltrb.shape[1:]).to(device=ltrb.device, dtype=ltrb.dtype)
    coor = idx * stride + stride / 2
    return torch.stack([coor[:, :, 1] - ltrb[0], coor[:, :, 0] - ltrb[1], ltrb[2] + coor[:, :, 1],
                        ltrb[3] + coor[:, :, 0]])


def bbox2ltrb(bbox, grid, stride):
    """box [4] -> [H, W, 4] distances from every cell centre."""
    idx = utils.full_index(grid).to(device=bbox.device).float()
    coor = idx * stride + stride / 2.0
    return torch.stack([coor[:, :, 1] - bbox[0], coor[:, :, 0] - bbox[1], bbox[2] - coor[:, :, 1],
                        bbox[3] - coor[:, :, 0]], dim=-1)


def paint_value(canvas, bbox, scale, val):
    b = (bbox * scale).round().long()
    canvas[b[1]:b[3] + 1, b[0]:b[2] + 1] = val
    return canvas


def simple_ltrb2bbox(ltrb, ctr_xy):
    x, y = ctr_xy
    return torch.stack([x - ltrb[0], y - ltrb[1], x + ltrb[2], y + ltrb[3]])


def topk_by_center(anchors, bbox, k):
    """fcos_head.py:106-116 (row index by floor division)."""
    h, w = anchors.shape[-2:]
    flat = anchors.reshape(4, -1)
    ctr = torch.stack(list(utils.center_of(flat)))
    bctr = torch.stack(list(utils.center_of(bbox))).view(-1, 1)
    _, k_inds = (ctr - bctr).norm(dim=0).topk(k, largest=False)
    return k_inds % w, k_inds // w, flat[:, k_inds], k_inds.numel()


def _normal_init(m, std, bias=0.0):
    nn.init.normal_(m.weight, 0.0, std)
    nn.init.constant_(m.bias, bias)


class FCOSHead(ChannelsLastConvs):
    def __init__(self, num_classes=21, in_channels=256, stacked_convs=4, feat_channels=256,
                 strides=(8, 16, 32, 64, 126), anchor_center_lt=False, reg_std=300, reg_mean=0,
                 reg_coef=(1.0, 1.0, 1.0, 1.0, 1.0), reg_coef_trainable=False, atss_cfg=None, loss_cls=None,
                 loss_bbox=None, loss_dfl=None, loss_centerness=None):
        super().__init__()
        from ..builder import build_module
        self.num_classes = num_classes
        self.cls_channels = num_classes - 1
        self.in_channels = in_channels
        self.stacked_convs = stacked_convs
        self.feat_channels = feat_channels
        self.strides = list(strides)
        self.anchor_center_lt = anchor_center_lt
        self.reg_std, self.reg_mean = reg_std, reg_mean
        self.reg_coef_init = list(reg_coef)
        self.reg_coef_trainable = reg_coef_trainable
        self.atss_cfg = atss_cfg
        if atss_cfg is not None:
            self.use_atss = True
            self.anchor_creators = [AnchorCreator(base=s, scales=[atss_cfg['scale']], aspect_ratios=[1.0],
                                                  center_lt=anchor_center_lt) for s in self.strides]
        else:
            if loss_cls['type'] == 'QualityFocalLoss' or (loss_bbox or {}).get('type') == 'DistributionFocalLoss':
                raise AssertionError('GFL losses need the ATSS sampler')
            self.use_atss = False
            self.level_scale_thr = [0, 64, 128, 256, 512, 1e6]
        if loss_cls['type'] not in ('FocalLoss', 'QualityFocalLoss'):
            raise AssertionError('loss_cls must be FocalLoss or QualityFocalLoss')
        if loss_cls['type'] == 'QualityFocalLoss':
            self.use_centerness, self.use_qfl = False, True
            if loss_centerness is not None:
                logging.warning('Found loss cfg for centerness while QFL loss is present, will ignore centerness.')
        else:
            self.use_centerness, self.use_qfl = True, False
        self.loss_cls = build_module(loss_cls)
        self.use_dfl = loss_dfl is not None
        if loss_bbox is None:
            if not self.use_dfl:
                raise AssertionError('loss_bbox or loss_dfl is required')
            self.loss_bbox = None
        else:
            if loss_bbox['type'] != 'GIoULoss':
                raise AssertionError('Bbox loss only support GIoULoss for FCOSHead')
            self.loss_bbox = build_module(loss_bbox)
        if self.use_dfl:
            if loss_dfl['type'] != 'DistributionFocalLoss':
                raise AssertionError('loss_dfl must be DistributionFocalLoss')
            self.loss_dfl = build_module(loss_dfl)
        if self.use_centerness:
            self.loss_centerness = build_module(loss_centerness)
        self.use_gfl = self.use_qfl or self.use_dfl
        self._anchor_cache = {}
        self.init_layers()

    def init_layers(self):
        def tower():
            layers = []
            for i in range(self.stacked_convs):
                cin = self.in_channels if i == 0 else self.feat_channels
                layers += [nn.Conv2d(cin, self.feat_channels, 3, padding=1), nn.ReLU(inplace=True)]
            return nn.Sequential(*layers)
        self.cls_convs = tower()
        self.reg_convs = tower()
        self.fcos_cls = nn.Conv2d(self.feat_channels, self.cls_channels, 3, padding=1)
        reg_out = self.loss_dfl.cls_channels * 4 if self.use_dfl else 4
        self.fcos_reg = nn.Conv2d(self.feat_channels, reg_out, 3, padding=1)
        self.fcos_center = nn.Conv2d(self.feat_channels, 1, 3, padding=1)
        if self.use_dfl:
            coef = torch.stack([torch.ones(self.loss_dfl.cls_channels) * x for x in self.reg_coef_init]).float()
        else:
            coef = torch.tensor(self.reg_coef_init, dtype=torch.float)
        self.reg_coef = nn.Parameter(coef, requires_grad=self.reg_coef_trainable)

    def init_weights(self):
        for tower in (self.cls_convs, self.reg_convs):
            for m in tower:
                if isinstance(m, nn.Conv2d):
                    _normal_init(m, 0.01)
        _normal_init(self.fcos_cls, 0.01, float(-np.log((1 - 0.01) / 0.01)))
        _normal_init(self.fcos_reg, 0.01)
        _normal_init(self.fcos_center, 0.01)

    def forward(self, xs):
        cls_t = [self.cls_convs(x) for x in xs]
        reg_t = [self.reg_convs(x) for x in xs]
        cls_outs = [self.fcos_cls(x) for x in cls_t]
        ctr_outs = [self.fcos_center(x) for x in reg_t]
        if self.use_dfl:
            reg_outs = []
            for i, x in enumerate(reg_t):
                coef = torch.cat([self.reg_coef[i].view(-1, 1)] * 4, dim=1)
                reg_outs.append(self.fcos_reg(x) * coef.view(-1, 1, 1))
        else:
            reg_outs = [torch.exp(self.fcos_reg(x) * self.reg_coef[i]) for i, x in enumerate(reg_t)]
        return cls_outs, reg_outs, ctr_outs

    # ------------------------------------------------------------ ATSS targets (HIP)
    def _flat_anchors(self, grids, device):
        key = (tuple((int(h), int(w)) for h, w in grids), str(device))
        a = self._anchor_cache.get(key)
        if a is None:
            a = torch.cat([ops.anchor_grid([g], [float(s)], c.ws, c.hs, 1, self.anchor_center_lt, device)
                           for g, s, c in zip(key[0], self.strides, self.anchor_creators)], 1).contiguous()
            self._anchor_cache[key] = a
        return a

    def targets_atss_batched(self, grids, gt_bboxes, gt_labels, img_metas, device):
        """Level-concatenated (cls [B, N] i64, reg [B, N, 4], ctr [B, N]) for the batch."""
        anchors = self._flat_anchors(grids, device)
        return ops.atss_assign(anchors, grids, [float(s) for s in self.strides], list(gt_bboxes), list(gt_labels),
                               [m['img_shape'][:2] for m in img_metas], int(self.atss_cfg['topk']))

    @staticmethod
    def _split_levels(flat, grids, dim):
        out, off = [], 0
        for h, w in grids:
            n = int(h) * int(w)
            out.append(flat[off:off + n].view(int(h), int(w), dim))
            off += n
        return out

    def single_image_targets_atss(self, cls_outs, reg_outs, ctr_outs, lvl_anchors, gt_bboxes, gt_labels, img_meta,
                                  train_cfg):
        """fcos_head.py:283-368: per-level ([H, W, 1] labels, [H, W, 4] ltrb, [H, W, 1] centerness)."""
        if not (len(cls_outs) == len(reg_outs) == len(self.strides) == len(lvl_anchors)):
            raise AssertionError('level count mismatch')
        grids = [tuple(x.shape[-2:]) for x in cls_outs]
        cls, reg, ctr = self.targets_atss_batched(grids, [gt_bboxes], [gt_labels], [img_meta], cls_outs[0].device)
        return (self._split_levels(cls[0], grids, 1), self._split_levels(reg[0], grids, 4),
                self._split_levels(ctr[0], grids, 1))

    # ------------------------------------------------------------ plain FCOS targets
    def single_image_targets(self, cls_outs, reg_outs, ctr_outs, gt_bboxes, gt_labels, img_meta, train_cfg):
        """fcos_head.py:371-420: scale-range assignment, larger gts first."""
        gt_bboxes, gt_labels = utils.sort_bbox(gt_bboxes, labels=gt_labels, descending=True)
        dev = cls_outs[0].device
        grids = [x.shape[-2:] for x in cls_outs]
        img_h, img_w = img_meta['img_shape'][:2]
        cls_tars = make_level_blanks(grids, 1, -1, torch.long, dev)
        reg_tars = make_level_blanks(grids, 4, -1, torch.float, dev)
        ctr_tars = make_level_blanks(grids, 1, -1, torch.float, dev)
        img_box = torch.tensor([0, 0, img_w, img_h], dtype=torch.float)
        for i, s in enumerate(self.strides):
            paint_value(cls_tars[i], img_box, 1 / s, 0)
            paint_value(ctr_tars[i], img_box, 1 / s, 0)
        for g in range(gt_bboxes.shape[1]):
            for j, s in enumerate(self.strides):
                ltrb = bbox2ltrb(gt_bboxes[:, g], grids[j], s)
                mx, _ = ltrb.max(2)
                m = positive_ltrb(ltrb) & (mx >= self.level_scale_thr[j]) & (mx < self.level_scale_thr[j + 1])
                cls_tars[j][m] = gt_labels[g]
                reg_tars[j][m] = ltrb[m]
        for i in range(len(self.strides)):
            pos = cls_tars[i] > 0
            ctr_tars[i][pos] = centerness(reg_tars[i]).unsqueeze(-1)[pos]
        return cls_tars, reg_tars, ctr_tars

    # ------------------------------------------------------------ losses
    def calc_loss_flat(self, cls_outs, reg_outs, ctr_outs, cls_tars, reg_tars, ctr_tars):
        """fcos_head.py:418-534 on batch-flattened tensors: cls_outs [C, M], reg_outs [4|4*bins, M],
        ctr_outs [1, M], cls_tars [M], reg_tars [M, 4], ctr_tars [M] (images outer, levels inner)."""
        chosen = cls_tars >= 0
        pos = cls_tars > 0
        num_pos = int(pos.sum())
        cls_as_weight, _ = cls_outs.detach()[:, pos].sigmoid().max(0)
        ctr_outs = ctr_outs.reshape(-1, 1)
        pos_ctr_outs = ctr_outs[pos, :]
        pos_ctr_tars = ctr_tars[pos]
        ctr_loss = self.loss_centerness(pos_ctr_outs, pos_ctr_tars) / num_pos if self.use_centerness else None
        pos_reg_tars = (reg_tars[pos, :].t() - self.reg_mean) / self.reg_std
        pos_reg_outs = reg_outs[:, pos]
        quality = None
        if self.use_dfl:
            cc, stride = self.loss_dfl.cls_channels, self.loss_dfl.stride
            y = pos_reg_tars.contiguous().view(-1)
            _, left_idx = length2class(y, cc, stride)
            pos_reg_outs = pos_reg_outs.reshape(cc, -1).t()
            dfl_loss = self.loss_dfl(pos_reg_outs, y, left_idx, weight=cls_as_weight.repeat(4).view(-1),
                                     avg_factor=4.0)
        else:
            dfl_loss = None
        if self.loss_bbox is None:
            bbox_loss = None
        elif self.use_dfl:
            out_ltrb = class2length(pos_reg_outs.softmax(-1), self.loss_dfl.stride).view(4, -1)
            a = simple_ltrb2bbox(out_ltrb, (0.0, 0.0))
            b = simple_ltrb2bbox(pos_reg_tars.reshape(4, -1), (0.0, 0.0))
            quality = utils.elem_iou(a.detach(), b)
            bbox_loss = self.loss_bbox(a, b, weight=cls_as_weight, avg_factor=num_pos)
        elif self.use_qfl:
            a = simple_ltrb2bbox(pos_reg_outs, (0.0, 0.0))
            b = simple_ltrb2bbox(pos_reg_tars, (0.0, 0.0))
            quality = utils.elem_iou(a.detach(), b)
            bbox_loss = self.loss_bbox(a, b, weight=cls_as_weight, avg_factor=num_pos)
        else:
            if self.reg_mean > 0:
                raise AssertionError('reg_mean must be <= 0 without GFL')
            a = simple_ltrb2bbox(pos_reg_outs, (0.0, 0.0))
            b = simple_ltrb2bbox(pos_reg_tars, (0.0, 0.0))
            bbox_loss = self.loss_bbox(a, b, weight=pos_ctr_tars, avg_factor=num_pos)
        if self.use_qfl:
            q_all = quality.new_zeros(chosen.numel())
            q_all[pos] = quality
            cls_loss = self.loss_cls(cls_outs[:, chosen].t(), q_all[chosen], cls_tars[chosen], avg_factor=num_pos)
        else:
            cls_loss = self.loss_cls(cls_outs[:, chosen].t(), cls_tars[chosen]) / num_pos
        res = {'cls_loss': cls_loss, 'ctr_loss': ctr_loss, 'dfl_loss': dfl_loss, 'bbox_loss': bbox_loss}
        return OrderedDict((k, v) for k, v in res.items() if v is not None)

    def calc_loss(self, cls_outs, reg_outs, ctr_outs, cls_tars, reg_tars, ctr_tars):
        """fcos_head.py:418: per-image lists of per-level outputs / targets."""
        cat_o = lambda xs: torch.cat([utils.concate_grid_result(x, False) for x in xs], dim=-1)
        cat_t = lambda xs: torch.cat([utils.concate_grid_result(x, True) for x in xs], dim=0)
        return self.calc_loss_flat(cat_o(cls_outs), cat_o(reg_outs), cat_o(ctr_outs),
                                   cat_t(cls_tars).view(-1), cat_t(reg_tars), cat_t(ctr_tars).view(-1))

    def forward_train(self, feats, gt_bboxes, gt_labels, img_metas, train_cfg):
        cls_outs, reg_outs, ctr_outs = self.forward(feats)
        grids = [tuple(x.shape[-2:]) for x in cls_outs]
        B = cls_outs[0].shape[0]
        flat_o = lambda xs: torch.cat([x.reshape(B, x.shape[1], -1) for x in xs], -1).permute(1, 0, 2).reshape(
            xs[0].shape[1], -1)
        if self.use_atss:
            cls_t, reg_t, ctr_t = self.targets_atss_batched(grids, gt_bboxes, gt_labels, img_metas,
                                                            cls_outs[0].device)
            return self.calc_loss_flat(flat_o(cls_outs), flat_o(reg_outs), flat_o(ctr_outs), cls_t.view(-1),
                                       reg_t.view(-1, 4), ctr_t.view(-1))
        tars = utils.unpack_multi_result(utils.multi_apply(
            self.single_image_targets, utils.split_by_image(cls_outs), utils.split_by_image(reg_outs),
            utils.split_by_image(ctr_outs), list(gt_bboxes), list(gt_labels), list(img_metas), train_cfg))
        return self.calc_loss(utils.split_by_image(cls_outs), utils.split_by_image(reg_outs),
                              utils.split_by_image(ctr_outs), *tars)

    # ------------------------------------------------------------ inference
    def image_candidates(self, cls_outs, reg_outs, ctr_outs, img_meta, test_cfg):
        """fcos_head.py:566-620 for one image: per-level decode, clamp, min-size filter, top-k
        by (centerness x) best class score.  Returns boxes [4, n], scores [C, n] and the
        centerness factor [n] (or None)."""
        use_center = self.use_centerness
        min_size = img_meta['scale_factor'] * test_cfg['min_bbox_size']
        img_size = img_meta['img_shape'][:2]
        bboxes, scores, ctrs = [], [], []
        for i in range(len(cls_outs)):
            if self.use_dfl:
                r = reg_outs[i]
                gs = r.shape[-2:]
                r = r.reshape(self.loss_dfl.cls_channels, -1).t().softmax(-1)
                ltrb = class2length(r, self.loss_dfl.stride) * self.reg_std + self.reg_mean
                bbox = ltrb2bbox(ltrb.view(4, *gs), self.strides[i])
            else:
                bbox = ltrb2bbox(reg_outs[i] * self.reg_std + self.reg_mean, self.strides[i])
            score = cls_outs[i].sigmoid().reshape(self.cls_channels, -1)
            ctr = ctr_outs[i].sigmoid().reshape(1, -1) if use_center else None
            bbox = utils.clamp_bbox(bbox.reshape(4, -1), img_size)
            keep = ((bbox[2] - bbox[0] + 1) > min_size) & ((bbox[3] - bbox[1] + 1) > min_size)
            score, bbox = score[:, keep], bbox[:, keep]
            ctr = ctr[:, keep] if use_center else None
            if 0 < test_cfg['pre_nms'] < score.shape[1]:
                mx, _ = (score * ctr).max(0) if use_center else score.max(0)
                _, top = mx.topk(test_cfg['pre_nms'])
                score, bbox = score[:, top], bbox[:, top]
                ctr = ctr[:, top] if use_center else None
            bboxes.append(bbox)
            scores.append(score)
            ctrs.append(ctr)
        sc = torch.cat(scores, 1)
        bx = torch.cat(bboxes, 1)
        ct = torch.cat(ctrs, 1).view(-1) if use_center else None
        return bx, sc, ct

    def predict_single_image(self, cls_outs, reg_outs, ctr_outs, img_meta, test_cfg):
        """fcos_head.py:566-627."""
        out = self._predict_batch([self.image_candidates(cls_outs, reg_outs, ctr_outs, img_meta, test_cfg)],
                                  test_cfg)
        return out[0][0], out[1][0], out[2][0]

    def _predict_batch(self, cands, test_cfg):
        """ONE class-wise batched multiclass NMS (csrc/mcnms.hip) over the images' candidates,
        rows padded to the largest image (fcos_head.py:621-627)."""
        B = len(cands)
        n = [int(bx.shape[1]) for bx, _, _ in cands]
        n_max = max(n)
        ref = cands[0][1]
        scores = ref.new_zeros(B, n_max, self.cls_channels)
        boxes = ref.new_zeros(B, n_max, 4)
        ctr = ref.new_zeros(B, n_max) if self.use_centerness else None
        for b, (bx, sc, ct) in enumerate(cands):
            scores[b, :n[b]] = sc.t()
            boxes[b, :n[b]] = bx.t()
            if ctr is not None:
                ctr[b, :n[b]] = ct
        res = ops.multiclass_nms_batched(boxes, scores, list(range(0, self.cls_channels)), test_cfg['nms_iou'],
                                         test_cfg['min_score'], test_cfg['max_per_img'], ctr,
                                         mode=test_cfg.get('nms_type', 'official'),
                                         num_rows=torch.tensor(n, dtype=torch.int32).to(ref.device))
        return [[kb.t() for kb, _, _ in res], [ks for _, ks, _ in res], [kl + 1 for _, _, kl in res]]

    def predict_bboxes(self, feats, img_metas, test_cfg):
        cls_outs, reg_outs, ctr_outs = self.forward(feats)
        ctrs = utils.split_by_image(ctr_outs) if self.use_centerness else [None] * len(img_metas)
        cands = [self.image_candidates(c, r, t, m, test_cfg) for c, r, t, m in
                 zip(utils.split_by_image(cls_outs), utils.split_by_image(reg_outs), ctrs, list(img_metas))]
        return self._predict_batch(cands, test_cfg)

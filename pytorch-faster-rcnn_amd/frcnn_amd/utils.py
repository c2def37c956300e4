"""Box utilities with the reference's API (lib/utils.py), computed by HIP kernels.

Signatures, argument meaning and errors follow the reference functions cited
per function; the arithmetic runs in libfrcnn_amd.so.  Pure-Python glue of
the reference (multi_apply & co.) is restated here because heads use it.
"""
import torch

from . import ops


def conv_layout(module):
    """Keep `module`'s Conv2d weights channels-last on a HIP device (the layout of the FPN's
    NHWC levels: MIOpen's faster 3x3 / 1x1 convolutions on them) and in the
    default layout elsewhere (CPU references).  Values are unchanged."""
    for m in module.modules():
        if isinstance(m, torch.nn.Conv2d) and m.weight.dim() == 4:
            fmt = torch.channels_last if m.weight.is_cuda else torch.contiguous_format
            if not m.weight.is_contiguous(memory_format=fmt):
                m.weight.data = m.weight.data.contiguous(memory_format=fmt)


class ChannelsLastConvs(torch.nn.Module):
    """Mixin: conv_layout after every device / dtype move (.to, .cuda, .cpu)."""

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        conv_layout(self)
        return self


def sum_list(lst):
    if len(lst) == 0:
        raise AssertionError('empty list')
    res = lst[0]
    for x in lst[1:]:
        res = res + x
    return res


def input_size(img_metas):
    """Max padded (h, w) over a batch (utils.py:24-26)."""
    pads = [m['pad_shape'][:2] for m in img_metas]
    return [max(p[i] for p in pads) for i in range(2)]


def index_of(bool_tsr):
    return tuple(torch.nonzero(bool_tsr).t())


def wh_from_xyxy(bbox):
    return bbox[2] - bbox[0] + 1, bbox[3] - bbox[1] + 1


def xyxy2xywh(xyxy):
    """utils.py:146-147: [4, n] inclusive-pixel xyxy -> xywh (w = x2 - x1 + 1)."""
    return torch.stack([xyxy[0], xyxy[1], xyxy[2] - xyxy[0] + 1, xyxy[3] - xyxy[1] + 1])


def xywh2xyxy(xywh):
    """utils.py:148-149."""
    return torch.stack([xywh[0], xywh[1], xywh[0] + xywh[2] - 1, xywh[1] + xywh[3] - 1])


def center_of(bbox):
    return (bbox[2] + bbox[0]) / 2, (bbox[3] + bbox[1]) / 2


def to_pair(val):
    if isinstance(val, int):
        return (val, val)
    val = tuple(val)
    if len(val) != 2:
        raise AssertionError('expected a pair')
    return val


def simplify_label(label):
    out = label.clone()
    out[label > 0] = 1
    return out


def _check4(*ts):
    for t in ts:
        if t.dim() != 2 or t.shape[0] != 4:
            raise AssertionError('boxes must be [4, n]')


def bbox2param(base, bbox, means=(0.0, 0.0, 0.0, 0.0), stds=(1.0, 1.0, 1.0, 1.0)):
    """utils.py:47-70: (tx, ty, tw, th) of bbox w.r.t. base, normalised by means/stds."""
    if base.shape != bbox.shape:
        raise AssertionError('base and bbox shapes differ')
    _check4(base)
    return ops.bbox2param(base, bbox, list(means), list(stds))


def param2bbox(base, param, means=(0.0, 0.0, 0.0, 0.0), stds=(1.0, 1.0, 1.0, 1.0), img_size=None):
    """utils.py:83-92 (+clamp_bbox when img_size is given)."""
    if base.shape != param.shape:
        raise AssertionError('base and param shapes differ')
    _check4(base)
    return ops.param2bbox(base, param, list(means), list(stds), img_size)


def batched_param2bbox(base, param, means=(0.0, 0.0, 0.0, 0.0), stds=(1.0, 1.0, 1.0, 1.0), img_size=None):
    """utils.py:96-106: param [4*ncls, n] in coordinate-major class layout."""
    if param.shape[0] % 4 != 0:
        raise AssertionError('param rows must be a multiple of 4')
    return ops.param2bbox(base, param, list(means), list(stds), img_size)


def clamp_bbox(bbox, img_size):
    """utils.py:109-120 (plain torch clamp: boundary glue, not on the hot path)."""
    H, W = img_size[:2]
    return torch.stack([bbox[0].clamp(0.0, W - 1), bbox[1].clamp(0.0, H - 1),
                        bbox[2].clamp(0.0, W - 1), bbox[3].clamp(0.0, H - 1)])


def calc_iou(a, b):
    """utils.py:151-172: [N, K] IoU table with +1 widths (bit-exact)."""
    if a.shape[0] != 4 or b.shape[0] != 4:
        raise AssertionError('boxes must be [4, n]')
    return ops.iou_table(a, b)


def elem_iou(a, b):
    """utils.py:174-182: element-wise IoU without +1."""
    if not (a.shape[0] == 4 and b.shape[0] == 4 and a.shape == b.shape):
        raise AssertionError('boxes must both be [4, n]')
    return ops.elem_iou(a, b)


def batched_nms(bbox, score, label, nms_iou, class_agnostic=False):
    """utils.py:211-221: class-aware NMS via the coordinate-offset trick."""
    n = score.numel()
    if n == 0:
        return bbox, score, label
    if class_agnostic:
        nms_bbox = bbox
    else:
        max_range = bbox.max()
        nms_bbox = bbox + (label * max_range).to(bbox).view(n, 1)
    keep = ops.nms(nms_bbox, score, nms_iou)
    return bbox[keep, :], score[keep], label[keep]


def multiclass_nms(bbox, score, nms_channel, nms_iou, min_score=-1, max_num=None, score_factor=None,
                   mode='official'):
    """utils.py:224-269 for one image: the class-wise batched kernel (ops.multiclass_nms_batched,
    csrc/mcnms.hip) with a batch of one."""
    if mode not in ('official', 'strict'):
        raise AssertionError('unknown mode {}'.format(mode))
    if score.dim() != 2:
        raise AssertionError('multiclass_nms only applies to multi-channel score')
    sf = None
    if score_factor is not None:  # [n] / [n, 1] per row, [n, C] per (row, class)
        per_row = score_factor.dim() == 1 or score_factor.shape[-1] == 1
        sf = score_factor.reshape(1, -1) if per_row else score_factor.unsqueeze(0)
    return ops.multiclass_nms_batched(bbox.unsqueeze(0), score.unsqueeze(0), nms_channel, nms_iou, min_score,
                                      max_num, sf, mode)[0]


def one_hot_embedding(label, n_cls):
    out = label.new_zeros((len(label), n_cls))
    out[torch.arange(len(label), device=label.device), label] = 1
    return out


def multi_apply(func, *args):
    """utils.py:278-296: call func per element of the list arguments."""
    lists = [a for a in args if isinstance(a, list)]
    n = len(lists[0]) if lists else 1
    for a in lists:
        if len(a) != n:
            raise ValueError('Arg: {} does not have the same length as others'.format(a))
    return [func(*[a[i] if isinstance(a, list) else a for a in args]) for i in range(n)]


def unpack_multi_result(multi_res):
    if len(multi_res) == 0:
        raise AssertionError('empty result list')
    return [[r[i] for r in multi_res] for i in range(len(multi_res[0]))]


def class_name(obj):
    return type(obj).__name__


def split_by_image(tsr_list):
    return [[x[i] for x in tsr_list] for i in range(tsr_list[0].shape[0])]


def init_module_normal(m, mean=0.0, std=1.0):
    for name, p in m.named_parameters():
        if 'weight' in name:
            p.data.normal_(mean, std)
        if 'bias' in name:
            p.data.zero_()


def full_index(size):
    """utils.py:338-341: [*size, len(size)] long tensor of every index (row-major)."""
    grids = torch.meshgrid(*[torch.arange(int(s)) for s in size], indexing='ij')
    return torch.stack(grids, dim=-1)


def sort_bbox(bbox, labels=None, descending=False):
    """utils.py:362-366: boxes [4, n] sorted by (w+1)(h+1) area."""
    w, h = wh_from_xyxy(bbox)
    _, idx = (w * h).sort(descending=descending)
    return bbox[:, idx], labels[idx] if labels is not None else None


def concate_grid_result(grid_res, last=True):
    """utils.py:372-374: per-level grid tensors flattened and concatenated."""
    grid_res = [x.reshape(-1, x.shape[-1]) if last else x.reshape(x.shape[0], -1) for x in grid_res]
    return torch.cat(grid_res, dim=0 if last else -1)

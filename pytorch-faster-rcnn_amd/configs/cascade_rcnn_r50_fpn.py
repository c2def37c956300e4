# Cascade R-CNN R50-FPN (BASELINE config 4), in the reference's config-file format.
# Hyper-parameters follow the reference's configs/cascade_rcnn_r50_fpn.py (3 stages,
# class-agnostic regression, stage IoU 0.5 / 0.6 / 0.7); data pipeline out of scope.

_strides = [4, 8, 16, 32, 64]
_stds = [[0.1, 0.1, 0.2, 0.2], [0.05, 0.05, 0.1, 0.1], [0.033, 0.033, 0.067, 0.067]]


def _loss(kind, **kw):
    return dict(type=kind, **kw)


model = dict(
    type='CascadeRCNN',
    num_stages=3,
    backbone=dict(type='ResNet', depth=50, frozen_stages=1, out_layers=(1, 2, 3, 4), pretrained=False),
    neck=dict(type='FPN', in_channels=[256, 512, 1024, 2048], out_channels=256, num_outs=5),
    rpn_head=dict(type='RPNHead', in_channels=256, feat_channels=256, anchor_scales=[8],
                  anchor_ratios=[0.5, 1.0, 2.0], anchor_strides=_strides,
                  target_means=[0.0] * 4, target_stds=[1.0] * 4,
                  loss_cls=_loss('CrossEntropyLoss', use_sigmoid=True, loss_weight=1.0),
                  loss_bbox=_loss('SmoothL1Loss', beta=1.0 / 9.0, loss_weight=1.0)),
    roi_extractor=dict(type='BasicRoIExtractor', output_size=(7, 7),
                       roi_layers=[dict(type='RoIAlign', spatial_scale=1.0 / s, sampling_ratio=2)
                                   for s in _strides[:4]]),
    rcnn_head=[dict(type='RCNNHead', in_channels=256, roi_out_size=(7, 7), fc_channels=[1024, 1024],
                    with_avg_pool=False, num_classes=21, target_means=[0.0] * 4, target_stds=std,
                    reg_class_agnostic=True,
                    loss_cls=_loss('CrossEntropyLoss', use_sigmoid=False, loss_weight=1.0),
                    loss_bbox=_loss('SmoothL1Loss', beta=1.0, loss_weight=1.0)) for std in _stds],
)

train_cfg = dict(
    rpn=dict(assigner=dict(type='MaxIoUAssigner', pos_iou=0.7, neg_iou=0.3, min_pos_iou=0.3),
             sampler=dict(type='RandomSampler', max_num=256, pos_num=128),
             allowed_border=0),
    rpn_proposal=dict(pre_nms=2000, post_nms=2000, max_num=2000, nms_iou=0.7, min_bbox_size=0),
    rcnn=[dict(assigner=dict(type='MaxIoUAssigner', pos_iou=t, neg_iou=t, min_pos_iou=t),
               sampler=dict(type='RandomSampler', max_num=512, pos_num=128)) for t in (0.5, 0.6, 0.7)],
    stage_loss_weight=[1.0, 0.5, 0.25],
)

test_cfg = dict(
    rpn=dict(pre_nms=1000, post_nms=1000, max_num=1000, nms_iou=0.7, min_bbox_size=0.0),
    rcnn=dict(min_score=0.05, nms_iou=0.5, max_per_img=100),
)

data = dict(train=dict(imgs_per_gpu=2), test=dict(imgs_per_gpu=2))

# optimiser of the reference config (lib/trainer: OptimizerHook clips, then SGD steps)
optimizer = dict(type='SGD', lr=0.0025, momentum=0.9, weight_decay=0.0001)
optimizer_config = dict(grad_clip=dict(max_norm=35, norm_type=2))

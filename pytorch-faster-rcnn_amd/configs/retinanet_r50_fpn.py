# RetinaNet R50-FPN (BASELINE config 3), in the reference's config-file format.
# Hyper-parameters follow the reference's configs/retinanet_r50_fpn.py; the data
# pipeline section is out of this build's scope.

model = dict(
    type='RetinaNet',
    backbone=dict(type='ResNet', depth=50, frozen_stages=1, out_layers=(1, 2, 3, 4), pretrained=False),
    neck=dict(type='FPN', in_channels=[256, 512, 1024, 2048], out_channels=256, start_level=1,
              extra_use_convs=True, num_outs=5),
    bbox_head=dict(type='RetinaHead', num_classes=21, in_channels=256, stacked_convs=4, feat_channels=256,
                   octave_base_scale=4, scales_per_octave=3, anchor_ratios=[0.5, 1.0, 2.0],
                   anchor_strides=[8, 16, 32, 64, 128],
                   loss_cls=dict(type='FocalLoss', alpha=0.25, gamma=2.0, loss_weight=1.0),
                   loss_bbox=dict(type='SmoothL1Loss', beta=1.0 / 9.0, loss_weight=1.0)))

train_cfg = dict(assigner=dict(type='MaxIoUAssigner', pos_iou=0.5, neg_iou=0.4, min_pos_iou=0.0),
                 allowed_border=-1, total_epochs=14)

test_cfg = dict(pre_nms=1000, min_bbox_size=0, min_score=0.05, nms_iou=0.5, nms_type='strict', max_per_img=100)

data = dict(train=dict(imgs_per_gpu=8), test=dict(imgs_per_gpu=8))

# optimiser of the reference config (lib/trainer: OptimizerHook clips, then SGD steps)
optimizer = dict(type='SGD', lr=0.00125, momentum=0.9, weight_decay=0.0001)
optimizer_config = dict(grad_clip=dict(max_norm=35, norm_type=2))

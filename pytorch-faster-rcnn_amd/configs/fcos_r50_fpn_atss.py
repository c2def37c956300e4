# ATSS R50-FPN (BASELINE config 5), in the reference's config-file format.
# Hyper-parameters follow the reference's configs/fcos_r50_fpn_atss.py;
# the data pipeline section is out of this build's scope.

model = dict(
    type='FCOS',
    backbone=dict(type='ResNet', depth=50, frozen_stages=1, out_layers=(1, 2, 3, 4), pretrained=False),
    neck=dict(type='FPN', in_channels=[256, 512, 1024, 2048], out_channels=256, start_level=1,
              extra_use_convs=True, extra_convs_on_inputs=False, num_outs=5, relu_before_extra_convs=False),
    bbox_head=dict(type='FCOSHead', num_classes=21, in_channels=256, stacked_convs=4, feat_channels=256,
                   strides=[8, 16, 32, 64, 128], reg_std=1200, reg_mean=0, reg_coef=[1.0] * 5,
                   reg_coef_trainable=True, atss_cfg=dict(topk=9, scale=8),
                   loss_cls=dict(type='FocalLoss', use_sigmoid=True, loss_weight=1.0),
                   loss_bbox=dict(type='GIoULoss', loss_weight=2.0),
                   loss_centerness=dict(type='CrossEntropyLoss', use_sigmoid=True, loss_weight=1.0)))

train_cfg = dict(allowed_border=-1, total_epochs=24)

test_cfg = dict(pre_nms=1000, min_bbox_size=0, min_score=0.05, nms_iou=0.6, nms_type='strict', max_per_img=100)

# optimiser of the reference config (lib/trainer: OptimizerHook clips, then SGD steps)
optimizer = dict(type='SGD', lr=0.00125, momentum=0.9, weight_decay=0.0001)
optimizer_config = dict(grad_clip=None)

"""Registry + build_module with the reference's contract (lib/builder.py:26-37):
`MODULES[cls.__name__] = cls`; build_module(cfg, *args, **kw) shallow-copies
the cfg, pops 'type', raises ValueError for unregistered types and calls
MODULES[type](*args, **cfg, **kw).  The reference's detectors, heads and the
torchvision RoIAlign/RoIPool names resolve to this framework's classes."""
import copy

from torch.optim import SGD

from .backbones import ResNet, ResLayerC5
from .necks import FPN
from .region import MaxIoUAssigner, RandomSampler, BasicRoIExtractor
from .losses import (FocalLoss, SmoothL1Loss, CrossEntropyLoss, GIoULoss, IoULoss, QualityFocalLoss,
                     DistributionFocalLoss)
from .heads import RPNHead, RCNNHead, RetinaHead, FCOSHead
from .detectors import CascadeRCNN, RetinaNet, FCOS
from .ops import RoIAlign, RoIPool

_MODULE_LIST = [RetinaNet, CascadeRCNN, FCOS, ResNet, ResLayerC5, FPN, RetinaHead, RPNHead, RCNNHead, FCOSHead,
                CrossEntropyLoss, SmoothL1Loss, FocalLoss, GIoULoss, IoULoss, QualityFocalLoss, DistributionFocalLoss,
                BasicRoIExtractor, RoIAlign, RoIPool, SGD, MaxIoUAssigner, RandomSampler]

MODULES = {cls.__name__: cls for cls in _MODULE_LIST}


def register(cls):
    MODULES[cls.__name__] = cls
    return cls


def build_module(cfg, *args, **kwargs):
    cfg = copy.copy(cfg)
    if 'type' not in cfg:
        raise AssertionError("cfg has no 'type'")
    m_type = cfg.pop('type')
    if m_type not in MODULES:
        raise ValueError("'{}' is not registered".format(m_type))
    return MODULES[m_type](*args, **cfg, **kwargs)

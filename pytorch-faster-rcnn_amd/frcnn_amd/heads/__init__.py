from .anchor_head import AnchorHead
from .rpn_head import RPNHead
from .bbox_head import BBoxHead
from .rcnn_head import RCNNHead
from .retina_head import RetinaHead

__all__ = ['AnchorHead', 'RPNHead', 'BBoxHead', 'RCNNHead', 'RetinaHead']

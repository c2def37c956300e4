from .anchor_head import AnchorHead
from .rpn_head import RPNHead
from .bbox_head import BBoxHead
from .rcnn_head import RCNNHead
from .retina_head import RetinaHead
from .fcos_head import FCOSHead

__all__ = ['AnchorHead', 'RPNHead', 'BBoxHead', 'RCNNHead', 'RetinaHead', 'FCOSHead']

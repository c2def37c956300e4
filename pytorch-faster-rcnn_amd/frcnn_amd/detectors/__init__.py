from .cascade_rcnn import CascadeRCNN
from .retinanet import RetinaNet
from .fcos import FCOS

__all__ = ['CascadeRCNN', 'RetinaNet', 'FCOS']

from .cascade_rcnn import CascadeRCNN
from .retinanet import RetinaNet

__all__ = ['CascadeRCNN', 'RetinaNet']

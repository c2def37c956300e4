"""frcnn_amd — MI355X-native (gfx950) Faster R-CNN detection hot path.

Reference: pengfeidip/pytorch-faster-rcnn (`lib/`).  The module names mirror
the reference's (`anchor`, `region`, `bbox`, `utils`, `builder`, `heads`,
`detectors`) so its detectors and configs run unchanged; the detection
primitives run as hand-written HIP kernels in libfrcnn_amd.so (C-ABI in
include/frcnn_amd.h).  There is no CPU fallback.
"""
from . import _lib
from .ops import set_sampler_mode, sampler_mode

__all__ = ['set_sampler_mode', 'sampler_mode', 'load_library']


def load_library():
    return _lib.load()

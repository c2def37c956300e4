"""ctypes loader of the TOOLS-ONLY library tools/lib/libfrcnn_tools.so (see
tools/build_tools.py): the product ABI (frcnn_amd._lib.SIGNATURES) plus the RoIAlign
laboratory entry points of tools/csrc/frcnn_tools.h.  Used by tools/bench_roi_align.py, tools/bench_nms.py and
tests/test_abi.py only; never by the product."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'pytorch-faster-rcnn_amd'))
from frcnn_amd import _lib  # noqa: E402

LIB_PATH = os.path.join(HERE, 'lib', 'libfrcnn_tools.so')
P, c_i32, c_i64, c_f32, c_vp, c_size = ctypes.POINTER, _lib.c_i32, _lib.c_i64, _lib.c_f32, _lib.c_vp, _lib.c_size
_RA = [c_i32, P(c_vp), P(c_i32), P(c_i64), P(c_f32), c_i32, c_i32, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i32]
TOOL_SIGNATURES = {
    'frh_roi_align_fwd_variant': (c_i32, [c_i32] + _RA + [c_vp, c_vp, c_size, c_vp]),
    'frh_roi_align_bwd_variant': (c_i32, [c_i32, c_i32, P(c_vp), P(c_vp), P(c_i32), P(c_i64), P(c_f32), c_i32, c_i32,
                                          c_vp, c_vp, c_i64, c_vp, c_vp, c_vp]),
    'frh_roi_align_workspace': (c_size, [c_i64]),
    'frh_nms_sorted_stamped': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_i32, ctypes.c_double, c_i32, c_vp, c_i64, c_vp,
                                       c_vp, c_size, c_vp, c_vp]),
    'frh_nms_fused_flag_bytes': (c_size, [c_i32, c_i32]),
    'frh_nms_fused_stamped': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_i32, ctypes.c_double, c_i32, c_vp, c_i64, c_vp,
                                      c_vp, c_vp, c_size, c_vp, c_vp]),
    'frh_rpn_proposals_launches': _lib.SIGNATURES['frh_rpn_proposals_strided'],
    'frh_rpn_proposals_nms2': _lib.SIGNATURES['frh_rpn_proposals_strided'],
    'frh_rpn_proposals_merge_launch': _lib.SIGNATURES['frh_rpn_proposals_strided'],
    'frh_sample_random_launches': _lib.SIGNATURES['frh_sample_random'],
    'frh_rpn_proposals_stamped': (c_i32, _lib.SIGNATURES['frh_rpn_proposals_strided'][1][:-1] + [c_vp, c_vp]),
    'frh_rpn_proposals_nms_stamped': (c_i32, _lib.SIGNATURES['frh_rpn_proposals_strided'][1][:-1] + [c_vp, c_vp]),
    'frh_sample_random_stamped': (c_i32, _lib.SIGNATURES['frh_sample_random'][1][:-1] + [c_vp, c_vp]),
}
_lib_t = None


def load():
    global _lib_t
    if _lib_t is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError('{} is missing: run python tools/build_tools.py'.format(LIB_PATH))
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in list(_lib.SIGNATURES.items()) + list(TOOL_SIGNATURES.items()):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lib_t = lib
    return _lib_t

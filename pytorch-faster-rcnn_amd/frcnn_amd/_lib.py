"""ctypes binding of the C-ABI in include/frcnn_amd.h (libfrcnn_amd.so).

This is the only way the Python host code reaches the HIP kernels.  There is
no CPU fallback: if the library is missing, or a tensor is not on a HIP
device, every op raises.  Symbols are declared with full argtypes so a
signature drift between header and binding fails at call time, not silently.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libfrcnn_amd.so')

c_i32, c_i64, c_f32, c_f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double
c_u64, c_size, c_vp = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
P = ctypes.POINTER

# name -> (restype, argtypes); mirrors include/frcnn_amd.h one to one
SIGNATURES = {
    'frh_abi_version': (c_i32, []),
    'frh_last_error': (ctypes.c_char_p, []),
    'frh_anchor_grid': (c_i32, [c_i32, P(c_i32), P(c_f32), c_vp, c_vp, c_i32, c_i32, c_vp, c_i64, c_vp]),
    'frh_inside_mask': (c_i32, [c_vp, c_i64, c_i32, P(c_i32), P(c_i32), c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    'frh_iou_table': (c_i32, [c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    'frh_elem_iou': (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp]),
    'frh_maxiou_assign_zero_bytes': (c_size, [c_i32, c_i32]),
    'frh_maxiou_assign_workspace': (c_size, [c_i32, c_i32, c_i64]),
    'frh_maxiou_assign': (c_i32, [c_i32, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp,
                                  c_f32, c_f32, c_f32, c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, c_vp, c_size,
                                  c_vp]),
    'frh_sample_workspace': (c_size, [c_i32, c_i64]),
    'frh_sample_zero_bytes': (c_size, [c_i32]),
    'frh_sample_candidates': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_size,
                                      c_vp]),
    'frh_sample_apply': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp,
                                 c_vp, c_vp]),
    'frh_sample_random': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_u64, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_size, c_vp]),
    'frh_anchor_target_workspace': (c_size, [c_i32, c_i64]),
    'frh_anchor_target': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                                  c_vp, c_i64, P(c_f32), P(c_f32), c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                  c_vp, c_vp, c_i64, c_vp, c_vp, c_size, c_vp]),
    'frh_gather_level_outputs': (c_i32, [c_i32, P(c_vp), P(c_i64), P(c_i64), c_i32, c_i64, c_vp, c_vp, c_vp,
                                         c_i64, c_vp]),
    'frh_scatter_level_grads': (c_i32, [c_i32, P(c_vp), P(c_i64), P(c_i64), c_i32, c_i64, c_vp, c_vp, c_vp,
                                        c_i64, c_vp]),
    'frh_gather_level_outputs_strided': (c_i32, [c_i32, P(c_vp), P(c_i64), P(c_i32), P(c_i64), c_i32, c_i32, c_i64,
                                                 c_vp, c_vp, c_vp, c_i64, c_vp]),
    'frh_scatter_level_grads_strided': (c_i32, [c_i32, P(c_vp), P(c_i64), P(c_i32), P(c_i64), c_i32, c_i32, c_i64,
                                                c_vp, c_vp, c_vp, c_i64, c_vp]),
    'frh_prepend_gt_labels': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp]),
    'frh_bbox_target_workspace': (c_size, [c_i32, c_i64]),
    'frh_bbox_target': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64,
                                c_vp, c_i64, P(c_f32), P(c_f32), c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                c_vp, c_i64, c_vp, c_vp, c_size, c_vp]),
    'frh_bbox2param': (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, P(c_f32), P(c_f32), c_vp, c_i64, c_vp]),
    'frh_param2bbox': (c_i32, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i32, P(c_f32), P(c_f32), c_i32, c_f32, c_f32,
                               c_vp, c_i64, c_vp]),
    'frh_rpn_proposals_workspace': (c_size, [c_i32, c_i32, P(c_i32), c_i32, c_i32]),
    'frh_rpn_proposals_nms_view': (c_i32, [c_i32, c_i32, P(c_i32), c_i32, c_i32, P(ctypes.c_int64)]),
    'frh_rpn_proposals': (c_i32, [c_i32, c_i32, P(c_vp), P(c_vp), P(c_i32), c_i32, c_i32, c_vp, c_i64,
                                  P(c_f32), P(c_f32), P(c_f32), P(c_f32), c_i32, c_i32, c_i32, c_f64, c_vp,
                                  c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    'frh_rpn_proposals_strided': (c_i32, [c_i32, c_i32, P(c_vp), P(c_vp), P(c_i64), P(c_i64), P(c_i32), c_i32, c_i32,
                                          c_vp, c_i64, P(c_f32), P(c_f32), P(c_f32), P(c_f32), c_i32, c_i32, c_i32,
                                          c_f64, c_vp, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    'frh_nms_workspace': (c_size, [c_i32, c_i32]),
    'frh_nms_sorted': (c_i32, [c_i32, c_vp, c_i64, c_vp, c_i32, c_f64, c_i32, c_vp, c_i64, c_vp, c_vp, c_size,
                               c_vp]),
    'frh_mcnms_workspace': (c_size, [c_i32, c_i32, c_i64]),
    'frh_mcnms_prepare': (c_i32, [c_i32, c_i32, c_i64, c_vp, c_vp, c_i64, c_i32, c_vp, c_i64, c_vp, c_i64, c_i32,
                                  c_vp, c_i64, c_vp, c_i32, c_i32, c_f32, c_vp, c_size, c_vp, c_vp]),
    'frh_mcnms_nms_workspace': (c_size, [c_i32, c_i32, c_i32, c_i64]),
    'frh_mcnms_finish': (c_i32, [c_i32, c_i32, c_i64, c_i32, c_i64, c_vp, c_i64, c_i32, c_vp, c_i64, c_i32, c_i32, c_f64,
                                 c_i32, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_size, c_vp, c_size, c_vp]),
    'frh_roi_level_map': (c_i32, [c_vp, c_i64, c_f32, c_i32, c_vp, c_vp]),
    'frh_roi_rows': (c_i32, [c_i32, c_vp, c_i64, c_i64, c_i32, P(c_i64), c_f32, c_i32, c_vp, c_vp, c_vp]),
    'frh_roi_rows_dev': (c_i32, [c_i32, c_vp, c_i64, c_i64, c_vp, c_f32, c_i32, c_vp, c_vp, c_vp]),
    'frh_roi_align_fwd': (c_i32, [c_i32, P(c_vp), P(c_i32), P(c_f32), c_i32, c_i32, c_i32, c_vp, c_vp, c_i64,
                                  c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    'frh_roi_align_bwd': (c_i32, [c_i32, P(c_vp), P(c_i32), P(c_f32), c_i32, c_i32, c_i32, c_vp, c_vp, c_i64,
                                  c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    'frh_roi_align_fwd_strided': (c_i32, [c_i32, P(c_vp), P(c_i32), P(c_i64), P(c_f32), c_i32, c_i32, c_vp,
                                          c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    'frh_roi_align_fwd_strided_timed': (c_i32, [c_i32, P(c_vp), P(c_i32), P(c_i64), P(c_f32), c_i32, c_i32, c_vp,
                                                c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp,
                                                c_vp]),
    'frh_roi_align_bwd_strided': (c_i32, [c_i32, P(c_vp), P(c_i32), P(c_i64), P(c_f32), c_i32, c_i32, c_vp,
                                          c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp]),
    'frh_roi_align_bwd_fixed': (c_i32, [c_i32, P(c_vp), P(c_vp), P(c_i32), P(c_i64), P(c_f32), c_i32, c_i32, c_vp,
                                        c_vp, c_i64, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp]),
    'frh_roi_pool_fwd': (c_i32, [c_vp, P(c_i64), c_i32, c_i32, c_i32, c_f32, c_vp, c_i64, c_i32, c_i32, c_vp,
                                 c_vp, c_vp]),
    'frh_roi_pool_bwd': (c_i32, [c_vp, P(c_i64), c_i32, c_i32, c_i32, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp,
                                 c_vp]),
    'frh_atss_workspace': (c_size, [c_i32, c_i32, c_i32, c_i32, c_i64]),
    'frh_bn_act': (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_i64, c_i32, c_i64, c_i32, c_vp]),
    'frh_bn_act_maxpool': (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_i64, c_i32, c_i32, c_i32, c_vp]),
    'frh_loss_workspace': (c_size, []),
    'frh_fpn_merge_nhwc': (c_i32, [c_vp, P(c_i64), c_vp, c_vp, c_i32, c_i32, c_vp, c_i32, c_i32, c_i32, c_i32, c_vp]),
    'frh_bias_act_nhwc': (c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, c_vp]),
    'frh_image_preprocess': (c_i32, [c_vp, c_i32, P(c_i64), P(c_i32), P(c_i32), P(c_i32), P(c_f32), P(c_f32), c_i32,
                                     c_vp, c_i32, c_i32, c_vp]),
    'frh_cls_loss_fwd': (c_i32, [c_i32, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_f32, c_f32, c_vp, c_vp,
                                 c_vp, c_size, c_vp]),
    'frh_cls_loss_bwd': (c_i32, [c_i32, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_f32, c_f32, c_vp, c_vp,
                                 c_i64, c_i64, c_vp]),
    'frh_smooth_l1_fwd': (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_f32,
                                  c_vp, c_vp, c_vp, c_size, c_vp]),
    'frh_smooth_l1_bwd': (c_i32, [c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_f32,
                                  c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    'frh_det_loss_fwd': (c_i32, [c_i32, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_f32, c_f32, c_f32, c_f32,
                                 c_vp, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_i64, c_f32,
                                 c_f32, c_f32, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    'frh_atss_assign': (c_i32, [c_i32, c_i32, P(c_i32), P(c_f32), c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_i32,
                                c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
}

ABI_VERSION = 3
_lib = None


def load():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError('frcnn_amd: {} is missing; run __graft_entry__.build() '
                           '(hipcc --offload-arch=gfx950)'.format(LIB_PATH))
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.frh_abi_version() != ABI_VERSION:
        raise RuntimeError('frcnn_amd: ABI version mismatch')
    _lib = lib
    return lib


def call(name, *args):
    """Invoke an entry point; a non-zero status raises RuntimeError with frh_last_error()."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != 0:
        msg = lib.frh_last_error().decode(errors='replace')
        raise RuntimeError('{} failed ({}): {}'.format(name, st, msg))


def query(name, *args):
    return getattr(load(), name)(*args)


def ptr(t):
    """Device pointer of a HIP tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError('frcnn_amd ops run on the HIP device only (got a {} tensor)'.format(t.device))
    return ctypes.c_void_p(t.data_ptr())


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def i32_array(vals):
    return (c_i32 * len(vals))(*[int(v) for v in vals])


def i64_array(vals):
    return (c_i64 * len(vals))(*[int(v) for v in vals])


def f32_array(vals):
    return (c_f32 * len(vals))(*[float(v) for v in vals])


def ptr_array(ts):
    return (c_vp * len(ts))(*[t.data_ptr() for t in ts])


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)

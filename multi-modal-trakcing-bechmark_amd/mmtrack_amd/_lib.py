"""ctypes binding of the in-tree C-ABI library ``libmmtrack.so`` (include/mmtrack.h).

The product path has no fallback: if the HIP library is missing or fails to load, importing
this module raises, so nothing can silently run on the CPU.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MMTRACK_LIB", os.path.join(_HERE, "libmmtrack.so"))

MMT_OK, MMT_E_ARG, MMT_E_STATE, MMT_E_HIP, MMT_E_WEIGHTS, MMT_E_BOX = 0, -1, -2, -3, -4, -5
MMT_MODEL_VIPT, MMT_MODEL_OSTRACK = 0, 1
MMT_PROMPT_NONE, MMT_PROMPT_SHAW, MMT_PROMPT_DEEP = 0, 1, 2


class MmtConfig(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int),
        ("prompt_type", ctypes.c_int),
        ("in_chans", ctypes.c_int),
        ("template_size", ctypes.c_int),
        ("search_size", ctypes.c_int),
        ("template_factor", ctypes.c_double),
        ("search_factor", ctypes.c_double),
        ("n_ce", ctypes.c_int),
        ("ce_loc", ctypes.c_int * 12),
        ("ce_keep_ratio", ctypes.c_double * 12),
        ("ce_template_index", ctypes.c_int),
        ("head_channels", ctypes.c_int),
        ("max_batch", ctypes.c_int),
        ("use_graphs", ctypes.c_int),
        ("debug_outputs", ctypes.c_int),
        ("precision", ctypes.c_int),
    ]


class MmtDimpParams(ctypes.Structure):
    _fields_ = [
        ("feat_stride", ctypes.c_float),
        ("log_step_length", ctypes.c_float),
        ("filter_reg", ctypes.c_float),
        ("min_filter_reg", ctypes.c_float),
        ("alpha_eps", ctypes.c_float),
        ("bin_displacement", ctypes.c_float),
        ("num_dist_bins", ctypes.c_int),
        ("label_w", ctypes.c_float * 128),
        ("mask_w", ctypes.c_float * 128),
        ("spatial_w", ctypes.c_float * 128),
    ]


class MmtPatchTf(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int),
        ("top", ctypes.c_int),
        ("left", ctypes.c_int),
        ("blur_ry", ctypes.c_int),
        ("blur_rx", ctypes.c_int),
        ("blur_fy", ctypes.c_float * 33),
        ("blur_fx", ctypes.c_float * 33),
        ("affine", ctypes.c_double * 6),
    ]


MMT_DIMP_MEMORY = 50


class MmtDimpState(ctypes.Structure):
    _fields_ = [
        ("pos", ctypes.c_float * 2), ("target_sz", ctypes.c_float * 2), ("base_target_sz", ctypes.c_float * 2),
        ("image_sz", ctypes.c_float * 2), ("target_scale", ctypes.c_float), ("min_scale_factor", ctypes.c_float),
        ("max_scale_factor", ctypes.c_float), ("frame_num", ctypes.c_int), ("num_init", ctypes.c_int),
        ("num_stored", ctypes.c_int), ("prev_replace", ctypes.c_int), ("coords", ctypes.c_float * 4),
        ("sample_weights", ctypes.c_float * MMT_DIMP_MEMORY), ("target_boxes", (ctypes.c_float * 4) * MMT_DIMP_MEMORY),
    ]


class MmtDimpFrame(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("stride", ctypes.c_int64), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("C", ctypes.c_int), ("pad_", ctypes.c_int)]


class MmtDimpTrackParams(ctypes.Structure):
    _fields_ = [
        ("img_sample_sz", ctypes.c_float * 2), ("feature_sz", ctypes.c_float * 2), ("kernel_size", ctypes.c_float * 2),
        ("target_not_found_threshold", ctypes.c_double), ("uncertain_threshold", ctypes.c_double),
        ("hard_sample_threshold", ctypes.c_double), ("distractor_threshold", ctypes.c_double),
        ("hard_negative_threshold", ctypes.c_double), ("target_neighborhood_scale", ctypes.c_double),
        ("dispalcement_scale", ctypes.c_double), ("target_inside_ratio", ctypes.c_double),
        ("low_score_opt_threshold", ctypes.c_double), ("learning_rate", ctypes.c_double),
        ("hard_negative_learning_rate", ctypes.c_double), ("init_samples_minimum_weight", ctypes.c_double),
        ("sample_memory_size", ctypes.c_int), ("train_sample_interval", ctypes.c_int), ("train_skipping", ctypes.c_int),
        ("net_opt_update_iter", ctypes.c_int), ("net_opt_hn_iter", ctypes.c_int), ("net_opt_low_iter", ctypes.c_int),
        ("update_classifier", ctypes.c_int),
    ]


class MmtConvGroup(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("w_hi", ctypes.c_void_p), ("w_lo", ctypes.c_void_p), ("w_scale", ctypes.c_float),
                ("bias", ctypes.c_void_p), ("resid", ctypes.c_void_p), ("y", ctypes.c_void_p), ("x_max", ctypes.c_void_p),
                ("x_scale", ctypes.c_float), ("y_max", ctypes.c_void_p), ("flags", ctypes.c_int)]


class MmtConvDs(ctypes.Structure):
    _fields_ = [("x2", ctypes.c_void_p), ("x2_max", ctypes.c_void_p), ("x2_scale", ctypes.c_float)]


class MmtDimpResult(ctypes.Structure):
    _fields_ = [("box", ctypes.c_float * 4), ("max_score", ctypes.c_float), ("flag", ctypes.c_int),
                ("num_iter", ctypes.c_int), ("n_samples", ctypes.c_int), ("replace_ind", ctypes.c_int),
                ("tv", ctypes.c_float * 2), ("sample_pos", ctypes.c_float * 2), ("sample_scale", ctypes.c_float),
                ("aux", ctypes.c_int * 4)]


ABI_VERSION = 5   # include/mmtrack.h MMT_ABI_VERSION

# every symbol include/mmtrack.h declares: name -> (restype, argtypes)
_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double
_F = ctypes.c_float
_I64 = ctypes.c_int64
SIGNATURES = {
    "mmt_create": (_I, [ctypes.POINTER(MmtConfig), _I, ctypes.POINTER(_P)]),
    "mmt_destroy": (None, [_P]),
    "mmt_last_error": (ctypes.c_char_p, [_P]),
    "mmt_version": (ctypes.c_char_p, []),
    "mmt_abi_version": (_I, []),
    "mmt_set_tensor": (_I, [_P, ctypes.c_char_p, _P, ctypes.POINTER(_I64), _I]),
    "mmt_finalize": (_I, [_P]),
    "mmt_num_expected_keys": (_I, [_P]),
    "mmt_expected_key": (ctypes.c_char_p, [_P, _I]),
    "mmt_initialize": (_I, [_P, _I, _P, _I, _I, _I, _I64, _I, ctypes.POINTER(_D)]),
    "mmt_track": (_I, [_P, _I, _P, _I, _I, _I, _I64, _I, ctypes.POINTER(_D), ctypes.POINTER(_F)]),
    "mmt_track_batch": (_I, [_P, _I, _I, ctypes.POINTER(_P), ctypes.POINTER(_I), ctypes.POINTER(_I), _I,
                             ctypes.POINTER(_I64), _I, ctypes.POINTER(_D), ctypes.POINTER(_F)]),
    "mmt_track_batch_submit": (_I, [_P, _I, _I, ctypes.POINTER(_P), ctypes.POINTER(_I), ctypes.POINTER(_I), _I,
                                    ctypes.POINTER(_I64), _I, ctypes.POINTER(_I64)]),
    "mmt_track_batch_fetch": (_I, [_P, _I64, ctypes.POINTER(_D), ctypes.POINTER(_F)]),
    "mmt_get_state": (_I, [_P, _I, ctypes.POINTER(_D)]),
    "mmt_set_state": (_I, [_P, _I, ctypes.POINTER(_D)]),
    "mmt_debug_fetch": (_I, [_P, ctypes.c_char_p, _I, _P, ctypes.c_size_t]),
    "mmt_debug_force_ce": (_I, [_P, _I, _P, ctypes.c_size_t]),
    "mmt_timing_enable": (_I, [_P, ctypes.c_char_p]),
    "mmt_timing_read": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_D), ctypes.POINTER(_D), ctypes.POINTER(_D)]),
    "mmt_xcorr": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _P]),
    "mmt_siamfc_crop": (_I, [_P, _I, _I, _I, ctypes.c_int64, _I, _P, _P, _P, _P, _I, _P, _P]),
    "mmt_siamfc_crop_nhwc": (_I, [_P, _I, _I, _I, ctypes.c_int64, _I, _P, _P, _P, _P, _I, _P, _P]),
    "mmt_xcorr_nhwc": (_I, [_P, ctypes.c_int64, _P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _P]),
    "mmt_siamfc_response": (_I, [_P, _I, _I, _I, ctypes.c_float, ctypes.c_double, _P, ctypes.c_double, _P, _P, _P]),
    "mmt_rgbd_workspace_bytes": (ctypes.c_size_t, []),
    "mmt_rgbd_assemble": (_I, [_P, ctypes.c_int64, _P, ctypes.c_int64, _I, _I, _I, _P, _P, ctypes.c_int64, _P,
                               ctypes.c_size_t, _P]),
    "mmt_set_frame_stream": (_I, [_P, _P]),
    "mmt_conv2d_f32": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _P]),
    "mmt_conv2d_f32_ld": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _I, _I, _P]),
    "mmt_conv_max_words": (ctypes.c_size_t, []),
    "mmt_conv2d_f16x3": (_I, [_P, _I, _I, _I, _I, _P, _P, _F, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P, _F, _P, _I, _P]),
    "mmt_conv2d_f16x3_ws_bytes": (ctypes.c_size_t, [_I, _I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "mmt_conv2d_f16x3_groups": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, ctypes.c_size_t, _P]),
    "mmt_conv2d_f16x3_ds_groups": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, ctypes.c_size_t, _P]),
    "mmt_maxpool2d_f32": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "mmt_image_normalize": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "mmt_image_normalize4": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "mmt_instance_l2norm_ws_bytes": (ctypes.c_size_t, [_I, _I, _I]),
    "mmt_instance_l2norm": (_I, [_P, _I, _I, _I, _I, _F, _F, _P, _P, _P, _P]),
    "mmt_prroi_pool": (_I, [_P, _I, _I, _I, _I, _P, _F, _I, _I, _P, _P]),
    "mmt_sample_patch": (_I, [_P, _I, _I, _I, ctypes.c_int64, _P, _I, _I, _P, _P]),
    "mmt_patch_transform": (_I, [_P, _I, _I, _I, ctypes.POINTER(MmtPatchTf), _I, _I, _P, _P]),
    "mmt_rgbx_merge": (_I, [_P, ctypes.c_int64, _P, ctypes.c_int64, _I, _I, _I, _P, ctypes.c_int64, _P]),
    "mmt_dimp_workspace_bytes": (ctypes.c_size_t, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "mmt_dimp_apply_filter": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "mmt_dimp_feat_transpose": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "mmt_dimp_optimize": (_I, [_P, _I, _I, _I, _I, _I, _P, _I, _I, _P, _P, ctypes.POINTER(MmtDimpParams), _I, _P,
                               ctypes.c_size_t, _P, _P]),
    "mmt_dimp_optimize_strided": (_I, [_P, _I64, _I64, _I, _I, _I, _I, _I, _P, _I, _I, _P, _I64, _I64, _P, _I64, _I64,
                                   ctypes.POINTER(MmtDimpParams), _I, _P, ctypes.c_size_t, _P]),
    "mmt_dimp_state_bytes": (ctypes.c_size_t, []),
    "mmt_dimp_track_optimize_ws_bytes": (ctypes.c_size_t, [_I, _I, _I, _I, _I, _I, _I]),
    "mmt_dimp_track_optimize": (_I, [_P, _I, _P, _P, _I, _I, _I, _P, _I, _I, ctypes.POINTER(MmtDimpParams), _I, _P,
                                     ctypes.c_size_t, _P]),
    "mmt_dimp_track_sample": (_I, [_P, _P, _I, ctypes.POINTER(MmtDimpTrackParams), _I, _I, _P, _P]),
    "mmt_dimp_track_sample_norm4": (_I, [_P, _P, _I, ctypes.POINTER(MmtDimpTrackParams), _I, _I, _P, _P, _P, _P, _P,
                                         ctypes.c_int64, _P]),
    "mmt_dimp_track_update": (_I, [_P, _I, _P, _I, _I, ctypes.POINTER(MmtDimpTrackParams), _P, _I64, _P, _P, _P]),
    "mmt_dimp_track_update_pinned": (_I, [_P, _I, _P, _I, _I, ctypes.POINTER(MmtDimpTrackParams), _P, _I64, _P, _P, _P,
                                          _P]),
    "mmt_host_alloc": (_P, [ctypes.c_size_t]),
    "mmt_host_free": (None, [_P]),
    "mmt_gemm_stamps": (_I, [_P]),
    "mmt_op_gemm": (_I, [_P, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _I, _I, _I, _I, _I, _I, _I, _P]),
    "mmt_gemm_force_config": (_I, [_I]),
    "mmt_op_attention": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "mmt_op_layernorm": (_I, [_P, _P, _P, _P, _P, _I, _P]),
    "mmt_op_gemm_f16x3": (_I, [_P, _P, _I64, _P, _P, _I64, _P, _P, _P, _I64, _P, _I64, _I, _I, _I, _I, _F, _F, _I, _I,
                               _P]),
    "mmt_op_attention_f16x3": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _F, _P]),
}

_lib = None


def load():
    """Load libmmtrack.so (raises ImportError if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libmmtrack.so not found at {LIB_PATH}; build it with "
                          f"`make -C multi-modal-trakcing-bechmark_amd/csrc` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mmt_abi_version() != ABI_VERSION:   # a stale library whose argument conventions differ
        raise ImportError(f"libmmtrack.so ABI {lib.mmt_abi_version()} != {ABI_VERSION} (include/mmtrack.h "
                          f"MMT_ABI_VERSION); rebuild it")
    _lib = lib
    return lib

"""ctypes binding of libgsr_hip.so (the C ABI declared in include/gsr.h).

There is no fallback: if the gfx950 library is missing or fails to load, importing the
rasterizer's _C module raises, so a GPU run can never silently use another path.
"""
from __future__ import annotations

import ctypes
import os

LIB_PATH = os.environ.get("GSR_LIBRARY") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgsr_hip.so")

RESIZE_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_i64 = ctypes.c_int64



class AdamGroup(ctypes.Structure):
    """gsr_adam_group (include/gsr_train.h)."""
    _fields_ = [("param", _vp), ("grad", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp), ("width", _i64),
                ("step_size", _f), ("bias_correction2_sqrt", _f), ("row_stride", _i64)]


class RowGroup(ctypes.Structure):
    """gsr_row_group (include/gsr_densify.h)."""
    _fields_ = [("param", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp), ("width", _i64)]


class TrainStepArgs(ctypes.Structure):
    """gsr_train_step_args (include/gsr_train.h)."""
    _fields_ = [("P", _i64), ("D", _i), ("M", _i), ("width", _i), ("height", _i),
                ("xyz", _vp), ("features", _vp), ("opacity", _vp), ("scaling", _vp), ("rotation", _vp),
                ("xyz_grad", _vp), ("features_grad", _vp), ("opacity_grad", _vp), ("scaling_grad", _vp),
                ("rotation_grad", _vp), ("exposure", _vp), ("exposure_grad", _vp), ("n_images", _i),
                ("image_index", _i), ("viewmatrix", _vp), ("projmatrix", _vp), ("campos", _vp), ("tan_fovx", _f),
                ("tan_fovy", _f), ("background", _vp), ("gt", _vp), ("alpha_mask", _vp), ("mono_invdepth", _vp),
                ("depth_mask", _vp), ("depth_weight", _f), ("lambda_dssim", ctypes.c_double),
                ("max_radii2D", _vp), ("xyz_gradient_accum", _vp), ("denom", _vp), ("n_groups", _i),
                ("groups", ctypes.POINTER(AdamGroup)), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("exposure_group", ctypes.POINTER(AdamGroup)),
                ("exposure_beta1", ctypes.c_double), ("exposure_beta2", ctypes.c_double),
                ("exposure_eps", ctypes.c_double), ("skybox_rows", _i64), ("scaffold_rows", _i64),
                ("max_scale", _f), ("losses", _vp), ("stream", _vp), ("depth_only", _i),
                ("depth_dens_weight", ctypes.c_double), ("skip_gaussian_step", _i)]


# exported symbol -> (restype, argtypes); must match include/gsr.h, gsr_train.h, gsr_hier.h, gsr_knn.h, gsr_densify.h
SIGNATURES = {
    "gsr_rasterize_forward": (_i, [RESIZE_FN, RESIZE_FN, RESIZE_FN, _vp, _i, _i, _i, _vp, _i, _i,
                                   _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _f, _f,
                                   _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp,
                                   ctypes.POINTER(_i64)]),
    "gsr_rasterize_forward_ex": (_i, [RESIZE_FN, RESIZE_FN, RESIZE_FN, _vp, _i, _i, _i, _vp, _i, _i,
                                      _vp, _vp, _vp, _vp, _vp, _f, _vp, _vp, _vp, _vp, _vp, _f, _f,
                                      _i, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp,
                                      ctypes.POINTER(_i64), ctypes.c_uint]),
    "gsr_rasterize_backward": (_i, [RESIZE_FN, _vp, _i, _i, _i, _i64, _vp, _i, _i, _vp, _vp, _vp, _vp, _f,
                                    _vp, _vp, _vp, _vp, _vp, _f, _f, _vp, _vp, _vp, _vp, _vp, _vp,
                                    _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp]),
    "gsr_mark_visible": (_i, [_i, _vp, _vp, _vp, _vp, _vp]),
    "gsr_set_profiling": (_i, [_i]),
    "gsr_stage_times_ms": (_i, [ctypes.POINTER(_f), _i]),
    "gsr_forward_stats": (_i, [ctypes.POINTER(_i64), _i]),
    "gsr_reset_capacity_hint": (_i, []),
    "gsr_set_bwd_segment": (_i, [_i]),
    "gsr_set_fwd_segment": (_i, [_i]),
    "gsr_set_split_gate": (_i, [_i]),
    "gsr_set_live_list": (_i, [_i]),
    "gsr_set_fwd_split_min": (_i, [_i]),
    "gsr_set_fwd_spin_limits": (_i, [_i64, _i64]),
    "gsr_segment_layout_check": (_i, [ctypes.c_int64, _i, _i, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "gsr_frame_stats": (_i, [_vp, _i, _i, _i, ctypes.POINTER(_i64), _i]),
    "gsr_blend_stats": (_i, [ctypes.POINTER(_i64), _i, _i]),
    "gsr_fwd_pool_stats": (_i, [ctypes.POINTER(_i64), _i, _i]),
    "gsr_debug_trace": (_i, [ctypes.POINTER(_i64), _i, _i]),
    "gsr_kstamp_read": (_i, [ctypes.POINTER(ctypes.c_uint64), _i]),
    "gsr_set_true_scale_gradient": (_i, [_i]),
    "gsr_set_deterministic": (_i, [_i]),
    "gsr_set_binning": (_i, [_i]),
    "gsr_abi_version": (_i, []),
    "gsr_last_error": (ctypes.c_char_p, []),
    "gsr_build_info": (ctypes.c_char_p, []),
    # include/gsr_train.h
    "gsr_l1_ssim_scratch_bytes": (ctypes.c_size_t, [_i, _i, _i]),
    "gsr_l1_ssim_forward": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "gsr_l1_ssim_backward": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "gsr_l1_ssim_forward_with_map": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _vp, _vp]),
    "gsr_l1_ssim_backward_from_map": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "gsr_photo_loss_forward": (_i, [_vp, _vp, _i, _i, _i, ctypes.c_double, _vp, _vp, _vp, _vp]),
    "gsr_photo_loss_backward": (_i, [_vp, _vp, _vp, _i, _i, _i, ctypes.c_double, _vp, _vp, _vp]),
    "gsr_sparse_adam_step": (_i, [_i, ctypes.POINTER(AdamGroup), _i64, _vp, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_double, _vp, _vp]),
    "gsr_densify_stats": (_i, [_i64, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsr_activate_forward": (_i, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsr_activate_backward": (_i, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsr_shrink_scales": (_i, [_i64, _i64, _vp, _f, _vp]),
    "gsr_depth_l1_scratch_bytes": (ctypes.c_size_t, [_i64]),
    "gsr_depth_l1_forward": (_i, [_vp, _vp, _vp, _i64, _f, _vp, _vp, _vp]),
    "gsr_depth_l1_backward": (_i, [_vp, _vp, _vp, _i64, _f, _vp, _vp, _vp]),
    "gsr_depth_only_scratch_bytes": (ctypes.c_size_t, [_i64]),
    "gsr_depth_only_loss_forward": (_i, [_vp, _vp, _vp, _i64, _f, ctypes.c_double, _vp, _vp, _vp]),
    "gsr_depth_only_loss_backward": (_i, [_vp, _vp, _vp, _i64, _f, ctypes.c_double, _vp, _vp, _vp]),
    "gsr_exposure_forward": (_i, [_vp, _vp, _i64, _vp, _vp]),
    "gsr_exposure_scratch_bytes": (ctypes.c_size_t, [_i64]),
    "gsr_exposure_backward": (_i, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "gsr_train_ctx_create": (_vp, []),
    "gsr_train_ctx_destroy": (None, [_vp]),
    "gsr_train_ctx_stats": (_i, [_vp, ctypes.POINTER(_i64), _i]),
    "gsr_train_step": (_i, [_vp, ctypes.POINTER(TrainStepArgs), ctypes.POINTER(_i64)]),
    # include/gsr_hier.h
    "gsr_interpolate_cut_forward": (_i, [_i64, _i, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                         _vp, _vp, _vp]),
    "gsr_expand_to_size_scratch_bytes": (ctypes.c_size_t, [_i64]),
    "gsr_expand_to_size": (_i, [_i64, _vp, _vp, _f, _vp, _vp, _vp, _vp, _i64, _vp, ctypes.c_size_t,
                                ctypes.POINTER(_i64), _vp]),
    "gsr_interpolation_weights": (_i, [_i64, _vp, _f, _vp, _vp, _f, _f, _f, _vp, _vp, _vp]),
    "gsr_densify_scratch_bytes": (ctypes.c_size_t, [_i64]),
    "gsr_densify_plan": (_i, [_i64, _i64, _vp, _vp, _vp, _vp, _f, _f, _f, _vp, _vp, _vp]),
    "gsr_densify_apply": (_i, [_i64, _i, ctypes.POINTER(RowGroup), ctypes.POINTER(RowGroup), _i, _i, _i, _vp, _i64,
                               _vp, _i64, _vp]),
    "gsr_knn_scratch_bytes": (ctypes.c_size_t, [_i64]),
    "gsr_knn_mean_dist2": (_i, [_i64, _vp, _vp, _vp, _vp]),
    "gsr_interpolate_cut_backward": (_i, [_i64, _i, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                          _vp, _vp, _vp, _vp, _vp]),
    "gsr_interpolate_cut_forward_act": (_i, [_i64, _i, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp,
                                             _vp, _vp, _vp, _vp, _vp]),
    "gsr_interpolate_cut_backward_act": (_i, [_i64, _i, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp,
                                              _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gsr_zero_grad_rows": (_i, [_i, ctypes.POINTER(_vp), ctypes.POINTER(_i64), _i64, _i64, _vp, _i64, _vp]),
}

ABI_VERSION = 6
_lib = None


class RasterizerLibraryError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load and type the library; raises RasterizerLibraryError if absent or mismatched."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RasterizerLibraryError(
            f"gfx950 rasterizer library not found at {path}; build it with "
            f"`python street-sparse-3dgs_amd/build_hip.py` (or __graft_entry__.build())")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover - depends on the host
        raise RasterizerLibraryError(f"failed to load {path}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gsr_abi_version() != ABI_VERSION:
        raise RasterizerLibraryError("libgsr_hip.so ABI version mismatch; rebuild it")
    _lib = lib
    return lib


def last_error() -> str:
    return load().gsr_last_error().decode("utf-8", "replace")

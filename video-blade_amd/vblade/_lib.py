"""ctypes binding of libvblade_hip.so (the C ABI declared in include/vblade.h).

This is the "reference-side binding a maintainer would add" (INTEGRATION.md): the reference is
Python, so its FFI for this path is a ctypes stub over the C ABI. There is deliberately no
fallback: if the HIP library is missing the import of any op raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VBLADE_LIB", os.path.join(_HERE, "libvblade_hip.so"))

VB_OK, VB_ERR_INVALID, VB_ERR_UNSUPPORTED, VB_ERR_LAUNCH = 0, -1, -2, -3
VB_DTYPE_BF16, VB_DTYPE_F16 = 0, 1

_i64x3 = ctypes.c_int64 * 3
_vp = ctypes.c_void_p
_i32p = ctypes.c_void_p  # device pointers are passed as integers


class AttnArgs(ctypes.Structure):
    """vb_attn_args (include/vblade.h)."""
    _fields_ = [
        ("q", _vp), ("k", _vp), ("v", _vp),
        ("q_stride", _i64x3), ("k_stride", _i64x3), ("v_stride", _i64x3),
        ("q_rows", _vp), ("kv_rows", _vp),
        ("use_main", ctypes.c_int),
        ("block_mask", _vp), ("mask_stride", _i64x3),
        ("kp", _vp), ("vp", _vp), ("kp_stride", _i64x3), ("vp_stride", _i64x3),
        ("Lkp", ctypes.c_int), ("kp_log_bias", ctypes.c_float),
        ("out", _vp), ("out_stride", _i64x3),
        ("lse", _vp),
        ("B", ctypes.c_int), ("H", ctypes.c_int), ("Lq", ctypes.c_int), ("Lk", ctypes.c_int),
        ("D", ctypes.c_int),
        ("scale", ctypes.c_float),
        ("dtype", ctypes.c_int),
        ("heavy_rows", ctypes.c_int),
        ("q_order", _vp), ("q_lengths", _vp), ("order_window", ctypes.c_int),
        ("work_queue", _vp),
    ]


class PredictArgs(ctypes.Structure):
    """vb_predict_args (include/vblade.h)."""
    _fields_ = [
        ("q", _vp), ("k", _vp),
        ("q_stride", _i64x3), ("k_stride", _i64x3),
        ("rows", _vp), ("q_off", _vp), ("k_off", _vp),
        ("B", ctypes.c_int), ("H", ctypes.c_int), ("L", ctypes.c_int), ("D", ctypes.c_int),
        ("block", ctypes.c_int), ("num_keep", ctypes.c_int),
        ("scale", ctypes.c_float), ("energy_threshold", ctypes.c_float),
        ("min_keep", ctypes.c_int), ("max_keep", ctypes.c_int), ("force_tail", ctypes.c_int),
        ("po", _vp), ("mask", _vp), ("mask_count", _vp),
        ("dtype", ctypes.c_int),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_uint64),
        ("staged_event", _vp),
        ("rand_q", _vp), ("rand_k", _vp),
        ("pool_v", _vp), ("pool_v_stride", _i64x3), ("pool_gap", ctypes.c_int),
        ("pool_kp", _vp), ("pool_vp", _vp), ("pool_k_r", _vp), ("pool_v_r", _vp),
        ("pyr_k", _vp), ("pyr_v", _vp),
        ("philox", ctypes.c_int), ("philox_seed", ctypes.c_uint64), ("philox_offset", ctypes.c_uint64),
        ("mask_level", ctypes.c_int), ("level_bands", ctypes.c_int),
        ("level_band_value", _vp), ("level_band_start", _vp), ("level_band_end", _vp),
        ("mask_rows_kept", _vp),
    ]


class BwdArgs(ctypes.Structure):
    """vb_attn_bwd_args (include/vblade.h)."""
    _fields_ = [
        ("q", _vp), ("q_stride", _i64x3),
        ("k", _vp), ("v", _vp), ("k_stride", _i64x3), ("v_stride", _i64x3),
        ("q_rows", _vp), ("kv_rows", _vp),
        ("block_mask", _vp), ("mask_stride", _i64x3),
        ("out", _vp), ("out_stride", _i64x3),
        ("lse", _vp),
        ("kp", _vp), ("vp", _vp), ("kp_stride", _i64x3), ("vp_stride", _i64x3),
        ("Lkp", ctypes.c_int),
        ("out2", _vp), ("out2_stride", _i64x3),
        ("lse2", _vp), ("alpha", _vp),
        ("pool_gap", ctypes.c_int),
        ("dout", _vp), ("dout_stride", _i64x3),
        ("dq", _vp), ("dq_stride", _i64x3),
        ("dk", _vp), ("dv", _vp), ("dk_stride", _i64x3), ("dv_stride", _i64x3),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_uint64),
        ("B", ctypes.c_int), ("H", ctypes.c_int), ("Lq", ctypes.c_int), ("Lk", ctypes.c_int),
        ("D", ctypes.c_int),
        ("scale", ctypes.c_float),
        ("dtype", ctypes.c_int),
        ("heavy_rows", ctypes.c_int),
        ("kernel_select", ctypes.c_int), ("kernels_ran", ctypes.POINTER(ctypes.c_int32)),
    ]


class MlAttnArgs(ctypes.Structure):
    """vb_ml_attn_args (include/vblade.h)."""
    _fields_ = [
        ("q", _vp), ("q_stride", _i64x3),
        ("q_rows", _vp),
        ("kpyr", _vp), ("vpyr", _vp),
        ("level_mask", _vp), ("mask_stride", _i64x3),
        ("out", _vp), ("out_stride", _i64x3),
        ("lse", _vp),
        ("B", ctypes.c_int), ("H", ctypes.c_int), ("L", ctypes.c_int), ("D", ctypes.c_int),
        ("scale", ctypes.c_float),
        ("ref_tail", ctypes.c_int),
        ("dtype", ctypes.c_int),
        ("heavy_rows", ctypes.c_int),
        ("work_queue", _vp),
    ]


class MlBwdArgs(ctypes.Structure):
    """vb_ml_attn_bwd_args (include/vblade.h)."""
    _fields_ = [
        ("q", _vp), ("q_stride", _i64x3),
        ("rows", _vp),
        ("kpyr", _vp), ("vpyr", _vp),
        ("level_mask", _vp), ("mask_stride", _i64x3),
        ("out", _vp), ("out_stride", _i64x3),
        ("lse", _vp),
        ("dout", _vp), ("dout_stride", _i64x3),
        ("dq", _vp), ("dq_stride", _i64x3),
        ("dk", _vp), ("dv", _vp), ("dk_stride", _i64x3), ("dv_stride", _i64x3),
        ("workspace", _vp), ("workspace_bytes", ctypes.c_uint64),
        ("B", ctypes.c_int), ("H", ctypes.c_int), ("L", ctypes.c_int), ("D", ctypes.c_int),
        ("scale", ctypes.c_float),
        ("ref_tail", ctypes.c_int),
        ("dtype", ctypes.c_int),
        ("heavy_rows", ctypes.c_int),
        ("kernel_select", ctypes.c_int), ("kernels_ran", ctypes.POINTER(ctypes.c_int32)),
    ]


# vb_attn_bwd_args.kernel_select / kernels_ran bits (include/vblade.h)
VB_BWD_SEL_DKDV_ROUND3, VB_BWD_SEL_DQ_ROUND3, VB_BWD_SEL_DQ_RING4 = 1, 2, 4
VB_BWD_RAN_DKDV_PIPE, VB_BWD_RAN_DKDV_ROUND3 = 1, 2
VB_BWD_RAN_DQ_PIPE_RING2, VB_BWD_RAN_DQ_PIPE_RING4, VB_BWD_RAN_DQ_ROUND3 = 4, 8, 16
VB_BWD_RAN_ML_PYRAMID = 32
VB_WORK_QUEUE_INTS = 288
ABI_VERSION = 4

# name -> (restype, argtypes); must list every symbol include/vblade.h declares
SIGNATURES = {
    "vb_last_error": (ctypes.c_char_p, []),
    "vb_abi_version": (ctypes.c_int, []),
    "vb_gilbert3d_perm": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp]),
    "vb_block_sparse_attn_fwd": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_float, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        _vp, _vp, ctypes.c_int, _vp]),
    "vb_attn_fwd": (ctypes.c_int, [ctypes.POINTER(AttnArgs), _vp]),
    "vb_mask_predict_workspace_size": (ctypes.c_uint64, [ctypes.POINTER(PredictArgs)]),
    "vb_mask_predict": (ctypes.c_int, [ctypes.POINTER(PredictArgs), _vp]),
    "vb_sample_offsets": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]),
    "vb_energy_mask": (ctypes.c_int, [
        _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp]),
    "vb_pool_kv": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    "vb_attn_bwd_workspace_size": (ctypes.c_uint64, [ctypes.POINTER(BwdArgs)]),
    "vb_attn_bwd": (ctypes.c_int, [ctypes.POINTER(BwdArgs), _vp]),
    "vb_block_sparse_attn_bwd_workspace_size": (ctypes.c_uint64, [ctypes.c_int] * 3),
    "vb_block_sparse_attn_bwd": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
        ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        _vp, _vp, _vp, _vp, ctypes.c_uint64, ctypes.c_int, _vp]),
    "vb_kv_pyramid_rows": (ctypes.c_int, [ctypes.c_int]),
    "vb_kv_pyramid": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_int, _vp, _vp, _vp]),
    "vb_level_mask": (ctypes.c_int, [
        _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp, _vp, _vp,
        ctypes.c_int, _vp, _vp]),
    "vb_ml_attn_fwd": (ctypes.c_int, [ctypes.POINTER(MlAttnArgs), _vp]),
    "vb_ml_attn_bwd_workspace_size": (ctypes.c_uint64, [ctypes.POINTER(MlBwdArgs)]),
    "vb_ml_attn_bwd": (ctypes.c_int, [ctypes.POINTER(MlBwdArgs), _vp]),
    "vb_lse_combine": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
        ctypes.c_float, ctypes.c_int, _vp, _vp, _vp]),
}

_lib = None


class VBladeError(RuntimeError):
    """A failed library call; ``code`` is the VB_ERR_* value it returned (None for host checks)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


def load() -> ctypes.CDLL:
    """Load libvblade_hip.so once; raise (never fall back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VBladeError(
            f"libvblade_hip.so not found at {LIB_PATH}; build it with "
            "`make -C video-blade_amd` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.vb_abi_version() != ABI_VERSION:
        raise VBladeError("libvblade_hip.so ABI version mismatch")
    _lib = lib
    return lib


def check(code: int, what: str):
    if code != VB_OK:
        msg = load().vb_last_error().decode(errors="replace")
        raise VBladeError(f"{what} failed ({code}): {msg}", code)

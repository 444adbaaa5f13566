"""ctypes binding of libpldepth_hip.so (the C ABI declared in include/pldepth_hip.h).

There is no fallback: importing the product path without the built library raises. Every call
checks the returned status and raises ``PLDError`` with ``pld_last_error()``'s text.
"""
import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# PLD_LIB_PATH: load another build of the same ABI (A/B experiments, tools/ab_lib.sh)
LIB_PATH = os.environ.get("PLD_LIB_PATH") or os.path.join(_HERE, "libpldepth_hip.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "pldepth_hip.h")

P = C.c_void_p
I32 = C.c_int
I64 = C.c_int64
U64 = C.c_uint64
F32 = C.c_float
SZ = C.c_size_t


class PLDError(RuntimeError):
    pass


class ConvArgs(C.Structure):
    """Mirror of ``pld_conv_args``."""
    _fields_ = [
        ("x1", P), ("x2", P), ("c1", I32), ("c2", I32),
        ("n", I32), ("h", I32), ("w", I32),
        ("kh", I32), ("kw", I32), ("sh", I32), ("sw", I32), ("pad_t", I32), ("pad_l", I32),
        ("oh", I32), ("ow", I32), ("cout", I32),
        ("in_scale", P), ("in_shift", P), ("in_act", I32), ("tile", I32),
        ("ws", P), ("ws_bytes", SZ), ("math", I32), ("w_split", P),
    ]


_SIGS = {
    "pld_last_error": (C.c_char_p, []),
    "pld_version": (I32, []),
    "pld_listmle_fwd_bwd": (I32, [P, P, I32, I32, I32, I32, P, P, P, I32, P]),
    "pld_adam_amsgrad": (I32, [P, P, P, P, P, I64, F32, F32, F32, F32, I64, F32, P]),
    "pld_adam_amsgrad_dev": (I32, [P, P, P, P, P, I64, P, P, F32, F32, F32, F32, P]),
    "pld_step_increment": (I32, [P, P]),
    "pld_set_scalar_f32": (I32, [P, F32, P]),
    "pld_sampler_draw_dev": (I32, [P, I32, I32, I32, U64, P, I32, P, P]),
    "pld_dropconnect_scales_dev": (I32, [P, I32, F32, U64, P, I32, I32, P]),
    "pld_dropconnect_scales_multi": (I32, [P, I32, I32, P, P, U64, U64, P, I32, P]),
    "pld_conv2d_fwd": (I32, [C.POINTER(ConvArgs), P, P, P, I32, P]),
    "pld_conv2d_dgrad": (I32, [C.POINTER(ConvArgs), P, P, P, I32, P, I32, P]),
    "pld_conv2d_wgrad_workspace_size": (SZ, [C.POINTER(ConvArgs)]),
    "pld_conv2d_wgrad": (I32, [C.POINTER(ConvArgs), P, P, I32, P, SZ, P]),
    "pld_conv_num_tiles": (I32, []),
    "pld_conv2d_fwd_bn_stats_workspace_size": (SZ, [C.POINTER(ConvArgs)]),
    "pld_conv2d_fwd_bn_stats": (I32, [C.POINTER(ConvArgs), P, P, P, F32, F32, P, P, P, P, P, SZ,
                                      P]),
    "pld_conv_num_schedules": (I32, [I32]),
    "pld_conv_schedule_class": (I32, [I32, I32]),
    "pld_conv_schedule_desc": (C.c_char_p, [I32, I32]),
    "pld_conv_kernel_kind": (I32, [C.POINTER(ConvArgs), I32]),
    "pld_conv_kernel_name": (C.c_char_p, [C.POINTER(ConvArgs), I32]),
    "pld_conv2d_fwd_workspace_size": (SZ, [C.POINTER(ConvArgs)]),
    "pld_conv2d_dgrad_workspace_size": (SZ, [C.POINTER(ConvArgs)]),
    "pld_filter_to_native": (I32, [P, I32, I32, I32, I32, P, P]),
    "pld_filter_split": (I32, [P, I64, I32, P, P]),
    "pld_filter_to_dgrad": (I32, [P, I32, I32, I32, I32, P, P]),
    "pld_filter_refresh": (I32, [P, I32, I32, I32, I32, P, P, P, P, P]),
    "pld_filter_refresh_plan": (I32, [I32, I32, I32, I32, P, P, P, P, P]),
    "pld_filter_refresh_multi": (I32, [P, I32, I32, P]),
    "pld_channel_reduce_workspace_size": (SZ, [I64, I32]),
    "pld_channel_sum": (I32, [P, I64, I32, P, I32, P, P]),
    "pld_bn_stats": (I32, [P, I64, I32, F32, F32, P, P, P, P, P, P]),
    "pld_bn_apply": (I32, [P, I64, I32, P, P, P, P, I32, P, I32, P, P]),
    "pld_bn_bwd": (I32, [P, P, I64, I32, P, P, P, P, I32, P, P, I32, P, I32, P, P, I32, P, P]),
    "pld_channel_affine_act": (I32, [P, I64, I32, P, P, I32, P, P]),
    "pld_bn_bwd_coeffs": (I32, [P, P, I64, I32, P, P, P, P, I32, P, P, I32, P, P, P]),
    "pld_pgemm_ok": (I32, [I32, I32]),
    "pld_pgemm_bn_act": (I32, [P, I64, I32, P, P, P, P, I32, P, I32, P, I32, P, I32, P]),
    "pld_pgemm_bn_bwd": (I32, [P, P, I64, I32, P, P, P, P, I32, P, P, I32, P, I32, P]),
    "pld_bn_add_apply": (I32, [P, I64, I32, P, P, P, P, P, I32, P, P]),
    "pld_bn_scale_add_apply": (I32, [P, I64, I32, P, P, P, P, P, I32, P, I32, P, P]),
    "pld_bn_bwd_scaled": (I32, [P, P, I64, I32, P, P, P, P, I32, P, I32, P, I32, P, P, I32, P,
                                P]),
    "pld_bn_add_bwd": (I32, [P, P, I64, I32, P, P, P, P, P, I32, P, I32, P, I32, P, P, I32, P,
                             P]),
    "pld_maxpool2d_fwd": (I32, [P, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, P, P, P]),
    "pld_maxpool2d_bwd": (I32, [P, P, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, P, I32,
                                P]),
    "pld_upsample2x_fwd": (I32, [P, I32, I32, I32, I32, P, P]),
    "pld_upsample2x_fwd_bn": (I32, [P, I32, I32, I32, I32, P, P, P, P, I32, P, P]),
    "pld_upsample2x_bwd": (I32, [P, I32, I32, I32, I32, P, I32, P]),
    "pld_upconv_wgrad_workspace_size": (SZ, [I32]),
    "pld_upconv_bwd_workspace_size": (SZ, [I32]),
    "pld_upconv_bwd": (I32, [P, I32, I32, I32, I32, P, P, P, P, P, P, P, P, P, I32, P, P, I32, P,
                             SZ, P]),
    "pld_upconv_fwd": (I32, [P, I32, I32, I32, I32, P, P, P, P, P, P, P, P]),
    "pld_upconv_wgrad": (I32, [P, I32, I32, I32, I32, P, P, P, P, P, P, P, SZ, P]),
    "pld_upconv_dgrad": (I32, [P, I32, I32, I32, I32, P, P, P]),
    "pld_residual_add": (I32, [P, P, P, I32, I64, P, P]),
    "pld_scale_per_sample": (I32, [P, P, I32, I64, P, I32, P]),
    "pld_dropconnect_scales": (I32, [P, I32, F32, U64, U64, I32, I32, P]),
    "pld_bn_inference_coeffs": (I32, [P, P, P, P, I32, F32, P, P, P]),
    "pld_bn_train_coeffs": (I32, [P, P, P, P, I32, P, P, P]),
    "pld_channel_pad_affine": (I32, [P, I64, I32, I32, P, P, P, P]),
    "pld_dwconv_fwd": (I32, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, P, P]),
    "pld_dwconv_fwd_bn": (I32, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, P, P, P,
                                P, I32, P, P]),
    "pld_dwconv_fwd_bn_stats_workspace_size": (SZ, [I32, I32, I32, I32, I32]),
    "pld_dwconv_fwd_bn_stats": (I32, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, P,
                                      P, P, P, I32, P, F32, F32, P, P, P, P, P, SZ, P]),
    "pld_dwconv_dgrad": (I32, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, P, I32, P]),
    "pld_dwconv_dgrad_bn_bwd_workspace_size": (SZ, [I32, I32, I32, I32, I32]),
    "pld_dwconv_dgrad_bn_bwd": (I32, [P, I32, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, P,
                                      I32, P, P, P, P, P, I32, P, I32, P, P, I32, P, P, SZ, P]),
    "pld_se_workspace_size": (SZ, [I32, I32, I32, I32]),
    "pld_se_fwd": (I32, [P, I32, I32, I32, I32, P, P, P, P, P, P, P, P, P]),
    "pld_se_bwd": (I32, [P, P, I32, I32, I32, I32, P, P, P, P, P, P, P]),
    "pld_se_fwd_bn": (I32, [P, P, P, P, P, I32, I32, I32, I32, I32, P, P, P, P, P, P, P, P, P]),
    "pld_se_bwd_bn": (I32, [P, P, P, P, P, P, I32, I32, I32, I32, I32, P, P, P, P, P, P, P]),
    "pld_se_bwd_bn_full_workspace_size": (SZ, [I32, I32, I32, I32]),
    "pld_se_bwd_bn_full": (I32, [P, P, P, P, P, P, I32, I32, I32, I32, I32, P, P, P, P, P, P, I32,
                                 P, P, I32, P, SZ, P]),
    "pld_sampler_workspace_size": (SZ, [I32, I32, I32, I32, I32, I32]),
    "pld_sampler_compact": (I32, [P, I32, I32, I32, P, P, P, P, P, P]),
    "pld_sampler_compact_workspace_size": (SZ, [I32, I32, I32]),
    "pld_sampler_draw": (I32, [P, I32, I32, I32, U64, U64, I32, P, P]),
    "pld_sampler_rank": (I32, [P, P, P, P, P, I32, I32, I32, I32, I32, I32, P, P, P]),
    "pld_sampler_candidates": (I32, [I32, I32]),
    "pld_resize_bilinear": (I32, [P, I32, I32, I32, I32, I32, I32, P, P]),
    "pld_resize_nearest": (I32, [P, I32, I32, I32, I32, I32, I32, P, P]),
    "pld_ordinal_error": (I32, [P, P, I32, I64, P, P, I32, P, P]),
    "pld_dcg_ratio": (I32, [P, P, I32, I64, P, I32, P, P]),
    "pld_graph_begin": (I32, [P]),
    "pld_graph_end": (I32, [P, C.POINTER(P)]),
    "pld_graph_launch": (I32, [P, P]),
    "pld_graph_destroy": (I32, [P]),
}

# functions returning a value rather than a status
_NON_STATUS = {"pld_last_error", "pld_version", "pld_pgemm_ok", "pld_conv_num_tiles", "pld_conv_num_schedules",
               "pld_conv_schedule_class", "pld_conv_schedule_desc",
               "pld_conv_kernel_kind", "pld_conv_kernel_name",
               "pld_conv2d_fwd_workspace_size", "pld_conv2d_dgrad_workspace_size", "pld_conv2d_wgrad_workspace_size",
               "pld_conv2d_fwd_bn_stats_workspace_size",
               "pld_dwconv_fwd_bn_stats_workspace_size",
               "pld_channel_reduce_workspace_size", "pld_se_workspace_size",
               "pld_sampler_workspace_size", "pld_sampler_candidates",
               "pld_sampler_compact_workspace_size", "pld_upconv_wgrad_workspace_size",
               "pld_upconv_bwd_workspace_size", "pld_se_bwd_bn_full_workspace_size",
               "pld_dwconv_dgrad_bn_bwd_workspace_size",
               "pld_filter_refresh_plan"}


def declared_symbols(header=HEADER):
    """Every ``pld_*`` function declared in include/pldepth_hip.h."""
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pld_[a-z0-9_]+)\s*\(", txt)))


class _Lib:
    def __init__(self, path=LIB_PATH):
        if not os.path.exists(path):
            raise PLDError(
                f"{path} not found: build the HIP library first (python -m pldepth_amd.build). "
                "There is no CPU fallback.")
        self._dll = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            fn = getattr(self._dll, name)
            fn.restype = res
            fn.argtypes = args
            if name in _NON_STATUS:
                setattr(self, name, fn)
            else:
                setattr(self, name, self._wrap(name, fn))

    def _wrap(self, name, fn):
        err = self._dll.pld_last_error

        def call(*args):
            rc = fn(*args)
            if rc != 0:
                raise PLDError(f"{name} failed ({rc}): {err().decode(errors='replace')}")
            return rc

        call.__name__ = name
        return call


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _Lib()
    return _LIB

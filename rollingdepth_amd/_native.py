"""ctypes binding of librdmi.so (include/rdmi.h).

The library is mandatory: importing this module without the built .so raises, so the product
path can never silently fall back to PyTorch or CPU arithmetic.  Build it with
`python -m rollingdepth_amd._build` (or `__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes as C
import os

_LIB_PATH = os.environ.get("RDMI_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "librdmi.so")

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_long
f32 = C.c_float


class GemmArgs(C.Structure):
    _fields_ = [
        ("A", vp), ("lda", i64), ("strideA", i64),
        ("W", vp), ("ldw", i64), ("strideW", i64),
        ("C", vp), ("ldc", i64), ("strideC", i64), ("c_f32", i32),
        ("bias", vp),
        ("residual", vp), ("ldr", i64), ("strideR", i64),
        ("rowbias", vp), ("rows_per_group", i32), ("rowbias_ld", i64),
        ("alpha", f32),
        ("M", i32), ("N", i32), ("K", i32), ("batch", i32),
        ("epilogue", i32),
        ("gn_part", vp), ("gn_ld", i64),
        ("dtype", i32),
    ]


class ConvArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("w", vp), ("y", vp),
        ("bias", vp), ("residual", vp), ("rowbias", vp),
        ("B", i32), ("H", i32), ("W", i32), ("Cin", i32), ("Cout", i32), ("kh", i32), ("kw", i32),
        ("stride", i32), ("pad_top", i32), ("pad_left", i32), ("upsample", i32), ("Ho", i32), ("Wo", i32),
        ("Kp", i32),
        ("y_ld", i64), ("res_ld", i64), ("alpha", f32), ("rowbias_ld", i64),
        ("gn_part", vp), ("gn_ld", i64),
        ("in_mean_rstd", vp), ("in_gamma", vp), ("in_beta", vp), ("in_groups", i32), ("in_silu", i32),
        ("dtype", i32),
        ("w_up2", vp),
        ("in_affine", vp),
    ]


class AlignerArgs(C.Structure):
    _fields_ = [
        ("n_dil", i32),
        ("x", vp * 8), ("s", vp * 8), ("t", vp * 8),
        ("n", i32 * 8), ("stride", i32 * 8),
        ("w", i32 * 8), ("seq_len", i32), ("P", i64),
        ("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("lmda2", f32), ("lmda3", f32),
        ("depth_w", f32), ("loss_scale", f32),
        ("iters", i32),
        ("history", vp), ("workspace", vp),
    ]


# name -> (restype, argtypes)
_SIGS = {
    "rdmi_last_error": (C.c_char_p, []),
    "rdmi_version": (i32, []),
    "rdmi_gemm": (i32, [C.POINTER(GemmArgs), vp]),
    "rdmi_conv2d": (i32, [C.POINTER(ConvArgs), vp]),
    "rdmi_conv2d_in_gn_supported": (i32, [C.POINTER(ConvArgs)]),
    "rdmi_groupnorm_workspace": (i64, [i32, i32]),
    "rdmi_groupnorm_stats": (i32, [vp, i32, i32, i64, i32, i32, f32, vp, vp, vp]),
    "rdmi_groupnorm_stats_partials": (i32, [vp, i64, i32, i64, i32, i32, f32, vp, vp]),
    "rdmi_groupnorm_apply": (i32, [vp, vp, i32, i32, i64, i32, i32, vp, vp, vp, i32, vp]),
    "rdmi_conv3x3_to1_gn_workspace": (i64, [i32, i32, i32]),
    "rdmi_conv3x3_to1_gn": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, i32, vp, f32, vp, i32, vp, vp]),
    "rdmi_layernorm": (i32, [vp, vp, i32, i64, i32, vp, vp, f32, vp]),
    "rdmi_attention_fwd": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i64, i64, i64, i64, i64, i64, i64, i64,
                                 f32, i32, vp]),
    "rdmi_attention_smallkv": (i32, [vp, vp, vp, vp, i32, i32, i32, i32, i32, i64, i64, i64, i64, i64, f32, i32, vp]),
    "rdmi_cross_attn_pair": (i32, [vp, vp, i64, i32, i32, vp, vp, f32, vp, vp, vp, vp]),
    "rdmi_softmax_rows": (i32, [vp, vp, i64, i64, i64, f32, i32, vp]),
    "rdmi_nchw_to_nhwc": (i32, [vp, i32, vp, i32, i32, i32, i32, i32, i32, f32, i64, i64, vp]),
    "rdmi_nhwc_to_nchw_f32": (i32, [vp, i32, i64, vp, i32, i32, i32, i32, f32, f32, vp]),
    "rdmi_concat_channels": (i32, [vp, i32, vp, i32, vp, i64, i32, vp]),
    "rdmi_resize_nearest": (i32, [vp, i32, i32, i32, i32, vp, i32, i32, i32, vp]),
    "rdmi_transpose": (i32, [vp, vp, i32, i64, i64, i64, i64, i32, vp]),
    "rdmi_gather_unet_input": (i32, [vp, i64, vp, i64, i32, vp, i32, i64, vp, i32, vp]),
    "rdmi_ddim_combine": (i32, [vp, i64, vp, i64, vp, i64, i64, i32, i32, f32, f32, f32, i64, i32, vp]),
    "rdmi_snippet_average": (i32, [vp, i32, i32, i32, i32, i64, i32, i32, vp, i32, vp]),
    "rdmi_snippet_accumulate": (i32, [vp, i32, i32, i32, i32, i32, i32, i64, i32, i32, vp, vp]),
    "rdmi_snippet_finish": (i32, [vp, i32, i32, i32, i32, i64, i32, i32, vp, i32, vp]),
    "rdmi_colorize": (i32, [vp, i32, i64, vp, vp, i32, vp, vp, vp]),
    "rdmi_resize_workspace": (C.c_size_t, [i32, i32, i32, i32, i32, i32]),
    "rdmi_attention_d512": (i32, [vp, vp, vp, vp, i32, i32, i32, i32] + [i64] * 8 + [C.c_float, vp, vp]),
    "rdmi_resize": (i32, [vp, i32, i64, i64, i64, i64, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    "rdmi_minmax": (i32, [vp, i32, i64, vp, vp, vp]),
    "rdmi_renormalize_f32": (i32, [vp, i64, vp, vp]),
    "rdmi_aligner_workspace": (i64, [C.POINTER(AlignerArgs)]),
    "rdmi_aligner_optimize": (i32, [C.POINTER(AlignerArgs), vp]),
    "rdmi_aligner_prepare": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp]),
    "rdmi_aligner_merge": (i32, [i32, C.POINTER(vp), i32, C.POINTER(vp), C.POINTER(vp), C.POINTER(i32),
                                 C.POINTER(i32), C.POINTER(i32), i32, i64, vp, vp, vp]),
    "rdmi_groupnorm_affine": (i32, [vp, vp, vp, i32, i32, i32, vp, vp]),
    "rdmi_aligner_merge_partial_window": (i32, [i32, C.POINTER(vp), i32, C.POINTER(vp), C.POINTER(vp),
                                                C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32),
                                                C.POINTER(i32), i32, i32, i64, vp, vp, vp]),
    "rdmi_aligner_merge_finish_pieces": (i32, [i32, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32), i32, i32, i64,
                                               i32, C.POINTER(i32), C.POINTER(i32), vp, vp, vp]),
}

RDMI_F16, RDMI_F32, RDMI_U8, RDMI_F32_X3, RDMI_F32_X6 = 0, 1, 2, 3, 4
RDMI_RESIZE_NEAREST, RDMI_RESIZE_BILINEAR, RDMI_RESIZE_BICUBIC = 0, 1, 2

EXPORTED = tuple(_SIGS)


def _load():
    if not os.path.exists(_LIB_PATH):
        raise ImportError(
            f"librdmi.so not found at {_LIB_PATH}: build it with `python -m rollingdepth_amd._build` "
            "(the HIP path has no fallback)")
    lib = C.CDLL(_LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class RdmiError(RuntimeError):
    pass


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib.rdmi_last_error().decode(errors="replace")
        raise RdmiError(f"{what or 'librdmi'} failed (code {rc}): {msg}")

"""ctypes binding of libvda.so (the C ABI declared in include/vda.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) and loaded from this
package directory.  There is no fallback: if the library is missing or fails to load, every op
raises ``VDAUnavailable``.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int32, c_int64, c_void_p, POINTER

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VDA_LIB_OVERRIDE") or os.path.join(_HERE, "libvda.so")  # override: tuning experiments only
TORCH_LIB_PATH = os.path.join(_HERE, "libvda_torch.so")  # TORCH_LIBRARY(vda) over the C ABI (csrc/vda_torch.cpp)
if os.environ.get("VDA_LIB_OVERRIDE"):  # tuning builds: the op library linked next to the override libvda.so
    _ov = os.path.join(os.path.dirname(os.path.abspath(os.environ["VDA_LIB_OVERRIDE"])), "libvda_torch.so")
    if os.path.exists(_ov):
        TORCH_LIB_PATH = _ov

# Every symbol include/vda.h declares (checked by tests/test_capi.py).
EXPORTED = (
    "vda_version", "vda_epilogue_size", "vda_last_error", "vda_gemm", "vda_conv2d", "vda_conv2d_workspace", "vda_layernorm",
    "vda_conv2d_res2_upsample_ok",
    "vda_row_stats", "vda_groupnorm", "vda_groupnorm_workspace",
    "vda_groupnorm_linear", "vda_groupnorm_linear_workspace", "vda_groupnorm_linear_fused",
    "vda_spatial_attention", "vda_temporal_attention", "vda_upsample_bilinear", "vda_patch_im2col",
    "vda_depth_head", "vda_depth_head_workspace", "vda_preprocess_frames", "vda_depth_resize",
    "vda_gemm_f32", "vda_conv2d_f32", "vda_layernorm_f32", "vda_groupnorm_f32", "vda_spatial_attention_f32",
    "vda_temporal_attention_f32", "vda_upsample_bilinear_f32", "vda_patch_im2col_f32", "vda_depth_head_f32",
)
# The tuning build (make tune -> build/tune/libvda.so, include/vda_tune.h) adds these.
TUNE_EXPORTED = ("vda_debug_force_tile", "vda_debug_gemm_sched", "vda_debug_gemm_desync", "vda_debug_gemm_epi",
                 "vda_debug_strip_split", "vda_debug_hconv", "vda_debug_dconv", "vda_debug_attn",
                 "vda_debug_dconv_stagger")
TUNE_LIB_PATH = os.path.join(os.path.dirname(_HERE), "build", "tune", "libvda.so")

ACT_NONE, ACT_GELU, ACT_GEGLU, ACT_RELU = 0, 1, 2, 3
STORE_ROWS, STORE_PIXEL_SHUFFLE = 0, 1


class VDAUnavailable(RuntimeError):
    pass


class VDAError(RuntimeError):
    pass


class Epilogue(ctypes.Structure):
    """Mirror of ``vda_epilogue`` (include/vda.h)."""
    _fields_ = [
        ("bias", c_void_p), ("rowbias", c_void_p), ("rdiv", c_int32), ("rmod", c_int32),
        ("gamma", c_void_p), ("res", c_void_p), ("ldres", c_int64), ("res2", c_void_p),
        ("ldres2", c_int64), ("act", c_int32), ("store", c_int32), ("ps_k", c_int32),
        ("ps_cout", c_int32), ("ps_hin", c_int32), ("ps_win", c_int32),
        ("ln_stats", c_void_p), ("ln_colsum", c_void_p), ("ln_parts", c_int32), ("ln_eps", c_float),
        ("stats_out", c_void_p), ("res2_h", c_int32), ("res2_w", c_int32), ("sched", c_void_p),
        ("drop_period", c_int32),
    ]


_lib = None
_load_error = None


def _declare(lib):
    P, I, L, F = c_void_p, c_int32, c_int64, c_float
    EP = POINTER(Epilogue)
    sig = {
        "vda_version": ([], ctypes.c_char_p),
        "vda_epilogue_size": ([], L),
        "vda_last_error": ([], ctypes.c_char_p),
        "vda_gemm": ([P, L, P, P, L, I, I, I, EP, P], I),
        "vda_conv2d": ([P, P, P, I, I, I, I, I, I, I, I, I, I, I, EP, P, L, P], I),
        "vda_conv2d_workspace": ([I, I, I, I, I, I, I, I], L),
        "vda_conv2d_res2_upsample_ok": ([I, I, I, I, I, I, I, I], I),
        "vda_layernorm": ([P, L, P, P, P, I, I, F, I, P], I),
        "vda_row_stats": ([P, L, P, I, I, F, P], I),
        "vda_groupnorm": ([P, P, P, P, I, I, I, I, F, P, P], I),
        "vda_groupnorm_workspace": ([I, I, I, I], L),
        "vda_groupnorm_linear": ([P, P, P, I, I, I, I, F, P, P, P, I, P, P, L, P], I),
        "vda_groupnorm_linear_workspace": ([I, I, I, I, I], L),
        "vda_groupnorm_linear_fused": ([I, I, I], I),
        "vda_spatial_attention": ([P, P, I, I, I, I, F, P], I),
        "vda_temporal_attention": ([P, P, I, I, I, I, I, F, F, P], I),
        "vda_upsample_bilinear": ([P, P, I, I, I, I, I, I, P], I),
        "vda_patch_im2col": ([P, P, I, I, I, I, P], I),
        "vda_depth_head": ([P, P, P, P, P, P, P, I, I, I, I, I, I, P], I),
        "vda_depth_head_workspace": ([I, I, I, I, I, I], L),
        "vda_preprocess_frames": ([P, P, I, I, I, I, I, POINTER(F), POINTER(F), P], I),
        "vda_depth_resize": ([P, P, I, I, I, I, I, P], I),
        "vda_gemm_f32": ([P, L, P, P, L, I, I, I, EP, P], I),
        "vda_conv2d_f32": ([P, P, P, I, I, I, I, I, I, I, I, I, EP, P], I),
        "vda_layernorm_f32": ([P, L, P, P, P, I, I, F, I, P], I),
        "vda_groupnorm_f32": ([P, P, P, P, I, I, I, I, F, P], I),
        "vda_spatial_attention_f32": ([P, P, I, I, I, I, F, P], I),
        "vda_temporal_attention_f32": ([P, P, I, I, I, I, I, F, F, P], I),
        "vda_upsample_bilinear_f32": ([P, P, I, I, I, I, I, I, P], I),
        "vda_patch_im2col_f32": ([P, P, I, I, I, I, P], I),
        "vda_depth_head_f32": ([P, P, P, P, P, P, P, P, I, I, I, I, I, I, P], I),
        "vda_debug_force_tile": ([I], I),
        "vda_debug_gemm_sched": ([I, I], I),
        "vda_debug_gemm_desync": ([I], I),
        "vda_debug_strip_split": ([I], I),
        "vda_debug_hconv": ([I], I),
        "vda_debug_dconv": ([I], I),
        "vda_debug_dconv_stagger": ([I], I),
        "vda_debug_gemm_epi": ([I], I),
        "vda_debug_attn": ([I, I], I),
    }
    for name, (args, res) in sig.items():
        if name.startswith("vda_debug_") and not hasattr(lib, name):
            continue  # tuning hooks: only in the tuning build
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def lib():
    """Return the loaded libvda (raises VDAUnavailable if it cannot be loaded)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise VDAUnavailable(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = f"libvda.so not found at {LIB_PATH}; run `make` (or __graft_entry__.build())"
        raise VDAUnavailable(_load_error)
    try:
        l = ctypes.CDLL(LIB_PATH)
        _declare(l)
        if l.vda_epilogue_size() != ctypes.sizeof(Epilogue):  # the ctypes mirror must match include/vda.h
            raise OSError(f"vda_epilogue is {l.vda_epilogue_size()} bytes in the library, {ctypes.sizeof(Epilogue)} "
                          f"in _lib.Epilogue: rebuild libvda.so or update the mirror")
    except OSError as e:  # pragma: no cover - depends on the runtime
        _load_error = f"failed to load {LIB_PATH}: {e}"
        raise VDAUnavailable(_load_error) from e
    _lib = l
    return _lib


_torch_ops = None


def torch_ops():
    """``torch.ops.vda`` after loading libvda_torch.so (raises VDAUnavailable if it cannot be loaded).
    libvda.so is loaded first through ctypes from the same path, so the tuning hooks set through
    ``lib()`` act on the library the operators call."""
    global _torch_ops
    if _torch_ops is not None:
        return _torch_ops
    lib()
    if not os.path.exists(TORCH_LIB_PATH):
        raise VDAUnavailable(f"libvda_torch.so not found at {TORCH_LIB_PATH}; run `make` (or __graft_entry__.build())")
    import torch
    try:
        torch.ops.load_library(TORCH_LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the runtime
        raise VDAUnavailable(f"failed to load {TORCH_LIB_PATH}: {e}") from e
    _torch_ops = torch.ops.vda
    return _torch_ops


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().vda_last_error().decode(errors="replace")
        raise VDAError(f"{what} failed (rc={rc}): {msg}")

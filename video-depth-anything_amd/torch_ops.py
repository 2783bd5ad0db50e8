"""``torch.ops.vda.*``: the libvda kernels registered as PyTorch custom operators.

Each op has a CUDA (HIP) kernel registration that calls the C ABI through ``ops.py`` and a Meta
registration (output shape / dtype only) so the ops trace under fake tensors and torch.compile as
opaque nodes.  There is deliberately NO CPU registration: a CPU tensor reaches the dispatcher's
"no kernel for CPU" error instead of a silent fallback.  Activation dtype (fp16, or fp32 for fp32
mode) follows the input, as in ``ops.py``.

The module forward calls ``ops.py`` directly (no dispatcher hop per launch); these registrations
are the operator-level boundary for torch users, e.g.::

    import vda_amd.torch_ops  # registers the library once
    y = torch.ops.vda.gemm(x, w, bias, None, 1, 1, None, None, None, 1)  # fc1 + GELU
"""
from __future__ import annotations

import torch

from . import ops

_LIB = torch.library.Library("vda", "DEF")

_SCHEMAS = {
    "gemm": "gemm(Tensor x, Tensor w, Tensor? bias, Tensor? rowbias, int rdiv, int rmod, Tensor? gamma, "
            "Tensor? res, Tensor? res2, int act) -> Tensor",
    "conv2d": "conv2d(Tensor x, Tensor w, int ks, int stride, int pad, Tensor? bias, bool pre_relu, int act, "
              "Tensor? res, Tensor? res2) -> Tensor",
    "conv_transpose_ks": "conv_transpose_ks(Tensor x, Tensor w, Tensor bias, int BT, int h, int w_, int k) -> Tensor",
    "layernorm": "layernorm(Tensor x, Tensor gamma, Tensor beta, float eps, int skip_period) -> Tensor",
    "groupnorm": "groupnorm(Tensor x, Tensor gamma, Tensor beta, int frames, int groups, float eps) -> Tensor",
    "spatial_attention": "spatial_attention(Tensor qkv, int B, int N, int H, int D) -> Tensor",
    "temporal_attention": "temporal_attention(Tensor qkv, int B, int T, int S, int H, int D) -> Tensor",
    "upsample_bilinear": "upsample_bilinear(Tensor x, int Ho, int Wo) -> Tensor",
    "patch_im2col": "patch_im2col(Tensor img, int Kp, bool fp32) -> Tensor",
    "depth_head": "depth_head(Tensor x, Tensor w1, Tensor b1, Tensor w2, Tensor b2, int Ho, int Wo) -> Tensor",
    "preprocess_frames": "preprocess_frames(Tensor frames, int H, int W) -> Tensor",
    "depth_resize": "depth_resize(Tensor depth, int ho, int wo) -> Tensor",
}
for _s in _SCHEMAS.values():
    _LIB.define(_s)


def _gemm(x, w, bias, rowbias, rdiv, rmod, gamma, res, res2, act):
    return ops.gemm(x, w, bias=bias, rowbias=rowbias, rdiv=rdiv, rmod=rmod, gamma=gamma, res=res, res2=res2, act=act)


def _conv2d(x, w, ks, stride, pad, bias, pre_relu, act, res, res2):
    return ops.conv2d(x, w, ks=ks, stride=stride, pad=pad, bias=bias, pre_relu=pre_relu, act=act, res=res, res2=res2)


def _layernorm(x, gamma, beta, eps, skip_period):
    return ops.layernorm(x, gamma, beta, eps, skip_period=skip_period)


def _im2col(img, Kp, fp32):
    return ops.patch_im2col(img, Kp, dtype=torch.float32 if fp32 else torch.float16)


def _depth_head(x, w1, b1, w2, b2, Ho, Wo):
    if x.dtype == torch.float32:
        return ops.depth_head_f32(x, w1, b1, w2, b2, Ho, Wo)
    return ops.depth_head(x, w1, b1, w2, b2, Ho, Wo)


_IMPL = {
    "gemm": _gemm, "conv2d": _conv2d, "conv_transpose_ks": ops.conv_transpose_ks, "layernorm": _layernorm,
    "groupnorm": ops.groupnorm, "spatial_attention": ops.spatial_attention,
    "temporal_attention": ops.temporal_attention, "upsample_bilinear": ops.upsample_bilinear,
    "patch_im2col": _im2col, "depth_head": _depth_head, "preprocess_frames": ops.preprocess_frames,
    "depth_resize": ops.depth_resize,
}
for _n, _f in _IMPL.items():
    _LIB.impl(_n, _f, "CUDA")


# ---- Meta (shape-only) registrations ---------------------------------------------------------
def _m_gemm(x, w, bias, rowbias, rdiv, rmod, gamma, res, res2, act):
    n = w.shape[0] // 2 if act == 2 else w.shape[0]
    return x.new_empty((x.shape[0], n))


def _m_conv2d(x, w, ks, stride, pad, bias, pre_relu, act, res, res2):
    BT, H, W, _ = x.shape
    return x.new_empty((BT, (H + 2 * pad - ks) // stride + 1, (W + 2 * pad - ks) // stride + 1, w.shape[0]))


def _m_convt(x, w, bias, BT, h, w_, k):
    return x.new_empty((BT, h * k, w_ * k, w.shape[0] // (k * k)))


def _m_ln(x, gamma, beta, eps, skip_period):
    R, C = x.shape
    return x.new_empty((R if skip_period == 0 else (R // (skip_period + 1)) * skip_period, C))


_META = {
    "gemm": _m_gemm, "conv2d": _m_conv2d, "conv_transpose_ks": _m_convt, "layernorm": _m_ln,
    "groupnorm": lambda x, g, b, f, gr, e: x.new_empty(x.shape),
    "spatial_attention": lambda qkv, B, N, H, D: qkv.new_empty((B * N, H * D)),
    "temporal_attention": lambda qkv, B, T, S, H, D: qkv.new_empty((B * T * S, H * D)),
    "upsample_bilinear": lambda x, Ho, Wo: x.new_empty((x.shape[0], Ho, Wo, x.shape[3])),
    "patch_im2col": lambda img, Kp, fp32: img.new_empty(
        (img.shape[0] * (1 + (img.shape[2] // 14) * (img.shape[3] // 14)), Kp),
        dtype=torch.float32 if fp32 else torch.float16),
    "depth_head": lambda x, w1, b1, w2, b2, Ho, Wo: x.new_empty((x.shape[0], Ho, Wo), dtype=torch.float32),
    "preprocess_frames": lambda fr, H, W: fr.new_empty((fr.shape[0], 3, H, W), dtype=torch.float32),
    "depth_resize": lambda d, ho, wo: d.new_empty((d.shape[0], ho, wo)),
}
for _n, _f in _META.items():
    _LIB.impl(_n, _f, "Meta")

"""Tensor-level API of the libvda kernels: thin keyword wrappers over ``torch.ops.vda.*``.

The operators are native: ``csrc/vda_torch.cpp`` registers them with ``TORCH_LIBRARY(vda, m)``
(CUDA = HIP and Meta keys) in ``libvda_torch.so``, which validates device / dtype / layout,
allocates outputs and workspaces through the PyTorch caching allocator and launches through the C
ABI of ``include/vda.h`` on the current HIP stream (so whole forwards can be captured in a HIP
graph).  Activations are fp16 NHWC / token-major; biases, scales and norm affines fp32.  There is
deliberately no CPU path: an op on a CPU tensor, or without the native libraries, raises.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib
from ._lib import ACT_NONE, ACT_GELU, ACT_GEGLU, ACT_RELU, STORE_ROWS, STORE_PIXEL_SHUFFLE  # noqa: F401

Tensor = torch.Tensor


# Optional per-launch timing of tagged launches (bench.py's roofline leg).  When a tag is enabled,
# the launch is bracketed by two events on the launch stream; nothing else changes.
_PROBE: Optional[dict] = None


def enable_probe(tags):
    global _PROBE
    _PROBE = {t: [] for t in tags}


def take_probe():
    """Return {tag: [(ms, flop) per launch]} for the probed launches (synchronises) and disable
    probing; flop = 2*M*N*K of that launch."""
    global _PROBE
    out = {}
    if _PROBE:
        torch.cuda.synchronize()
        out = {t: [(a.elapsed_time(b), fl) for a, b, fl in ev] for t, ev in _PROBE.items()}
    _PROBE = None
    return out


def _vda():
    """torch.ops.vda, loading libvda_torch.so (TORCH_LIBRARY over libvda's C ABI) on first use.
    Raises VDAUnavailable when the native libraries are missing: there is no fallback."""
    return _lib.torch_ops()


def _need(t: Tensor, dtype, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"vda op: {name} must be a GPU tensor (no CPU path in the product)")
    if t.dtype != dtype:
        raise RuntimeError(f"vda op: {name} must be {dtype}, got {t.dtype}")


def gemm(x: Tensor, w: Tensor, *, bias=None, rowbias=None, rdiv=1, rmod=1, gamma=None, res=None,
         res2=None, act=ACT_NONE, ln_stats=None, ln_colsum=None, ln_parts=0, ln_eps=1e-6, stats_out=None,
         sched=None, drop_period=0, out: Optional[Tensor] = None, tag: Optional[str] = None) -> Tensor:
    """out[M, N'] = epi(x[M, K] @ w[N, K]^T); N' = N (N/2 for GEGLU). x may be a row-strided view.
    fp16 x/w -> vda_gemm; fp32 x/w -> vda_gemm_f32 (fp32 mode).  torch.ops.vda.gemm[.out].
    ``ln_stats`` + ``ln_colsum`` fold a LayerNorm of x into the GEMM (vda.h): ln_stats is either
    ``row_stats(x)`` ([M, 2] (mean, rstd), ln_parts=0) or the [M, P, 2] partial sums another GEMM wrote
    through ``stats_out`` while producing x (ln_parts=P, ln_eps the LayerNorm eps).  ``stats_out``
    ([M, ceil(N/256), 2] fp32) receives this GEMM's per-row partial (sum, sumsq) of its output.
    ``sched`` (int32 [>= 9], zeroed once; see ``sched_counters``) lets the persistent 256x256 GEMM take its
    tiles by atomic ticket; one counter set per stream (vda.h vda_epilogue.sched).  ``drop_period`` = P > 0:
    x is frames of P token rows, the first the cls token; the output leaves those rows out
    ([M - ceil(M / P), N'], the LN-folded projects GEMM on an encoder tap, vda.h drop_period)."""
    _need(x, x.dtype, "x")
    probe = _PROBE is not None and tag in _PROBE
    if probe:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    v = _vda()
    if out is None:
        out = v.gemm(x, w, bias, rowbias, int(rdiv), int(rmod), gamma, res, res2, int(act), ln_stats, ln_colsum,
                     int(ln_parts), float(ln_eps), stats_out, sched, int(drop_period))
    else:
        v.gemm.out(x, w, bias, rowbias, int(rdiv), int(rmod), gamma, res, res2, int(act), ln_stats, ln_colsum,
                   int(ln_parts), float(ln_eps), stats_out, sched, int(drop_period), out=out)
    if probe:
        ev1.record()
        _PROBE[tag].append((ev0, ev1, 2.0 * x.shape[0] * w.shape[0] * x.shape[1]))
    return out


_SCHED = {}


def sched_counters(device=None) -> Tensor:
    """The tile-scheduler counters (int32 [16], zero) of the current stream on `device`: one set per
    stream, so that GEMMs on different streams never share one (vda_epilogue.sched).  The kernels leave
    them zero after every launch."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    st = torch.cuda.current_stream(dev)
    key = (dev.index, st.cuda_stream)
    t = _SCHED.get(key)
    if t is None:
        t = torch.zeros(16, dtype=torch.int32, device=dev)
        _SCHED[key] = t
    return t


def conv_transpose_ks(x: Tensor, w: Tensor, bias: Tensor, BT: int, h: int, w_: int, k: int) -> Tensor:
    """ConvTranspose2d(kernel = stride = k) as one GEMM with a pixel-shuffle store.
    x [BT*h*w, Cin]; w [k*k*Cout, Cin] packed (i, j, co); bias [k*k*Cout] fp32 -> [BT, h*k, w*k, Cout]."""
    _need(x, x.dtype, "x")
    return _vda().conv_transpose_ks(x, w, bias, int(BT), int(h), int(w_), int(k))


def conv2d(x: Tensor, w: Tensor, *, ks=3, stride=1, pad=1, bias=None, pre_relu=False, act=ACT_NONE,
           res=None, res2=None, up=None) -> Tensor:
    """NHWC conv.  x [BT, H, W, Cin] fp16; w [Cout, ks, ks, Cin] fp16 -> [BT, Ho, Wo, Cout].
    `up=(Hu, Wu)` reads x through a bilinear align_corners=True resize to (Hu, Wu) first.
    The strip conv's split workspace comes from the caching allocator per call (no shared state)."""
    _need(x, x.dtype, "x")
    return _vda().conv2d(x, w, int(ks), int(stride), int(pad), bias, bool(pre_relu), int(act), res, res2,
                         None if up is None else [int(up[0]), int(up[1])])


def layernorm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float, *, skip_period: int = 0,
              rows: Optional[int] = None) -> Tensor:
    """Row LayerNorm of x [R, C] (row-strided ok).  skip_period=np drops each frame's cls row."""
    _need(x, x.dtype, "x")
    return _vda().layernorm(x, gamma, beta, float(eps), int(skip_period), rows)


def row_stats(x: Tensor, eps: float) -> Tensor:
    """Per-row LayerNorm statistics of x [R, C] fp16: [round_up(R, 2), 2] fp32 (mean, rstd)."""
    _need(x, torch.float16, "x")
    return _vda().row_stats(x, float(eps))


def groupnorm(x: Tensor, gamma: Tensor, beta: Tensor, frames: int, groups: int, eps: float) -> Tensor:
    """GroupNorm on NHWC frames: x [F*S, C] -> same."""
    _need(x, x.dtype, "x")
    return _vda().groupnorm(x, gamma, beta, int(frames), int(groups), float(eps))


def groupnorm_linear(x: Tensor, gamma: Tensor, beta: Tensor, frames: int, groups: int, eps: float, w: Tensor, *,
                     bias=None, stats_out=None) -> Tensor:
    """GroupNorm on NHWC frames then Linear: x [F*S, C] -> GN(x) @ w[N, C]^T + bias, [F*S, N]
    (motion_module.py:116-119, norm + proj_in).  fp16: one fused kernel for groups 32, N = C in
    {64, 128, 256} (vda.h vda_groupnorm_linear), else GroupNorm + GEMM through a workspace; ``stats_out``
    ([F*S, 1, 2] fp32) receives the per-row (sum, sumsq) of the output for a following LN-folded GEMM."""
    _need(x, x.dtype, "x")
    return _vda().groupnorm_linear(x, gamma, beta, int(frames), int(groups), float(eps), w, bias, stats_out)


def spatial_attention(qkv: Tensor, B: int, N: int, H: int, D: int = 64) -> Tensor:
    _need(qkv, qkv.dtype, "qkv")
    return _vda().spatial_attention(qkv, int(B), int(N), int(H), int(D))


def temporal_attention(qkv: Tensor, B: int, T: int, S: int, H: int, D: int, rope_theta: float = 0.0) -> Tensor:
    """Softmax attention over the T frames of every site; ``rope_theta`` > 0 rotates q and k first
    (pe='rope', attention.py:403-429: pairs (2i, 2i+1) of all H*D channels, angle t * theta^(-2i/C))."""
    _need(qkv, qkv.dtype, "qkv")
    return _vda().temporal_attention(qkv, int(B), int(T), int(S), int(H), int(D), float(rope_theta))


def upsample_bilinear(x: Tensor, Ho: int, Wo: int) -> Tensor:
    _need(x, x.dtype, "x")
    return _vda().upsample_bilinear(x, int(Ho), int(Wo))


def patch_im2col(img: Tensor, Kp: int, dtype=torch.float16) -> Tensor:
    """images [BT, 3, H, W] fp32 -> im2col rows [BT*(1+np), Kp] of ``dtype`` (fp16, or fp32 for fp32 mode)."""
    _need(img, torch.float32, "img")
    return _vda().patch_im2col(img, int(Kp), dtype)


def depth_head(x: Tensor, w1_split: Tensor, b1: Tensor, w2: Tensor, b2: Tensor, Ho: int, Wo: int) -> Tensor:
    """Depth tail: bilinear resize to (Ho, Wo), 3x3 conv (split-fp16 fp32 weights) -> ReLU -> 1x1 -> ReLU.
    x [BT, H, W, C] fp16; w1_split [64, 3, 3, C] fp16 (hi rows 0..31, lo rows 32..63) -> depth [BT, Ho, Wo] fp32.
    The resize workspace is allocated only for shapes the fused halo kernel does not serve."""
    _need(x, torch.float16, "x")
    return _vda().depth_head(x, w1_split, b1, w2, b2, int(Ho), int(Wo))


def depth_head_f32(x: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor, Ho: int, Wo: int) -> Tensor:
    """fp32-mode depth tail: x [BT, H, W, C] fp32; w1 [32, 3, 3, C] fp32 -> depth [BT, Ho, Wo] fp32."""
    _need(x, torch.float32, "x")
    return _vda().depth_head(x, w1, b1, w2, b2, int(Ho), int(Wo))


def preprocess_frames(frames: Tensor, H: int, W: int, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)) -> Tensor:
    """uint8 frames [N, h, w, 3] (GPU) -> normalised network input [N, 3, H, W] fp32 (bicubic resize)."""
    _need(frames, torch.uint8, "frames")
    if frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError(f"frames must be [N, h, w, 3] uint8, got {tuple(frames.shape)}")
    return _vda().preprocess_frames(frames, int(H), int(W), [float(v) for v in mean], [float(v) for v in std])


def depth_resize(depth: Tensor, ho: int, wo: int) -> Tensor:
    """depth [N, H, W] fp32 (GPU) -> [N, ho, wo] fp32, bilinear align_corners=True."""
    _need(depth, torch.float32, "depth")
    return _vda().depth_resize(depth, int(ho), int(wo))

"""Tensor-level wrappers over the libvda C ABI.

Each wrapper validates device / dtype / layout, allocates its output through the PyTorch caching
allocator, and launches on ``torch.cuda.current_stream()`` (so whole forwards can be captured in a
CUDA(HIP) graph).  Activations are fp16 NHWC / token-major; biases, scales and norm affines fp32.
There is deliberately no CPU path: calling an op on a CPU tensor, or without libvda, raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib
from ._lib import Epilogue, check, ACT_NONE, ACT_GELU, ACT_GEGLU, ACT_RELU, STORE_ROWS, STORE_PIXEL_SHUFFLE  # noqa: F401

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


def _stream(t: Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def _need(t: Tensor, dtype, name: str):
    if not t.is_cuda:
        raise RuntimeError(f"vda op: {name} must be a GPU tensor (no CPU path in the product)")
    if t.dtype != dtype:
        raise RuntimeError(f"vda op: {name} must be {dtype}, got {t.dtype}")


def _need_contig(t: Tensor, dtype, name: str):
    _need(t, dtype, name)
    if not t.is_contiguous():
        raise RuntimeError(f"vda op: {name} must be contiguous")


def _dt(x: Tensor):
    """Activation dtype of an op: fp16 (the shipped mode) or fp32 (fp32 mode, the *_f32 entry points)."""
    if x.dtype not in (torch.float16, torch.float32):
        raise RuntimeError(f"vda op: activations must be float16 or float32, got {x.dtype}")
    return x.dtype


def _epilogue(bias=None, rowbias=None, rdiv=1, rmod=1, gamma=None, res=None, res2=None,
              act=ACT_NONE, store=STORE_ROWS, ps=(0, 0, 0, 0), dt=torch.float16) -> Epilogue:
    e = Epilogue()
    for name, t in (("bias", bias), ("rowbias", rowbias), ("gamma", gamma)):
        if t is not None:
            _need_contig(t, torch.float32, name)
            setattr(e, name, t.data_ptr())
    e.rdiv, e.rmod = int(rdiv), int(rmod)
    if res is not None:
        _need(res, dt, "res")
        assert res.stride(-1) == 1
        e.res, e.ldres = res.data_ptr(), res.stride(-2) if res.dim() >= 2 else res.shape[-1]
    if res2 is not None:
        _need(res2, dt, "res2")
        assert res2.stride(-1) == 1
        e.res2, e.ldres2 = res2.data_ptr(), res2.stride(-2) if res2.dim() >= 2 else res2.shape[-1]
    e.act, e.store = int(act), int(store)
    e.ps_k, e.ps_cout, e.ps_hin, e.ps_win = (int(v) for v in ps)
    return e


def gemm(x: Tensor, w: Tensor, *, bias=None, rowbias=None, rdiv=1, rmod=1, gamma=None, res=None,
         res2=None, act=ACT_NONE, out: Optional[Tensor] = None, tag: Optional[str] = None) -> Tensor:
    """out[M, N'] = epi(x[M, K] @ w[N, K]^T); N' = N (N/2 for GEGLU). x may be a row-strided view.
    fp16 x/w -> vda_gemm; fp32 x/w -> vda_gemm_f32 (fp32 mode)."""
    dt = _dt(x)
    _need(x, dt, "x")
    _need_contig(w, dt, "w")
    assert x.dim() == 2 and x.stride(1) == 1, "x must be a 2-D row-major (possibly row-strided) matrix"
    M, K = x.shape
    N = w.shape[0]
    assert w.shape[1] == K, f"K mismatch {w.shape} vs {x.shape}"
    nout = N // 2 if act == ACT_GEGLU else N
    if out is None:
        out = torch.empty((M, nout), dtype=dt, device=x.device)
    assert out.dim() == 2 and out.stride(1) == 1 and out.shape == (M, nout) and out.dtype == dt
    e = _epilogue(bias, rowbias, rdiv, rmod, gamma, res, res2, act, dt=dt)
    probe = _PROBE is not None and tag in _PROBE
    if probe:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
    fn = _lib.lib().vda_gemm if dt == torch.float16 else _lib.lib().vda_gemm_f32
    rc = fn(x.data_ptr(), x.stride(0), w.data_ptr(), out.data_ptr(), out.stride(0), M, N, K, e, _stream(x))
    if probe:
        ev1.record()
        _PROBE[tag].append((ev0, ev1, 2.0 * M * N * K))
    check(rc, "vda_gemm")
    return out


def conv_transpose_ks(x: Tensor, w: Tensor, bias: Tensor, BT: int, h: int, w_: int, k: int) -> Tensor:
    """ConvTranspose2d(kernel = stride = k) as one GEMM with a pixel-shuffle store.
    x [BT*h*w, Cin]; w [k*k*Cout, Cin] packed (i, j, co); bias [k*k*Cout] fp32 -> [BT, h*k, w*k, Cout]."""
    dt = _dt(x)
    _need(x, dt, "x")
    _need_contig(w, dt, "w")
    M, K = x.shape
    N = w.shape[0]
    cout = N // (k * k)
    out = torch.empty((BT, h * k, w_ * k, cout), dtype=dt, device=x.device)
    e = _epilogue(bias=bias, store=STORE_PIXEL_SHUFFLE, ps=(k, cout, h, w_), dt=dt)
    fn = _lib.lib().vda_gemm if dt == torch.float16 else _lib.lib().vda_gemm_f32
    rc = fn(x.data_ptr(), x.stride(0), w.data_ptr(), out.data_ptr(), N, M, N, K, e, _stream(x))
    check(rc, "vda_gemm(pixel-shuffle)")
    return out


def conv2d(x: Tensor, w: Tensor, *, ks=3, stride=1, pad=1, bias=None, pre_relu=False, act=ACT_NONE,
           res=None, res2=None, up=None) -> Tensor:
    """NHWC conv.  x [BT, H, W, Cin] fp16; w [Cout, ks, ks, Cin] fp16 -> [BT, Ho, Wo, Cout].
    `up=(Hu, Wu)` reads x through a bilinear align_corners=True resize to (Hu, Wu) first."""
    dt = _dt(x)
    _need_contig(x, dt, "x")
    _need_contig(w, dt, "w")
    BT, H, W, Cin = x.shape
    Cout = w.shape[0]
    assert w.shape[1:] == (ks, ks, Cin), f"weight {tuple(w.shape)} vs Cin={Cin} ks={ks}"
    Hi, Wi = (up if up is not None else (H, W))
    Ho = (Hi + 2 * pad - ks) // stride + 1
    Wo = (Wi + 2 * pad - ks) // stride + 1
    out = torch.empty((BT, Ho, Wo, Cout), dtype=dt, device=x.device)
    r = res.reshape(-1, Cout) if res is not None else None
    r2 = res2.reshape(-1, Cout) if res2 is not None else None
    e = _epilogue(bias=bias, res=r, res2=r2, act=act, dt=dt)
    uh, uw = (up if up is not None else (0, 0))
    if dt == torch.float32:
        if up is not None:
            raise RuntimeError("vda conv2d: the fused-upsample loader is fp16-only")
        rc = _lib.lib().vda_conv2d_f32(x.data_ptr(), w.data_ptr(), out.data_ptr(), BT, H, W, Cin, Cout, ks, stride,
                                       pad, int(bool(pre_relu)), e, _stream(x))
        check(rc, "vda_conv2d_f32")
        return out
    rc = _lib.lib().vda_conv2d(x.data_ptr(), w.data_ptr(), out.data_ptr(), BT, H, W, Cin, Cout, ks, stride, pad,
                               int(bool(pre_relu)), uh, uw, e, _stream(x))
    check(rc, "vda_conv2d")
    return out


def layernorm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float, *, skip_period: int = 0,
              rows: Optional[int] = None, out: Optional[Tensor] = None) -> Tensor:
    """Row LayerNorm of x [R, C] (row-strided ok).  skip_period=np drops each frame's cls row.
    ``out`` (contiguous [rows, C]) may be a slice of a larger buffer."""
    dt = _dt(x)
    _need(x, dt, "x")
    _need_contig(gamma, torch.float32, "gamma")
    _need_contig(beta, torch.float32, "beta")
    assert x.dim() == 2 and x.stride(1) == 1
    R, C = x.shape
    if rows is None:
        rows = R if skip_period == 0 else (R // (skip_period + 1)) * skip_period
    if out is None:
        out = torch.empty((rows, C), dtype=dt, device=x.device)
    _need_contig(out, dt, "out")
    assert out.shape == (rows, C)
    fn = _lib.lib().vda_layernorm if dt == torch.float16 else _lib.lib().vda_layernorm_f32
    rc = fn(x.data_ptr(), x.stride(0), out.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                  rows, C, float(eps), int(skip_period), _stream(x))
    check(rc, "vda_layernorm")
    return out


def groupnorm(x: Tensor, gamma: Tensor, beta: Tensor, frames: int, groups: int, eps: float) -> Tensor:
    """GroupNorm on NHWC frames: x [F*S, C] -> same."""
    dt = _dt(x)
    _need_contig(x, dt, "x")
    R, C = x.shape
    S = R // frames
    out = torch.empty_like(x)
    if dt == torch.float32:
        rc = _lib.lib().vda_groupnorm_f32(x.data_ptr(), out.data_ptr(), gamma.data_ptr(), beta.data_ptr(), frames, S,
                                          C, groups, float(eps), _stream(x))
    else:
        nws = _lib.lib().vda_groupnorm_workspace(frames, S, C, groups)
        ws = torch.empty((nws,), dtype=torch.float32, device=x.device)
        rc = _lib.lib().vda_groupnorm(x.data_ptr(), out.data_ptr(), gamma.data_ptr(), beta.data_ptr(), frames, S, C,
                                      groups, float(eps), ws.data_ptr(), _stream(x))
    check(rc, "vda_groupnorm")
    return out


def spatial_attention(qkv: Tensor, B: int, N: int, H: int, D: int = 64) -> Tensor:
    dt = _dt(qkv)
    _need_contig(qkv, dt, "qkv")
    assert qkv.shape == (B * N, 3 * H * D)
    out = torch.empty((B * N, H * D), dtype=dt, device=qkv.device)
    fn = _lib.lib().vda_spatial_attention if dt == torch.float16 else _lib.lib().vda_spatial_attention_f32
    rc = fn(qkv.data_ptr(), out.data_ptr(), B, N, H, D, float(D) ** -0.5,
                                          _stream(qkv))
    check(rc, "vda_spatial_attention")
    return out


def temporal_attention(qkv: Tensor, B: int, T: int, S: int, H: int, D: int, rope_theta: float = 0.0) -> Tensor:
    """Softmax attention over the T frames of every site; ``rope_theta`` > 0 rotates q and k first
    (pe='rope', attention.py:403-429: pairs (2i, 2i+1) of all H*D channels, angle t * theta^(-2i/C))."""
    dt = _dt(qkv)
    _need_contig(qkv, dt, "qkv")
    assert qkv.shape == (B * T * S, 3 * H * D)
    out = torch.empty((B * T * S, H * D), dtype=dt, device=qkv.device)
    fn = _lib.lib().vda_temporal_attention if dt == torch.float16 else _lib.lib().vda_temporal_attention_f32
    rc = fn(qkv.data_ptr(), out.data_ptr(), B, T, S, H, D, float(D) ** -0.5, float(rope_theta), _stream(qkv))
    check(rc, "vda_temporal_attention")
    return out


def upsample_bilinear(x: Tensor, Ho: int, Wo: int) -> Tensor:
    dt = _dt(x)
    _need_contig(x, dt, "x")
    BT, H, W, C = x.shape
    out = torch.empty((BT, Ho, Wo, C), dtype=dt, device=x.device)
    fn = _lib.lib().vda_upsample_bilinear if dt == torch.float16 else _lib.lib().vda_upsample_bilinear_f32
    rc = fn(x.data_ptr(), out.data_ptr(), BT, H, W, C, Ho, Wo, _stream(x))
    check(rc, "vda_upsample_bilinear")
    return out


def patch_im2col(img: Tensor, Kp: int, dtype=torch.float16) -> Tensor:
    """images [BT, 3, H, W] fp32 -> im2col rows [BT*(1+np), Kp] of ``dtype`` (fp16, or fp32 for fp32 mode)."""
    _need_contig(img, torch.float32, "img")
    BT, _, H, W = img.shape
    np_ = (H // 14) * (W // 14)
    out = torch.empty((BT * (1 + np_), Kp), dtype=dtype, device=img.device)
    fn = _lib.lib().vda_patch_im2col if dtype == torch.float16 else _lib.lib().vda_patch_im2col_f32
    rc = fn(img.data_ptr(), out.data_ptr(), BT, H, W, Kp, _stream(img))
    check(rc, "vda_patch_im2col")
    return out


def depth_head(x: Tensor, w1_split: Tensor, b1: Tensor, w2: Tensor, b2: Tensor, Ho: int, Wo: int) -> Tensor:
    """Depth tail: bilinear resize to (Ho, Wo), 3x3 conv (split-fp16 fp32 weights) -> ReLU -> 1x1 -> ReLU.
    x [BT, H, W, C] fp16; w1_split [64, 3, 3, C] fp16 (hi rows 0..31, lo rows 32..63) -> depth [BT, Ho, Wo] fp32."""
    _need_contig(x, torch.float16, "x")
    _need_contig(w1_split, torch.float16, "w1_split")
    for n, t in (("b1", b1), ("w2", w2), ("b2", b2)):
        _need_contig(t, torch.float32, n)
    BT, H, W, C = x.shape
    assert w1_split.shape == (64, 3, 3, C)
    ws = torch.empty((BT, Ho, Wo, C), dtype=torch.float16, device=x.device)
    out = torch.empty((BT, Ho, Wo), dtype=torch.float32, device=x.device)
    rc = _lib.lib().vda_depth_head(x.data_ptr(), w1_split.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                                   out.data_ptr(), ws.data_ptr(), BT, H, W, C, Ho, Wo, _stream(x))
    check(rc, "vda_depth_head")
    return out


def preprocess_frames(frames: Tensor, H: int, W: int, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)) -> Tensor:
    """uint8 frames [N, h, w, 3] (GPU) -> normalised network input [N, 3, H, W] fp32 (bicubic resize)."""
    _need(frames, torch.uint8, "frames")
    if frames.dim() != 4 or frames.shape[-1] != 3:
        raise ValueError(f"frames must be [N, h, w, 3] uint8, got {tuple(frames.shape)}")
    frames = frames.contiguous()
    N, h, w, _ = frames.shape
    out = torch.empty((N, 3, H, W), dtype=torch.float32, device=frames.device)
    if N == 0:
        return out
    m3 = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s3 = (ctypes.c_float * 3)(*[float(v) for v in std])
    rc = _lib.lib().vda_preprocess_frames(frames.data_ptr(), out.data_ptr(), N, h, w, H, W, m3, s3, _stream(frames))
    check(rc, "vda_preprocess_frames")
    return out


def depth_resize(depth: Tensor, ho: int, wo: int) -> Tensor:
    """depth [N, H, W] fp32 (GPU) -> [N, ho, wo] fp32, bilinear align_corners=True."""
    _need_contig(depth, torch.float32, "depth")
    N, H, W = depth.shape
    out = torch.empty((N, ho, wo), dtype=torch.float32, device=depth.device)
    if N == 0:
        return out
    rc = _lib.lib().vda_depth_resize(depth.data_ptr(), out.data_ptr(), N, H, W, ho, wo, _stream(depth))
    check(rc, "vda_depth_resize")
    return out


def depth_head_f32(x: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor, Ho: int, Wo: int) -> Tensor:
    """fp32-mode depth tail: x [BT, H, W, C] fp32; w1 [32, 3, 3, C] fp32 -> depth [BT, Ho, Wo] fp32."""
    _need_contig(x, torch.float32, "x")
    for n, t in (("w1", w1), ("b1", b1), ("w2", w2), ("b2", b2)):
        _need_contig(t, torch.float32, n)
    BT, H, W, C = x.shape
    assert w1.shape == (32, 3, 3, C)
    up = torch.empty((BT, Ho, Wo, C), dtype=torch.float32, device=x.device)
    mid = torch.empty((BT * Ho * Wo, 32), dtype=torch.float32, device=x.device)
    out = torch.empty((BT, Ho, Wo), dtype=torch.float32, device=x.device)
    rc = _lib.lib().vda_depth_head_f32(x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(),
                                       out.data_ptr(), up.data_ptr(), mid.data_ptr(), BT, H, W, C, Ho, Wo, _stream(x))
    check(rc, "vda_depth_head_f32")
    return out

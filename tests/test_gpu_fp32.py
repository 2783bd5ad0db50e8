"""fp32 mode (infer_video_depth(fp32=True): the reference's autocast-off path) on the exact-f32 MFMA.

Parity tier (i) of SURVEY.md §8(d): fp32 mode vs the reference's fp32 goldens, bar rel-L1 <= 1e-5
(summation-order rounding only).  Per-op tests compare each *_f32 entry point with torch fp32 on the
CPU at 2e-6 rel-L1 (exact-f32 products, fp32 accumulation in a different order).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import vda_amd
from vda_amd import ops
from vda_amd._lib import ACT_GELU, ACT_GEGLU, ACT_RELU
from vda_amd.model import _geglu_interleave
from helpers import GOLDEN_CASES, load_golden, recipe_state_dict, rel_l1, vda_oracle

pytestmark = pytest.mark.gpu
TOL_OP = 2e-6
TOL_MODEL = 1e-5  # SURVEY.md §8(d) tier (i)


def c(t):
    return t.to("cuda", torch.float32).contiguous()


def rnd(*s, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*s, generator=g, dtype=torch.float64).float() * scale


def rel(a, b):
    return rel_l1(a.cpu(), b.cpu())


@pytest.mark.parametrize("M,N,K", [(300, 384, 200), (1370, 1152, 384), (77, 64, 96), (5, 48, 8), (129, 132, 588)])
def test_gemm_f32_epilogues(M, N, K):
    x, w, b = rnd(M, K, seed=1), rnd(N, K, scale=K ** -0.5, seed=2), rnd(N, scale=0.1, seed=3)
    ref = x.double() @ w.double().t() + b.double()
    assert rel(ops.gemm(c(x), c(w), bias=c(b)), ref) < TOL_OP
    assert rel(ops.gemm(c(x), c(w), bias=c(b), act=ACT_GELU), F.gelu(ref)) < TOL_OP
    assert rel(ops.gemm(c(x), c(w), bias=c(b), act=ACT_RELU), F.relu(ref)) < TOL_OP
    gam, res, res2 = rnd(N, seed=7).abs() + 0.1, rnd(M, N, seed=8), rnd(M, N, seed=9)
    r = c(res)
    ops.gemm(c(x), c(w), bias=c(b), gamma=c(gam), res=r, res2=c(res2), out=r)
    assert rel(r, res.double() + res2.double() + gam.double() * ref) < TOL_OP
    T, S = 7, 11
    rb = rnd(T, N, seed=10)
    y = ops.gemm(c(x), c(w), rowbias=c(rb), rdiv=S, rmod=T)
    assert rel(y, x.double() @ w.double().t() + rb.double()[(torch.arange(M) // S) % T]) < TOL_OP


def test_gemm_f32_geglu_and_pixel_shuffle():
    M, I, K = 333, 96, 64
    x, w, b = rnd(M, K, seed=11), rnd(2 * I, K, scale=K ** -0.5, seed=12), rnd(2 * I, scale=0.1, seed=13)
    y = ops.gemm(c(x), c(_geglu_interleave(w)), bias=c(_geglu_interleave(b)), act=ACT_GEGLU)
    hg = x.double() @ w.double().t() + b.double()
    assert rel(y, hg[:, :I] * F.gelu(hg[:, I:])) < TOL_OP
    BT, hh, ww, Cin, Cout, k = 2, 5, 7, 32, 24, 4
    xi = rnd(BT, Cin, hh, ww, seed=14)
    wt, bt = rnd(Cin, Cout, k, k, scale=0.1, seed=15), rnd(Cout, seed=16)
    ref = F.conv_transpose2d(xi.double(), wt.double(), bt.double(), stride=k).permute(0, 2, 3, 1)
    wp = wt.permute(2, 3, 1, 0).reshape(k * k * Cout, Cin)
    y = ops.conv_transpose_ks(c(xi.permute(0, 2, 3, 1).reshape(-1, Cin)), c(wp), c(bt.repeat(k * k)), BT, hh, ww, k)
    assert rel(y, ref) < TOL_OP


@pytest.mark.parametrize("Cin,Cout,stride,pre_relu", [(64, 48, 1, False), (32, 64, 2, False), (128, 32, 1, True)])
def test_conv_f32(Cin, Cout, stride, pre_relu):
    x = rnd(2, Cin, 19, 23, seed=20)
    w, b = rnd(Cout, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=21), rnd(Cout, scale=0.1, seed=22)
    xin = F.relu(x) if pre_relu else x
    ref = F.conv2d(xin.double(), w.double(), b.double(), stride=stride, padding=1).permute(0, 2, 3, 1)
    res = rnd(*ref.shape, seed=23)
    y = ops.conv2d(c(x.permute(0, 2, 3, 1)), c(w.permute(0, 2, 3, 1)), stride=stride, bias=c(b), pre_relu=pre_relu,
                   act=ACT_RELU, res=c(res))
    assert rel(y, res.double() + F.relu(ref)) < TOL_OP


def test_attention_f32():
    B, N, H, D = 2, 150, 3, 64
    qkv = rnd(B * N, 3 * H * D, seed=30)
    q, k, v = qkv.double().view(B, N, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = ((q * D ** -0.5) @ k.transpose(-1, -2)).softmax(-1) @ v
    y = ops.spatial_attention(c(qkv), B, N, H, D)
    assert rel(y, ref.permute(0, 2, 1, 3).reshape(B * N, H * D)) < TOL_OP
    for (Bt, T, S, Ht, Dt) in [(1, 32, 37, 8, 128), (2, 7, 5, 8, 24), (1, 32, 9, 8, 8)]:
        qkv = rnd(Bt * T * S, 3 * Ht * Dt, seed=31 + T)
        y = ops.temporal_attention(c(qkv), Bt, T, S, Ht, Dt)
        t = qkv.double().view(Bt, T, S, 3, Ht, Dt).permute(3, 0, 2, 4, 1, 5)  # [3, B, S, H, T, D]
        o = ((t[0] @ t[1].transpose(-1, -2)) * Dt ** -0.5).softmax(-1) @ t[2]
        assert rel(y, o.permute(0, 3, 1, 2, 4).reshape(Bt * T * S, Ht * Dt)) < TOL_OP


def test_norms_resize_f32():
    x = rnd(50, 1024, seed=40) * 3 + 1
    g, b = rnd(1024, seed=41), rnd(1024, seed=42)
    assert rel(ops.layernorm(c(x), c(g), c(b), 1e-6), F.layer_norm(x.double(), (1024,), g.double(), b.double(), 1e-6)) < TOL_OP
    y = ops.layernorm(c(x), c(g), c(b), 1e-6, skip_period=9)  # 5 frames of 1 + 9 tokens
    ref = F.layer_norm(x.view(5, 10, 1024)[:, 1:].reshape(45, 1024).double(), (1024,), g.double(), b.double(), 1e-6)
    assert rel(y, ref) < TOL_OP
    F_, S, C = 3, 37, 256
    xg = rnd(F_ * S, C, seed=43)
    gg, bg = rnd(C, seed=44), rnd(C, seed=45)
    ref = F.group_norm(xg.view(F_, S, C).permute(0, 2, 1).double(), 32, gg.double(), bg.double(), 1e-6)
    assert rel(ops.groupnorm(c(xg), c(gg), c(bg), F_, 32, 1e-6), ref.permute(0, 2, 1).reshape(F_ * S, C)) < TOL_OP
    xu = rnd(2, 8, 13, 12, seed=46)
    ref = F.interpolate(xu.double(), size=(29, 31), mode="bilinear", align_corners=True).permute(0, 2, 3, 1)
    assert rel(ops.upsample_bilinear(c(xu.permute(0, 2, 3, 1)), 29, 31), ref) < TOL_OP


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_fp32_forward_matches_reference_golden(name):
    x, depth, _, meta = load_golden(name)
    m = _model(meta["encoder"])
    d = m(x.cuda(), skip_tmp_block=meta["skip_tmp_block"], fp32=True).cpu()
    assert d.dtype == torch.float32 and d.shape == depth.shape
    err = rel_l1(d, depth)
    print(f"fp32 {name}: rel-L1 vs reference = {err:.3e}")
    assert err <= TOL_MODEL


def test_fp32_video_and_stream_match_reference():
    import json
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "video_vits_57f.npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    m = _model("vits")
    d, _ = m.infer_video_depth(z["frames"], meta["fps"], input_size=meta["input_size"], fp32=True)
    err = float(np.abs(d - z["depth"]).sum() / np.abs(z["depth"]).sum())
    print(f"fp32 video: rel-L1 vs reference = {err:.3e}")
    assert err <= TOL_MODEL
    s = np.load(os.path.join(os.path.dirname(__file__), "golden", "stream_vits_50f.npz"), allow_pickle=False)
    sm = json.loads(str(s["meta"]))
    d, _ = m.infere_single_image(s["frames"], 24, input_size=sm["input_size"], fp32=True, **sm["cases"]["kf2_12"])
    err = float(np.abs(d - s["depth_kf2_12"]).sum() / np.abs(s["depth_kf2_12"]).sum())
    print(f"fp32 stream kf2_12: rel-L1 vs reference = {err:.3e}")
    assert err <= TOL_MODEL


_M = {}


def _model(enc):
    if enc not in _M:
        _M[enc] = vda_amd.build_model(enc, recipe_state_dict(enc), device="cuda")
    return _M[enc]

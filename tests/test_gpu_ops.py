"""Per-kernel parity: each libvda entry point (through the C ABI) vs a torch fp32 CPU reference.

Tolerances are stated per test; they cover fp16 storage of inputs/outputs with fp32 accumulation.
"""
import math

import pytest
import torch
import torch.nn.functional as F

import vda_amd
from vda_amd import ops
from vda_amd._lib import ACT_GELU, ACT_GEGLU, ACT_RELU, Epilogue
from vda_amd.model import _geglu_interleave
from tunelib import tune_lib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().sum() / b.abs().sum().clamp_min(1e-30))


def h(t):
    return t.to(DEV, torch.float16).contiguous()


def f32(t):
    return t.to(DEV, torch.float32).contiguous()


def rnd(*s, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*s, generator=g) * scale).half().float()


@pytest.mark.parametrize("M,N,K", [(300, 384, 200), (128, 128, 64), (1370, 1152, 384), (77, 64, 96), (5, 48, 8),
                                   (4000, 3072, 1024)])
def test_gemm_bias(M, N, K):
    x, w, b = rnd(M, K, seed=1), rnd(N, K, scale=K ** -0.5, seed=2), rnd(N, scale=0.1, seed=3)
    y = ops.gemm(h(x), h(w), bias=f32(b))
    ref = x @ w.t() + b
    assert rel(y, ref) < 2e-3  # fp16 output rounding


def test_gemm_gelu_ls_residual_rowbias():
    M, N, K = 700, 256, 320
    x, w, b = rnd(M, K, seed=4), rnd(N, K, scale=K ** -0.5, seed=5), rnd(N, scale=0.1, seed=6)
    gam, res = rnd(N, seed=7).abs() + 0.1, rnd(M, N, seed=8)
    y = ops.gemm(h(x), h(w), bias=f32(b), act=ACT_GELU)
    assert rel(y, F.gelu(x @ w.t() + b)) < 2e-3
    r = h(res)
    ops.gemm(h(x), h(w), bias=f32(b), gamma=f32(gam), res=r, out=r)  # in place, like the encoder
    assert rel(r, res + gam * (x @ w.t() + b)) < 2e-3
    T, S = 7, 100
    rb = rnd(T, N, seed=9)
    y = ops.gemm(h(x), h(w), rowbias=f32(rb), rdiv=S, rmod=T)
    ref = x @ w.t() + rb[(torch.arange(M) // S) % T]
    assert rel(y, ref) < 2e-3


@pytest.mark.parametrize("K", [64, 128, 192])
def test_gemm_persistent_tiles(K):
    """> 256 tiles: the dense phased GEMM walks tiles persistently, staggers half its blocks and
    streams the next tile's first K step under each epilogue (nk = 1, 2, 3 cover the prologue cases)."""
    M, N = 20000, 1024
    x, w, b = rnd(M, K, seed=31), rnd(N, K, scale=K ** -0.5, seed=32), rnd(N, scale=0.1, seed=33)
    ref = x @ w.t() + b
    assert rel(ops.gemm(h(x), h(w), bias=f32(b)), ref) < 2e-3
    assert rel(ops.gemm(h(x), h(w), bias=f32(b), act=ACT_GELU), F.gelu(ref)) < 2e-3
    res = rnd(M, N, seed=34)
    r = h(res)
    ops.gemm(h(x), h(w), bias=f32(b), res=r, out=r)
    assert rel(r, res + ref) < 2e-3
    gam = rnd(N, seed=35).abs() + 0.1
    r2 = h(res)
    ops.gemm(h(x), h(w), bias=f32(b), gamma=f32(gam), res=r2, res2=h(res), out=r2)
    assert rel(r2, 2 * res + gam * ref) < 2e-3
    T, S = 5, 4000
    rb = rnd(T, N, seed=36)
    y = ops.gemm(h(x), h(w), rowbias=f32(rb), rdiv=S, rmod=T)
    assert rel(y, x @ w.t() + rb[(torch.arange(M) // S) % T]) < 2e-3
    w2, b2 = rnd(2 * N, K, scale=K ** -0.5, seed=37), rnd(2 * N, scale=0.1, seed=38)
    y = ops.gemm(h(x), h(_geglu_interleave(w2)), bias=f32(_geglu_interleave(b2)), act=ACT_GEGLU)
    hh, g = (x @ w2.t() + b2).chunk(2, -1)
    assert rel(y, hh * F.gelu(g)) < 2e-3


def test_gemm_geglu():
    M, C = 333, 64
    x = rnd(M, C, seed=10)
    w = rnd(8 * C, C, scale=C ** -0.5, seed=11)
    b = rnd(8 * C, scale=0.1, seed=12)
    y = ops.gemm(h(x), h(_geglu_interleave(w)), bias=f32(_geglu_interleave(b)), act=ACT_GEGLU)
    hh, g = (x @ w.t() + b).chunk(2, -1)
    assert rel(y, hh * F.gelu(g)) < 2e-3


def test_gemm_strided_rows():
    M, N, K = 200, 128, 128
    big = rnd(M, 3 * K, seed=13)
    w = rnd(N, K, scale=K ** -0.5, seed=14)
    y = ops.gemm(h(big)[:, K:2 * K], h(w))
    assert rel(y, big[:, K:2 * K] @ w.t()) < 2e-3


@pytest.mark.parametrize("k,cin,cout,BT,hh,ww", [(4, 48, 48, 3, 5, 7), (2, 96, 96, 3, 5, 7), (4, 256, 256, 3, 5, 7),
                                                  # large M: the phased 256x256 kernel with the pixel-shuffle store
                                                  (4, 256, 256, 4, 37, 37), (2, 512, 512, 4, 37, 37),
                                                  # the staged row epilogue's remapped whole-pixel stores (cout %
                                                  # 256 == 0, w >= 16), ragged tiles and row wraps
                                                  (4, 256, 256, 12, 19, 23), (2, 512, 512, 6, 17, 41)])
def test_conv_transpose_pixel_shuffle(k, cin, cout, BT, hh, ww):
    x = rnd(BT, cin, hh, ww, seed=15)
    w = rnd(cin, cout, k, k, scale=cin ** -0.5, seed=16)
    b = rnd(cout, scale=0.1, seed=17)
    ref = F.conv_transpose2d(x, w, b, stride=k).permute(0, 2, 3, 1)
    wp = w.permute(2, 3, 1, 0).reshape(k * k * cout, cin)
    y = ops.conv_transpose_ks(h(x.permute(0, 2, 3, 1).reshape(-1, cin)), h(wp), f32(b.repeat(k * k)), BT, hh, ww, k)
    assert rel(y, ref) < 2e-3


@pytest.mark.parametrize("cin,cout,stride,H,W,BT", [(64, 64, 1, 9, 11, 2), (48, 64, 1, 12, 12, 2), (256, 256, 1, 19, 19, 2),
                                                    (384, 384, 2, 9, 9, 2), (1024, 256, 1, 5, 5, 2), (96, 32, 1, 3, 4, 2),
                                                    # large M: the phased 256x256 kernel (uniform-tap / general loaders)
                                                    (256, 256, 1, 40, 40, 4), (48, 256, 1, 40, 40, 4),
                                                    (512, 256, 2, 60, 60, 8), (256, 128, 1, 60, 60, 4)])
def test_conv3x3(cin, cout, stride, H, W, BT):
    x = rnd(BT, cin, H, W, seed=18)
    w = rnd(cout, cin, 3, 3, scale=(9 * cin) ** -0.5, seed=19)
    b = rnd(cout, scale=0.1, seed=20)
    ref = F.conv2d(x, w, b, stride=stride, padding=1)
    y = ops.conv2d(h(x.permute(0, 2, 3, 1)), h(w.permute(0, 2, 3, 1)), stride=stride, bias=f32(b))
    assert rel(y, ref.permute(0, 2, 3, 1)) < 2e-3


@pytest.mark.parametrize("cin,cout,H,W,BT", [(1024, 1024, 37, 37, 12), (512, 256, 60, 60, 8), (256, 512, 31, 45, 16)])
def test_conv3x3_stride2_im2col_route(cin, cout, H, W, BT):
    """Stride-2 3x3 convs with >= 4096 output pixels (the DPT reassemble's resize_layers[3], dpt.py:77-82)
    run as an explicit im2col into the workspace + the dense GEMM: bit-identical to the implicit-GEMM
    conv (the same K order), and vs torch fp32."""
    x = rnd(BT, cin, H, W, seed=21)
    w = rnd(cout, cin, 3, 3, scale=(9 * cin) ** -0.5, seed=22)
    b = rnd(cout, scale=0.1, seed=23)
    xh, wh = h(x.permute(0, 2, 3, 1)), h(w.permute(0, 2, 3, 1))
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    assert vda_amd._libvda().vda_conv2d_workspace(BT, H, W, cin, cout, 3, 2, 1) == BT * Ho * Wo * 9 * cin * 2
    y = ops.conv2d(xh, wh, stride=2, bias=f32(b))
    T = tune_lib()
    with T.route(force_tile=-2):  # every special route off: the implicit-GEMM conv
        assert T.lib.vda_conv2d_workspace(BT, H, W, cin, cout, 3, 2, 1) == 0
        y_imp = T.conv2d(xh, wh, stride=2, bias=f32(b))
    assert torch.equal(y, y_imp)
    ref = F.conv2d(x, w, b, stride=2, padding=1).permute(0, 2, 3, 1)
    assert rel(y, ref) < 2e-3


def test_conv3x3_rcu_fusion_epilogue():
    """out = x0 + conv2(relu(conv1(relu(x1)))) + x1  (blocks.py:78-91, :146-150)."""
    BT, C, H, W = 2, 64, 10, 13
    x0, x1 = rnd(BT, C, H, W, seed=21), rnd(BT, C, H, W, seed=22)
    w1, w2 = rnd(C, C, 3, 3, scale=(9 * C) ** -0.5, seed=23), rnd(C, C, 3, 3, scale=(9 * C) ** -0.5, seed=24)
    b1, b2 = rnd(C, scale=0.1, seed=25), rnd(C, scale=0.1, seed=26)
    t = F.relu(F.conv2d(F.relu(x1), w1, b1, padding=1))
    ref = F.conv2d(t, w2, b2, padding=1) + x1 + x0
    nh = lambda t: h(t.permute(0, 2, 3, 1).contiguous())
    tt = ops.conv2d(nh(x1), nh(w1), bias=f32(b1), pre_relu=True, act=ACT_RELU)
    y = ops.conv2d(tt, nh(w2), bias=f32(b2), res=nh(x1), res2=nh(x0))
    assert rel(y, ref.permute(0, 2, 3, 1)) < 3e-3


def test_conv3x3_fused_upsample():
    BT, C, H, W = 2, 64, 7, 9
    x = rnd(BT, C, H, W, seed=27)
    w = rnd(32, C, 3, 3, scale=(9 * C) ** -0.5, seed=28)
    b = rnd(32, scale=0.1, seed=29)
    up = F.interpolate(x, size=(14, 18), mode="bilinear", align_corners=True)
    ref = F.conv2d(up, w, b, padding=1)
    y = ops.conv2d(h(x.permute(0, 2, 3, 1)), h(w.permute(0, 2, 3, 1)), bias=f32(b), up=(14, 18))
    assert rel(y, ref.permute(0, 2, 3, 1)) < 3e-3


@pytest.mark.parametrize("C", [384, 1024, 256, 64, 128, 512])
def test_layernorm(C):
    R = 517
    x = rnd(R, C, seed=30) * 2 + 0.5
    g, b = rnd(C, seed=31) * 0.1 + 1, rnd(C, seed=32) * 0.1
    y = ops.layernorm(h(x), f32(g), f32(b), 1e-6)
    assert rel(y, F.layer_norm(x, (C,), g, b, eps=1e-6)) < 2e-3


@pytest.mark.parametrize("C", [384, 256])
def test_layernorm_skip_cls(C):
    BT, np_ = 3, 10
    x = rnd(BT, np_ + 1, C, seed=33)
    g, b = rnd(C, seed=34) * 0.1 + 1, rnd(C, seed=35) * 0.1
    y = ops.layernorm(h(x.reshape(-1, C)), f32(g), f32(b), 1e-6, skip_period=np_)
    ref = F.layer_norm(x, (C,), g, b, eps=1e-6)[:, 1:].reshape(-1, C)
    assert rel(y, ref) < 2e-3


@pytest.mark.parametrize("C,S", [(1024, 50), (256, 70), (384, 33), (64, 90), (192, 300), (256, 5476)])
def test_groupnorm(C, S):
    """Both GroupNorm paths: the workspace (three-pass, row-coalesced) path ops uses, and the
    one-block-per-group path the C ABI runs with ws = NULL; a large common offset checks that the
    shifted one-pass variance does not cancel."""
    Fr = 3
    x = rnd(Fr, S, C, seed=36) + 0.3
    x[1] += 40.0
    g, b = rnd(C, seed=37) * 0.1 + 1, rnd(C, seed=38) * 0.1
    xh = h(x.reshape(-1, C))
    y = ops.groupnorm(xh, f32(g), f32(b), Fr, 32, 1e-6)
    ref = F.group_norm(xh.float().cpu().view(Fr, S, C).permute(0, 2, 1), 32, g, b, eps=1e-6)
    ref = ref.permute(0, 2, 1).reshape(-1, C)
    assert rel(y, ref) < 2e-3
    assert torch.equal(y, ops.groupnorm(xh, f32(g), f32(b), Fr, 32, 1e-6))  # deterministic
    y0 = torch.empty_like(xh)
    gd, bd = f32(g), f32(b)  # keep the device copies alive across the launch
    rc = vda_amd._libvda().vda_groupnorm(xh.data_ptr(), y0.data_ptr(), gd.data_ptr(), bd.data_ptr(), Fr, S,
                                         C, 32, 1e-6, None, torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    assert rel(y0, ref) < 2e-3


@pytest.mark.parametrize("Fr,S,C,N", [(32, 1369, 256, 256), (4, 361, 256, 256), (2, 5476, 256, 256), (3, 12, 256, 256),
                                      (5, 37, 128, 128), (2, 70, 64, 64), (1, 7, 64, 64), (3, 50, 256, 512),
                                      (2, 33, 128, 64), (2, 361, 1024, 1024)])
def test_groupnorm_linear(Fr, S, C, N):
    """groupnorm_linear (motion_module.py:116-119: GroupNorm(32, eps 1e-6) then proj_in) against torch fp32
    GroupNorm -> Linear on the same fp16 inputs / weights.  (C, N) with N = C in {64, 128, 256} take the fused
    kernel (ragged tile tails: S = 12, 7, 37; frames shorter than a 32-row tile), the others the GroupNorm +
    GEMM composition.  Bar 2e-3 rel-L1 (fp16 output rounding and the fp16 normalised operand, as the reference's
    autocast GroupNorm -> Linear); against this library's composition 2e-4: the fused kernel forms gn_apply's
    operand bits and differs only in the fp32 accumulation order.  One frame
    carries a large offset (the shifted one-pass variance).  stats_out: per-row (sum, sumsq) of the stored
    fp16 output, checked against a recomputation from it."""
    x = rnd(Fr, S, C, seed=140) + 0.3
    x[Fr // 2] += 20.0
    g, b = rnd(C, seed=141) * 0.2 + 1, rnd(C, seed=142) * 0.2
    w, bias = rnd(N, C, scale=C ** -0.5, seed=143), rnd(N, scale=0.1, seed=144)
    xh = h(x.reshape(-1, C))
    gn = F.group_norm(xh.float().cpu().view(Fr, S, C).permute(0, 2, 1), 32, g, b, eps=1e-6)
    ref = gn.permute(0, 2, 1).reshape(-1, C) @ w.t() + bias
    fused = vda_amd._libvda().vda_groupnorm_linear_fused(C, 32, N) == 1
    assert fused == (N == C and C in (64, 128, 256))
    st = torch.full((Fr * S + 1, (N + 255) // 256, 2), float("nan"), device=DEV)
    y = ops.groupnorm_linear(xh, f32(g), f32(b), Fr, 32, 1e-6, h(w), bias=f32(bias), stats_out=st)
    assert y.shape == (Fr * S, N) and y.dtype == torch.float16
    assert rel(y, ref) < 2e-3
    unf = ops.gemm(ops.groupnorm(xh, f32(g), f32(b), Fr, 32, 1e-6), h(w), bias=f32(bias))
    assert rel(y, unf) < 2e-4  # and against this library's own two-kernel composition
    assert torch.equal(y, ops.groupnorm_linear(xh, f32(g), f32(b), Fr, 32, 1e-6, h(w), bias=f32(bias)))  # deterministic
    yf = y.float().view(Fr * S, -1, min(N, 256))
    exp = torch.stack([yf.sum(2), (yf * yf).sum(2)], -1)
    assert torch.allclose(st[:-1], exp, rtol=1e-5, atol=1e-3)
    assert torch.isnan(st[-1]).all()  # nothing written past row M - 1
    yn = ops.groupnorm_linear(xh, f32(g), f32(b), Fr, 32, 1e-6, h(w))  # no bias
    assert rel(yn, ref - bias) < 2e-3


def test_groupnorm_linear_large_rows():
    """The fused kernel at config-5's largest motion-module map (74 x 132 per frame, 32 frames: M = 312,576
    rows) against the GroupNorm + GEMM composition (round 6: bit-identical, tools/ab_gnl.py)."""
    Fr, S, C = 32, 74 * 132, 256
    torch.manual_seed(7)
    xh = (torch.randn(Fr * S, C, device=DEV) * 2 + 0.5).half()
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV) * 0.1
    w = (torch.randn(C, C, device=DEV) * C ** -0.5).half()
    bias = torch.randn(C, device=DEV) * 0.1
    y = ops.groupnorm_linear(xh, g, b, Fr, 32, 1e-6, w, bias=bias)
    unf = ops.gemm(ops.groupnorm(xh, g, b, Fr, 32, 1e-6), w, bias=bias)
    # the same operand bits (gn_apply's fma) and, against the phased GEMM, the same K order: bit-identical
    assert torch.equal(y, unf)


@pytest.mark.parametrize("BT,ntok,C,N,parts", [(4, 1370, 1024, 256, 0), (4, 1370, 1024, 512, 4), (12, 362, 384, 256, 0),
                                               (3, 1370, 1024, 1024, 4)])
def test_gemm_ln_fold_drop_period(BT, ntok, C, N, parts):
    """The DPT projects GEMM on an encoder tap with the final LayerNorm folded in and the cls rows dropped in the
    store (vda.h drop_period; dinov2.py:309-312 + dpt.py:60-68) against LayerNorm(skip_period) + GEMM: same
    rows, rel-L1 < 2e-3 (the fold's fp32 epilogue vs the fp16 normalised copy).  Statistics as row_stats
    ([M, 2]) or as 256-column partial sums ([M, P, 2], what the fc2 epilogue writes).  Frames of 1,370 and
    362 rows: tiles that start on a cls row, tiles crossing a frame boundary, a ragged last tile."""
    M = BT * ntok
    torch.manual_seed(5)
    x = (torch.randn(M, C, device=DEV) * 2 + 0.5).half()
    x[::97, :8] += 30.0  # a few rows with large channels (the residual stream's massive activations)
    gam = torch.rand(C, device=DEV) + 0.5
    bet = torch.randn(C, device=DEV) * 0.1
    w = torch.randn(N, C, device=DEV) * C ** -0.5
    b = torch.randn(N, device=DEV) * 0.1
    wg = (w * gam[None, :]).half()
    c1 = wg.float().sum(1)
    bb = w @ bet + b
    if parts:
        xf = x.float().view(M, parts, C // parts)
        st = torch.stack([xf.sum(-1), (xf * xf).sum(-1)], -1).contiguous()
    else:
        st = ops.row_stats(x, 1e-6)
    y = ops.gemm(x, wg, bias=bb, ln_stats=st, ln_parts=parts, ln_eps=1e-6, ln_colsum=c1, drop_period=ntok)
    assert y.shape == (BT * (ntok - 1), N)
    ref = ops.gemm(ops.layernorm(x, gam, bet, 1e-6, skip_period=ntok - 1), w.half(), bias=b)
    assert rel(y, ref) < 2e-3
    t = ops.layernorm(x, gam, bet, 1e-6).float().view(BT, ntok, C)[:, 1:].reshape(-1, C) @ w.half().float().t() + b
    assert rel(y, t) < 2e-3


def test_gemm_drop_period_validation():
    """drop_period is served by the phased route's LN-fold register epilogue only: other shapes are refused."""
    x = torch.zeros(4 * 362, 384, device=DEV, dtype=torch.float16)  # M = 1,448 < 4,096
    w = torch.zeros(256, 384, device=DEV, dtype=torch.float16)
    st = ops.row_stats(x, 1e-6)
    c1, bb = torch.zeros(256, device=DEV), torch.zeros(256, device=DEV)
    with pytest.raises(RuntimeError, match="drop_period"):
        ops.gemm(x, w, bias=bb, ln_stats=st, ln_colsum=c1, drop_period=362)
    x = torch.zeros(32 * 141, 384, device=DEV, dtype=torch.float16)  # frames of 141 rows < 256
    with pytest.raises(RuntimeError, match="drop_period"):
        ops.gemm(x, w, bias=bb, ln_stats=ops.row_stats(x, 1e-6), ln_colsum=c1, drop_period=141)


@pytest.mark.parametrize("B,N,H", [(2, 200, 3), (1, 1370, 16), (3, 82, 6), (1, 64, 1)])
def test_spatial_attention(B, N, H):
    D = 64
    qkv = rnd(B * N, 3 * H * D, seed=39)
    y = ops.spatial_attention(h(qkv), B, N, H, D)
    q, k, v = qkv.reshape(B, N, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = ((q @ k.transpose(-1, -2)) * D ** -0.5).softmax(-1) @ v
    ref = ref.transpose(1, 2).reshape(B * N, H * D)
    assert rel(y, ref) < 3e-3


@pytest.mark.parametrize("ramp", ["up", "spike", "down"])
def test_spatial_attention_rebase(ramp):
    """The online softmax re-bases only when a lane's P sum for a 64-key tile passes 2^15: keys whose
    scores climb tile after tile ("up": +~6 log2 units per tile), a single huge-score key late in the
    sequence ("spike": P would overflow fp16 without the re-base) and falling scores ("down": the
    first tile's reference stays, later P underflow towards 0) all match torch fp32."""
    B, N, H, D = 2, 600, 2, 64
    g = torch.Generator().manual_seed(7)
    q = torch.randn(B, N, H, D, generator=g)
    k = torch.randn(B, N, H, D, generator=g)
    v = torch.randn(B, N, H, D, generator=g)
    pos = torch.arange(N, dtype=torch.float32)[None, :, None, None]
    q = q + 1.0  # a common direction u = (1, ..., 1): q.u ~ D for every query
    if ramp == "up":  # + ~40 log2 units over the sequence (~4 per tile)
        k = k + pos / N * 3.5
    elif ramp == "spike":  # one key ~46 log2 units above the rest
        k[:, 500] = 4.0
    else:
        k = k + (N - pos) / N * 3.5
    qkv = torch.stack([q, k, v], 2).reshape(B * N, 3 * H * D).half().float()
    y = ops.spatial_attention(h(qkv), B, N, H, D)
    qq, kk, vv = qkv.reshape(B, N, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = ((qq @ kk.transpose(-1, -2)) * D ** -0.5).softmax(-1) @ vv
    ref = ref.transpose(1, 2).reshape(B * N, H * D)
    assert torch.isfinite(y.float()).all()
    assert rel(y, ref) < 3e-3


@pytest.mark.parametrize("B,T,S,D", [(1, 32, 37, 128), (1, 8, 10, 32), (2, 5, 9, 48), (1, 32, 20, 8), (1, 3, 4, 24)])
def test_temporal_attention(B, T, S, D):
    H = 8
    C = H * D
    qkv = rnd(B * T * S, 3 * C, seed=40) * 2
    y = ops.temporal_attention(h(qkv), B, T, S, H, D)
    t = qkv.reshape(B, T, S, 3, H, D).permute(3, 0, 2, 4, 1, 5)  # 3, B, S, H, T, D
    q, k, v = t[0], t[1], t[2]
    o = ((q @ k.transpose(-1, -2)) * D ** -0.5).softmax(-1) @ v  # B, S, H, T, D
    ref = o.permute(0, 3, 1, 2, 4).reshape(B * T * S, C)
    assert rel(y, ref) < 3e-3


def test_upsample_bilinear():
    x = rnd(2, 32, 19, 19, seed=41)
    ref = F.interpolate(x, size=(37, 37), mode="bilinear", align_corners=True)
    y = ops.upsample_bilinear(h(x.permute(0, 2, 3, 1)), 37, 37)
    assert rel(y, ref.permute(0, 2, 3, 1)) < 2e-3


def test_patch_embed_im2col_gemm():
    BT, H, W, C = 2, 42, 56, 64
    img = rnd(BT, 3, H, W, seed=42)
    w = rnd(C, 3, 14, 14, scale=588 ** -0.5, seed=43)
    b = rnd(C, scale=0.1, seed=44)
    ref = F.conv2d(img, w, b, stride=14).flatten(2).transpose(1, 2)  # [BT, np, C]
    a = ops.patch_im2col(img.to(DEV).contiguous(), 592)
    wp = F.pad(w.reshape(C, -1), (0, 4))
    np_ = (H // 14) * (W // 14)
    rb = torch.cat([torch.zeros(1, C), b.expand(np_, C)], 0)
    y = ops.gemm(a, h(wp), rowbias=f32(rb), rdiv=1, rmod=np_ + 1).view(BT, np_ + 1, C)
    assert float(y[:, 0].abs().max()) == 0.0
    assert rel(y[:, 1:], ref) < 2e-3


@pytest.mark.parametrize("C,Hin,Win,Ho,Wo,BT", [(32, 16, 20, 28, 42, 2), (128, 20, 24, 37, 51, 2), (64, 9, 9, 16, 16, 1),
                                                 (128, 37, 37, 70, 70, 3), (96, 10, 12, 20, 22, 1)])
def test_depth_head_fp32(C, Hin, Win, Ho, Wo, BT):
    """Depth tail: the halo-tiled kernel (C = 32 or C % 64 == 0; tile edges 16 with partial tiles here),
    the implicit-GEMM kernel (other C, and the tuning override) vs torch fp32."""
    x = rnd(BT, C, Hin, Win, seed=45)
    b1 = rnd(32, scale=0.1, seed=47)
    w2, b2 = rnd(1, 32, 1, 1, seed=48).abs() * 0.2, torch.tensor([0.05])
    w1 = torch.randn(32, C, 3, 3, generator=torch.Generator().manual_seed(46)) * (9 * C) ** -0.5  # full fp32 weights
    xh = h(x.permute(0, 2, 3, 1))
    up = F.interpolate(xh.float().cpu().permute(0, 3, 1, 2), size=(Ho, Wo), mode="bilinear", align_corners=True)
    up = up.half().float()  # the resized map is stored in fp16 (as the reference's autocast interpolate does)
    ref = F.relu(F.conv2d(F.relu(F.conv2d(up, w1, b1, padding=1)), w2, b2))[:, 0]
    wn = w1.permute(0, 2, 3, 1)
    split = torch.cat([wn.half(), (wn - wn.half().float()).half()], 0).to(DEV).contiguous()
    args = (split, f32(b1), f32(w2.reshape(-1)), f32(b2), Ho, Wo)
    y = ops.depth_head(xh, *args)
    # the conv keeps the fp32 weights as hi + lo fp16 halves (22 of 24 mantissa bits) with fp32
    # accumulation: agreement at ~1e-6
    assert rel(y, ref) < 1e-5
    T = tune_lib()
    assert torch.equal(T.depth_head(xh, *args), y)  # the tuning build's automatic route is the product's
    with T.route(force_tile=13):  # the implicit-GEMM depth kernel
        y_old = T.depth_head(xh, *args)
    assert rel(y_old, ref) < 1e-5


def test_ops_reject_cpu_tensors():
    with pytest.raises(RuntimeError):
        ops.gemm(torch.zeros(4, 8, dtype=torch.float16), torch.zeros(4, 8, dtype=torch.float16))


def test_c_abi_groupnorm_linear_direct():
    """vda_groupnorm_linear through ctypes with the caller's workspace (as a non-torch host would bind it,
    INTEGRATION.md) == torch.ops.vda.groupnorm_linear, bitwise, on both routes (fused C = 256; composed
    C = 256 -> N = 512), with stats_out."""
    from vda_amd import _lib
    import vda_amd.torch_ops  # noqa: F401
    lib = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    Fr, S, C = 3, 77, 256
    xh = h(rnd(Fr * S, C, seed=150) + 0.2)
    g, b = f32(rnd(C, seed=151) * 0.2 + 1), f32(rnd(C, seed=152) * 0.1)
    for N in (256, 512):
        wh, bias = h(rnd(N, C, scale=C ** -0.5, seed=153)), f32(rnd(N, scale=0.1, seed=154))
        nws = lib.vda_groupnorm_linear_workspace(Fr, S, C, 32, N)
        ws = torch.empty(nws, dtype=torch.uint8, device=DEV)
        y = torch.empty(Fr * S, N, dtype=torch.float16, device=DEV)
        so = torch.empty(Fr * S, (N + 255) // 256, 2, device=DEV)
        rc = lib.vda_groupnorm_linear(xh.data_ptr(), g.data_ptr(), b.data_ptr(), Fr, S, C, 32, 1e-6, wh.data_ptr(),
                                      bias.data_ptr(), y.data_ptr(), N, so.data_ptr(), ws.data_ptr(), nws, st)
        assert rc == 0, lib.vda_last_error()
        so1 = torch.empty_like(so)
        y1 = torch.ops.vda.groupnorm_linear(xh, g, b, Fr, 32, 1e-6, wh, bias, so1)
        assert torch.equal(y, y1) and torch.equal(so, so1)
        assert lib.vda_groupnorm_linear_fused(C, 32, N) == (1 if N == C else 0)


def test_c_abi_direct_matches_torch_ops():
    """The C ABI called straight through ctypes (as a non-torch host would) == torch.ops.vda.* (the native
    TORCH_LIBRARY registration over the same entry points), bitwise."""
    import ctypes
    from vda_amd import _lib
    import vda_amd.torch_ops  # noqa: F401
    lib = _lib.lib()
    st = torch.cuda.current_stream().cuda_stream
    x, w, b = rnd(300, 128, seed=70), rnd(256, 128, scale=128 ** -0.5, seed=71), rnd(256, scale=0.1, seed=72)
    xh, wh, bf = h(x), h(w), f32(b)
    y = torch.empty(300, 256, dtype=torch.float16, device=DEV)
    e = _lib.Epilogue()
    e.bias, e.rdiv, e.rmod, e.act = bf.data_ptr(), 1, 1, ACT_GELU
    assert lib.vda_gemm(xh.data_ptr(), 128, wh.data_ptr(), y.data_ptr(), 256, 300, 256, 128, ctypes.byref(e), st) == 0
    y1 = torch.ops.vda.gemm(xh, wh, bf, None, 1, 1, None, None, None, ACT_GELU)
    assert torch.equal(y, y1) and torch.equal(y, ops.gemm(xh, wh, bias=bf, act=ACT_GELU))
    m = h(rnd(2, 9, 11, 64, seed=73))
    assert torch.equal(torch.ops.vda.upsample_bilinear(m, 17, 21), ops.upsample_bilinear(m, 17, 21))
    # strip conv at 19^2 with Cin 1024 (layer4_rn): the caller's split workspace (C ABI) vs the op, which
    # allocates the same workspace per call from the caching allocator; and the unsplit (ws = NULL) run
    xc = h(rnd(4, 19, 19, 1024, seed=74))
    wc = h(rnd(256, 3, 3, 1024, scale=(9 * 1024) ** -0.5, seed=75))
    nws = lib.vda_conv2d_workspace(4, 19, 19, 1024, 256, 3, 1, 1)
    assert nws > 0
    ws = torch.empty(nws, dtype=torch.uint8, device=DEV)
    yc = torch.empty(4, 19, 19, 256, dtype=torch.float16, device=DEV)
    yn = torch.empty_like(yc)
    e0 = _lib.Epilogue()
    e0.rdiv = e0.rmod = 1
    args = (4, 19, 19, 1024, 256, 3, 1, 1, 0, 0, 0, ctypes.byref(e0))
    assert lib.vda_conv2d(xc.data_ptr(), wc.data_ptr(), yc.data_ptr(), *args, ws.data_ptr(), nws, st) == 0
    assert lib.vda_conv2d(xc.data_ptr(), wc.data_ptr(), yn.data_ptr(), *args, None, 0, st) == 0
    assert torch.equal(yc, ops.conv2d(xc, wc))
    ref = F.conv2d(xc.float().permute(0, 3, 1, 2), wc.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    assert rel(yc, ref) < 2e-3 and rel(yn, ref) < 2e-3


def test_depth_head_workspace_only_when_used():
    """The op allocates the resized-map workspace exactly when the library's path materialises the
    resize: the default (resize fused into the depth conv of vda_dconv.hip) none, the materialised
    variant (tuning build, vda_debug_dconv(2)) one [BT, 518, 518, C] fp16 map (no unused
    reservation), and both give the same depth."""
    x = h(rnd(2, 296, 296, 128, scale=0.5, seed=76))
    w1 = h(rnd(64, 3, 3, 128, scale=0.03, seed=77))
    b1, w2, b2 = f32(rnd(32, seed=78)), f32(rnd(32, seed=79)), f32(rnd(1, seed=80))

    def extra_bytes():
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        d = ops.depth_head(x, w1, b1, w2, b2, 518, 518)
        torch.cuda.synchronize()
        assert d.shape == (2, 518, 518)
        return torch.cuda.max_memory_allocated() - base, d

    dmap = 2 * 518 * 518 * 4
    extra, d0 = extra_bytes()  # default: resize fused into the depth conv
    assert extra <= dmap + (4 << 20), extra  # the fp32 depth (+ allocator rounding)
    assert vda_amd._libvda().vda_depth_head_workspace(2, 296, 296, 128, 518, 518) == 0
    T = tune_lib()
    with T.route(dconv=2):  # the same conv on a materialised resize: the library asks for one fp16 map
        assert T.depth_head_workspace(2, 296, 296, 128, 518, 518) == 2 * 518 * 518 * 128 * 2
        d1 = T.depth_head(x, w1, b1, w2, b2, 518, 518)
    assert torch.equal(d0, d1)


@pytest.mark.parametrize("Cin,H,W,relu", [(256, 130, 140, False), (128, 129, 131, True)])
def test_conv3x3_halo_cout128(Cin, H, W, relu):
    """3x3 convs with 128 outputs on maps >= 128^2 run the halo-tiled kernel (output_conv1, dpt.py:117);
    vs torch fp32 and vs the implicit-GEMM conv (tuning override)."""
    x = rnd(2, Cin, H, W, seed=80)
    w, b = rnd(128, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=81), rnd(128, scale=0.1, seed=82)
    ref = F.conv2d(x, w, b, padding=1)
    ref = (F.relu(ref) if relu else ref).permute(0, 2, 3, 1)
    xh, wh = h(x.permute(0, 2, 3, 1)), h(w.permute(0, 2, 3, 1))
    y = ops.conv2d(xh, wh, bias=f32(b), act=ACT_RELU if relu else 0)
    assert rel(y, ref) < 2e-3
    with tune_lib().route(force_tile=3) as T:
        y2 = T.conv2d(xh, wh, bias=f32(b), act=ACT_RELU if relu else 0)
    assert rel(y, y2) < 1e-3


@pytest.mark.parametrize("T,S,H,D", [(32, 37, 8, 128), (7, 5, 8, 24), (32, 9, 8, 32)])
def test_temporal_attention_rope(T, S, H, D):
    """rope_theta > 0: q/k channel pairs rotated by t * theta^(-2i/C) before the softmax (fp16 kernel)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import vda_oracle
    C = H * D
    qkv = rnd(T * S, 3 * C, seed=90 + D)
    y = ops.temporal_attention(h(qkv), 1, T, S, H, D, rope_theta=10000.0)
    t = qkv.half().float().view(T, S, 3, C).permute(1, 0, 2, 3)  # [S, T, 3, C]
    q = vda_oracle.rotary(t[:, :, 0].half()).float()  # rotated in fp32, rounded to fp16 like the reference
    k = vda_oracle.rotary(t[:, :, 1].half()).float()
    v = t[:, :, 2]
    sp = lambda z: z.reshape(S, T, H, D).permute(0, 2, 1, 3)  # noqa: E731
    o = ((sp(q) @ sp(k).transpose(-1, -2)) * D ** -0.5).softmax(-1) @ sp(v)
    ref = o.permute(2, 0, 1, 3).reshape(T * S, C)
    assert rel(y, ref) < 3e-3


@pytest.mark.parametrize("Cin,H,W,BT,mode", [(256, 148, 148, 2, "rcu2"), (256, 74, 74, 3, "rcu1"), (1024, 37, 37, 2, "plain"),
                                             (64, 17, 160, 2, "rcu2"), (32, 9, 16, 3, "rcu1"), (512, 5, 23, 2, "plain")])
def test_conv3x3_strip_cout256(Cin, H, W, BT, mode):
    """3x3 convs with 256 outputs on maps <= 160 wide on the strip-tiled halo kernel (layerN_rn,
    blocks.py:20-32; RCU conv1 with pre-ReLU + ReLU, conv2 with the skip and fusion adds,
    blocks.py:78-91 / :146-150); partial last tiles, tiles spanning 3 rows, Cin = 32 .. 1024.
    vs torch fp32 and vs the implicit-GEMM conv (tuning build: vda_debug_force_tile(-3) takes the strip
    kernel for every Cin, the default only for Cin >= 512 or under-filled grids; -2 never)."""
    x = rnd(BT, Cin, H, W, seed=90)
    w, b = rnd(256, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=91), rnd(256, scale=0.1, seed=92)
    r1, r2 = rnd(BT, 256, H, W, seed=93), rnd(BT, 256, H, W, seed=94)
    nh = lambda t: h(t.permute(0, 2, 3, 1).contiguous())
    kw = {}
    if mode == "plain":
        ref = F.conv2d(x, w, padding=1)
    elif mode == "rcu1":
        ref = F.relu(F.conv2d(F.relu(x), w, b, padding=1))
        kw = dict(bias=f32(b), pre_relu=True, act=ACT_RELU)
    else:
        ref = F.conv2d(x, w, b, padding=1) + r1 + r2
        kw = dict(bias=f32(b), res=nh(r1), res2=nh(r2))
    ref = ref.permute(0, 2, 3, 1)
    xh, wh = nh(x), nh(w)
    T = tune_lib()
    y0 = ops.conv2d(xh, wh, **kw)  # the product's route
    assert rel(y0, ref) < 2e-3
    with T.route(force_tile=-3):  # strip kernel for every Cin
        y = T.conv2d(xh, wh, **kw)
    assert rel(y, ref) < 2e-3
    with T.route(force_tile=-2):
        y2 = T.conv2d(xh, wh, **kw)
    assert rel(y, y2) < 1e-3


@pytest.mark.parametrize("Cin,H,W,BT,mode,split", [(1024, 19, 19, 4, "plain", 4), (256, 19, 19, 3, "rcu2", 4),
                                                   (256, 19, 19, 2, "rcu1", 8), (512, 17, 23, 2, "rcu2", 2),
                                                   (64, 19, 19, 2, "plain", 2), (256, 19, 19, 32, "rcu2", 0)])
def test_conv3x3_strip_split(Cin, H, W, BT, mode, split):
    """Strip conv with the input channels split over work items (fp32 partial slices summed in a
    fixed order by the finishing kernel, which applies bias / ReLU / the fp16 residual adds): the
    under-filled 19^2 maps (layer4_rn, refinenet4's RCU).  split 0 = the automatic choice.  vs torch
    fp32, vs the unsplit kernel, and bit-identical across runs (no atomics)."""
    x = rnd(BT, Cin, H, W, seed=190)
    w, b = rnd(256, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=191), rnd(256, scale=0.1, seed=192)
    r1, r2 = rnd(BT, 256, H, W, seed=193), rnd(BT, 256, H, W, seed=194)
    nh = lambda t: h(t.permute(0, 2, 3, 1).contiguous())
    kw = {}
    if mode == "plain":
        ref = F.conv2d(x, w, padding=1)
    elif mode == "rcu1":
        ref = F.relu(F.conv2d(F.relu(x), w, b, padding=1))
        kw = dict(bias=f32(b), pre_relu=True, act=ACT_RELU)
    else:
        ref = F.conv2d(x, w, b, padding=1) + r1 + r2
        kw = dict(bias=f32(b), res=nh(r1), res2=nh(r2))
    ref = ref.permute(0, 2, 3, 1)
    xh, wh = nh(x), nh(w)
    T = tune_lib()
    with T.route(force_tile=-3, strip_split=split):
        y = T.conv2d(xh, wh, **kw)
        y_again = T.conv2d(xh, wh, **kw)
    with T.route(force_tile=-3, strip_split=1):
        y1 = T.conv2d(xh, wh, **kw)
    assert torch.equal(y, y_again)
    assert rel(y, ref) < 2e-3
    assert rel(y, y1) < 1e-3


@pytest.mark.parametrize("C,Hin,Win,Ho,Wo,BT", [(128, 20, 24, 37, 51, 2), (64, 9, 9, 16, 16, 1), (128, 37, 37, 70, 70, 3),
                                                 (64, 30, 17, 53, 31, 2), (128, 12, 12, 12, 12, 1), (64, 5, 40, 33, 47, 1)])
def test_depth_head_fused_resize(C, Hin, Win, Ho, Wo, BT):
    """Depth tail with the bilinear resize fused into the patch building of the depth conv (default):
    bit-identical to the materialised resize + the same conv (tuning build: vda_debug_dconv(2)); and the
    older fused 8-wave halo conv (vda_debug_dconv(0)) bit-identical to the materialised resize + halo conv
    (vda_debug_force_tile(9)),
    both interpolating with the same fp32 formula and fp16 rounding; partial tiles, non-square maps,
    identity-size resize, aspect ratios far from 1."""
    x = rnd(BT, C, Hin, Win, seed=145)
    b1 = rnd(32, scale=0.1, seed=147)
    w2, b2 = rnd(1, 32, 1, 1, seed=148).abs() * 0.2, torch.tensor([0.05])
    w1 = torch.randn(32, C, 3, 3, generator=torch.Generator().manual_seed(146)) * (9 * C) ** -0.5
    xh = h(x.permute(0, 2, 3, 1))
    up = F.interpolate(xh.float().cpu().permute(0, 3, 1, 2), size=(Ho, Wo), mode="bilinear", align_corners=True)
    ref = F.relu(F.conv2d(F.relu(F.conv2d(up.half().float(), w1, b1, padding=1)), w2, b2))[:, 0]
    wn = w1.permute(0, 2, 3, 1)
    split = torch.cat([wn.half(), (wn - wn.half().float()).half()], 0).to(DEV).contiguous()
    args = (split, f32(b1), f32(w2.reshape(-1)), f32(b2), Ho, Wo)
    y = ops.depth_head(xh, *args)  # default: the 2-blocks-per-CU depth conv, resize fused into its patches
    T = tune_lib()
    with T.route(dconv=2):  # the same conv on a materialised resize
        y_mat2 = T.depth_head(xh, *args)
    assert torch.equal(y, y_mat2)
    with T.route(dconv=0):
        y_fused = T.depth_head(xh, *args)
    with T.route(force_tile=9):
        y_mat = T.depth_head(xh, *args)
    assert torch.equal(y_fused, y_mat)  # the older 8-wave halo kernels, fused vs materialised
    assert rel(y_fused, ref) < 1e-5
    assert rel(y, ref) < 1e-5


@pytest.mark.parametrize("BT,Cin,Hs,Ws,H,W,relu", [(2, 256, 70, 70, 140, 140, False), (2, 128, 64, 72, 128, 143, True),
                                                   (1, 64, 20, 150, 39, 299, False), (3, 128, 9, 9, 17, 17, False),
                                                   (4, 128, 148, 148, 296, 296, True)])
def test_conv3x3_halo_fused_resize(BT, Cin, Hs, Ws, H, W, relu):
    """output_conv1 shape class (3x3, Cout = 128) on a bilinear align_corners=True resize fused into the
    halo conv's patch staging: vs torch fp32, and bit-identical to resize + halo conv when the
    materialised path also takes the halo kernel (resized maps >= 128^2).  4 x 296^2: more tiles than CUs,
    so the interpolation waves build the next unit's patch across tile boundaries."""
    x = rnd(BT, Cin, Hs, Ws, seed=170)
    w = rnd(128, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=171)
    b = rnd(128, scale=0.1, seed=172)
    xh = h(x.permute(0, 2, 3, 1))
    up = F.interpolate(xh.float().cpu().permute(0, 3, 1, 2), size=(H, W), mode="bilinear", align_corners=True)
    ref = F.conv2d(up.half().float(), w, b, padding=1)
    if relu:
        ref = F.relu(ref)
    kw = dict(bias=f32(b), act=ACT_RELU if relu else 0)
    wh = h(w.permute(0, 2, 3, 1))
    y = ops.conv2d(xh, wh, up=(H, W), **kw)
    assert rel(y, ref.permute(0, 2, 3, 1)) < 2e-3
    if H * W >= 128 * 128:
        y_mat = ops.conv2d(ops.upsample_bilinear(xh, H, W), wh, **kw)
        assert torch.equal(y, y_mat)


@pytest.mark.parametrize("M,N,K,act", [(4001, 3072, 1024, 0), (4001, 4096, 1024, ACT_GELU), (301, 384, 384, 0),
                                       (300, 1536, 384, ACT_GELU), (43840, 1024, 1024, 0), (8200, 1024, 1024, ACT_GELU),
                                       (8200, 1152, 512, ACT_GELU), (5000, 768, 1024, 0)])
def test_gemm_layernorm_fold(M, N, K, act):
    """norm1 / norm2 folded into qkv / fc1 (block.py:84,87): rstd (x W'^T - mean colsum) + b' with
    W' = gamma (.) W, b' = W beta + b, stats from vda_row_stats, vs torch fp32 LayerNorm -> Linear."""
    g = torch.Generator().manual_seed(M + N)
    x = (torch.randn(M, K, generator=g) * 3 + torch.randn(M, 1, generator=g) * 2).half().float()  # row offsets
    gam = 1 + 0.2 * torch.randn(K, generator=g)
    bet = 0.1 * torch.randn(K, generator=g)
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = 0.1 * torch.randn(N, generator=g)
    ref = F.linear(F.layer_norm(x, (K,), gam, bet, eps=1e-6), w, b)
    if act == ACT_GELU:
        ref = F.gelu(ref)
    wg = (w * gam[None, :]).half()
    c1 = wg.float().sum(1)
    bb = w @ bet + b
    st = ops.row_stats(h(x), 1e-6)
    assert st.shape == ((M + 1) // 2 * 2, 2)
    mean, var = x.mean(1), x.var(1, unbiased=False)
    assert torch.allclose(st[:M, 0].cpu(), mean, atol=1e-4, rtol=1e-5)
    assert torch.allclose(st[:M, 1].cpu(), (var + 1e-6).rsqrt(), rtol=1e-4)
    y = ops.gemm(h(x), wg.to(DEV), bias=f32(bb), act=act, ln_stats=st, ln_colsum=f32(c1))
    err = rel(y, ref)
    # the unfused fp16 path for scale: LN output rounded to fp16, W rounded to fp16
    y0 = ops.gemm(ops.layernorm(h(x), f32(gam), f32(bet), 1e-6), h(w), bias=f32(b), act=act)
    err0 = rel(y0, ref)
    print(f"LN-folded GEMM {M}x{N}x{K} act={act}: rel-L1 {err:.2e} (unfused fp16 path {err0:.2e})")
    assert err < max(2 * err0, 2e-3)


@pytest.mark.parametrize("M,C", [(43808, 1024), (21904, 256), (4001, 256), (361, 1024), (300, 384)])
def test_gemm_layernorm_fold_geglu(M, C):
    """The motion modules' ff_norm folded into the GEGLU GEMM (motion_module.py:182, attention.py:363-384):
    the producer of the residual stream (to_out + residual) writes the row statistics (stats_out), the
    GEGLU GEMM applies rstd (h W'^T - mean colsum) + W beta + b to both halves before the gate, vs torch
    fp32 LayerNorm -> Linear -> GEGLU on the same stored fp16 residual.  Large M takes the phased
    256x256 kernel (LN-fold staged epilogue), small M the tile kernels (epi_geglu4)."""
    g = torch.Generator().manual_seed(M + C)
    inner = 4 * C
    a = (torch.randn(M, C, generator=g) * 0.5).half().float()          # attention output
    hres = (torch.randn(M, C, generator=g) * 2 + 1).half().float()    # residual stream before to_out
    wo, bo = torch.randn(C, C, generator=g) * C ** -0.5, 0.1 * torch.randn(C, generator=g)
    gam, bet = 1 + 0.2 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    w1, b1 = torch.randn(2 * inner, C, generator=g) * C ** -0.5, 0.1 * torch.randn(2 * inner, generator=g)
    st = torch.empty(M + 1, (C + 255) // 256, 2, device=DEV)
    hd = ops.gemm(h(a), h(wo), bias=f32(bo), res=h(hres), stats_out=st)  # to_out + residual, row statistics
    hv = hd.float().cpu()
    wg = _geglu_interleave(w1 * gam[None, :]).half()
    y = ops.gemm(hd, wg.to(DEV), bias=f32(_geglu_interleave(w1 @ bet + b1)), act=ACT_GEGLU, ln_stats=st,
                 ln_parts=st.shape[1], ln_eps=1e-5, ln_colsum=f32(wg.float().sum(1)))
    hh, gg = F.linear(F.layer_norm(hv, (C,), gam, bet, eps=1e-5), w1, b1).chunk(2, -1)
    ref = hh * F.gelu(gg)
    err = rel(y, ref)
    # the unfused fp16 path for scale: LayerNorm output rounded to fp16, then the GEGLU GEMM
    y0 = ops.gemm(ops.layernorm(hd, f32(gam), f32(bet), 1e-5), h(_geglu_interleave(w1)), bias=f32(_geglu_interleave(b1)),
                  act=ACT_GEGLU)
    err0 = rel(y0, ref)
    print(f"LN-folded GEGLU GEMM {M}x{2 * inner}x{C}: rel-L1 {err:.2e} (unfused fp16 path {err0:.2e})")
    assert y.shape == (M, inner)
    assert err < max(2 * err0, 2e-3)


@pytest.mark.parametrize("C,S,T,B", [(256, 300, 8, 2), (1024, 361, 4, 3), (256, 1369, 5, 1), (256, 256, 16, 1)])
def test_gemm_layernorm_fold_rowbias(C, S, T, B):
    """Motion-module q/k/v with its LayerNorm folded (motion_module.py:175, the EK 3 register epilogue):
    rstd (x W'^T - mean colsum) + W beta + the frame's PE row bias pe[t] W^T (t = (row / S) % T), the
    statistics as [M, P, 2] partials the producing GEMM writes; S = 300 / 361 put frame boundaries
    inside 256-row tiles (two PE rows per tile), B > 1 wraps t, S = 256 aligns them.  vs torch fp32
    LayerNorm -> + pe -> Linear, and vs the unfused route (LayerNorm kernel + row-bias GEMM)."""
    M, N = B * T * S, 3 * C
    g = torch.Generator().manual_seed(C + S + T)
    x = (torch.randn(M, C, generator=g) * 2 + torch.randn(M, 1, generator=g)).half().float()
    gam, bet = 1 + 0.2 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    w = torch.randn(N, C, generator=g) * C ** -0.5
    pe = torch.randn(T, C, generator=g) * 0.5
    t = (torch.arange(M) // S) % T
    ref = F.linear(F.layer_norm(x, (C,), gam, bet, eps=1e-5) + pe[t], w)
    rb = f32(pe @ w.t())
    P = C // 256
    xf = x.view(M, P, 256)
    parts = torch.zeros(M + 1, P, 2)
    parts[:M, :, 0], parts[:M, :, 1] = xf.sum(2), (xf * xf).sum(2)
    wg = (w * gam[None, :]).half()
    y = ops.gemm(h(x), wg.to(DEV), bias=f32(w @ bet), rowbias=rb, rdiv=S, rmod=T, ln_stats=f32(parts), ln_parts=P,
                 ln_eps=1e-5, ln_colsum=f32(wg.float().sum(1)))
    y0 = ops.gemm(ops.layernorm(h(x), f32(gam), f32(bet), 1e-5), h(w), rowbias=rb, rdiv=S, rmod=T)
    err, err0 = rel(y, ref), rel(y0, ref)
    print(f"LN-folded row-bias GEMM C={C} S={S} T={T} B={B}: rel-L1 {err:.2e} (unfused {err0:.2e})")
    assert err < max(2 * err0, 2e-3)


@pytest.mark.parametrize("M,N,K", [(5000, 1024, 512), (43808, 256, 256), (4001, 768, 256)])
def test_gemm_row_stats_no_residual(M, N, K):
    """stats_out on a GEMM without a residual (the motion modules' proj_in feeding the folded
    LayerNorm): the phased epilogue writes the per-row partials itself (no separate pass) and they
    equal torch sums of the stored fp16 values."""
    g = torch.Generator().manual_seed(M + N + K)
    x = (torch.randn(M, K, generator=g) * 0.5).half().float()
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = 0.1 * torch.randn(N, generator=g)
    P = (N + 255) // 256
    st = torch.full((M + 1, P, 2), float("nan"), device=DEV)
    y = ops.gemm(h(x), h(w), bias=f32(b), stats_out=st)
    yc = y.float().cpu()
    pad = torch.zeros(M, P * 256)
    pad[:, :N] = yc
    stc = st[:M].cpu()
    assert torch.allclose(stc[..., 0], pad.view(M, P, 256).sum(2), rtol=1e-4, atol=1e-3)
    assert torch.allclose(stc[..., 1], (pad * pad).view(M, P, 256).sum(2), rtol=1e-4, atol=1e-3)
    assert rel(y, F.linear(x, w, b)) < 2e-3


def test_gemm_layernorm_fold_rowbias_rejected_shapes():
    """LN fold + row bias exists on the phased route only: frames shorter than a tile (rdiv < 256)
    and N % 256 != 0 are rejected up front instead of running un-normalised."""
    from vda_amd import _lib
    lib = _lib.lib()
    x = torch.zeros(8192, 256, dtype=torch.float16, device=DEV)
    w = torch.zeros(768, 256, dtype=torch.float16, device=DEV)
    y = torch.empty(8192, 768, dtype=torch.float16, device=DEV)
    f = torch.zeros(8192 * 4, device=DEV)
    e = Epilogue(rdiv=100, rmod=8, bias=f.data_ptr(), rowbias=f.data_ptr(), ln_stats=f.data_ptr(),
                 ln_colsum=f.data_ptr(), ln_parts=1, ln_eps=1e-5)
    st = torch.cuda.current_stream().cuda_stream
    assert lib.vda_gemm(x.data_ptr(), 256, w.data_ptr(), y.data_ptr(), 768, 8192, 768, 256, e, st) == -22
    e.rdiv = 300
    assert lib.vda_gemm(x.data_ptr(), 256, w.data_ptr(), y.data_ptr(), 720, 8192, 720, 256, e, st) == -22


@pytest.mark.parametrize("Cin,H,W,BT,mode", [(256, 148, 148, 2, "rcu2"), (256, 148, 148, 2, "rcu1"), (256, 74, 74, 3, "plain"),
                                             (64, 9, 33, 2, "rcu2"), (128, 17, 40, 1, "rcu1"), (512, 8, 32, 2, "plain"),
                                             (64, 1, 1, 3, "rcu2"), (256, 37, 150, 1, "rcu2")])
def test_conv3x3_hconv_cout256(Cin, H, W, BT, mode):
    """3x3 / 256-output convs on the halo-tiled phased kernel (csrc/vda_hconv.hip; the refinenet RCU
    convs and layer1_rn, blocks.py:68-91, dpt.py:100-104): 8 x 32 tiles with partial edge tiles,
    patches clipped at every border, 1 .. 8 channel slabs, pre-ReLU + ReLU (RCU conv1), bias + skip
    + fusion adds (RCU conv2).  vs torch fp32, and vs the implicit-GEMM conv (fp32 accumulation in
    another K order: not bit-identical)."""
    x = rnd(BT, Cin, H, W, seed=290)
    w, b = rnd(256, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=291), rnd(256, scale=0.1, seed=292)
    r1, r2 = rnd(BT, 256, H, W, seed=293), rnd(BT, 256, H, W, seed=294)
    nh = lambda t: h(t.permute(0, 2, 3, 1).contiguous())
    kw = {}
    if mode == "plain":
        ref = F.conv2d(x, w, padding=1)
    elif mode == "rcu1":
        ref = F.relu(F.conv2d(F.relu(x), w, b, padding=1))
        kw = dict(bias=f32(b), pre_relu=True, act=ACT_RELU)
    else:
        ref = F.conv2d(x, w, b, padding=1) + r1 + r2
        kw = dict(bias=f32(b), res=nh(r1), res2=nh(r2))
    ref = ref.permute(0, 2, 3, 1)
    xh, wh = nh(x), nh(w)
    T = tune_lib()
    with T.route(hconv=1):
        y = T.conv2d(xh, wh, **kw)
        y_again = T.conv2d(xh, wh, **kw)
    assert rel(y, ref) < 2e-3
    assert torch.equal(y, y_again)
    with T.route(hconv=0, force_tile=-2):
        y2 = T.conv2d(xh, wh, **kw)
    assert rel(y, y2) < 1e-3


@pytest.mark.parametrize("BT,Cin,Hs,Ws,H,W", [(2, 256, 74, 74, 148, 148), (1, 256, 74, 132, 148, 264),
                                              (2, 64, 5, 17, 9, 33), (1, 128, 40, 12, 79, 23)])
def test_conv3x3_hconv_res2_upsample(BT, Cin, Hs, Ws, H, W):
    """refinenet1's RCU conv2 (blocks.py:146-150) with its skip input res2 = refinenet2's output read
    through the bilinear align_corners=True upsample (blocks.py:156-158) in the halo conv's epilogue:
    bit-identical to vda_upsample_bilinear + the same conv, vs torch fp32; the op materialises the
    upsample where the conv route has no such epilogue (same bits on that route)."""
    x = rnd(BT, Cin, H, W, seed=300)
    w, b = rnd(256, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=301), rnd(256, scale=0.1, seed=302)
    r1, r2 = rnd(BT, 256, H, W, seed=303), rnd(BT, 256, Hs, Ws, seed=304)
    nh = lambda t: h(t.permute(0, 2, 3, 1).contiguous())
    xh, wh, r1h, r2h = nh(x), nh(w), nh(r1), nh(r2)
    up = ops.upsample_bilinear(r2h, H, W)
    ref = F.conv2d(x, w, b, padding=1) + r1 + F.interpolate(r2, size=(H, W), mode="bilinear", align_corners=True)
    T = tune_lib()
    with T.route(hconv=1):
        assert T.lib.vda_conv2d_res2_upsample_ok(BT, H, W, Cin, 256, 3, 1, 1) == 1
        y = T.conv2d(xh, wh, bias=f32(b), res=r1h, res2=r2h)
        y_mat = T.conv2d(xh, wh, bias=f32(b), res=r1h, res2=up)
    assert torch.equal(y, y_mat)
    assert rel(y, ref.permute(0, 2, 3, 1)) < 2e-3
    if H * W >= 64 * 64:  # the product routes it the same way
        assert torch.equal(ops.conv2d(xh, wh, bias=f32(b), res=r1h, res2=r2h), y)
    with T.route(hconv=0, force_tile=-2):  # no upsampling epilogue on this route: rejected by the C ABI
        assert T.lib.vda_conv2d_res2_upsample_ok(BT, H, W, Cin, 256, 3, 1, 1) == 0
        with pytest.raises(RuntimeError, match="upsampled res2"):
            T.conv2d(xh, wh, bias=f32(b), res=r1h, res2=r2h)


def test_conv_res2_upsample_op_fallback():
    """The torch op materialises a lower-resolution res2 when the conv route has no upsampling
    epilogue (a 37^2 map: the implicit-GEMM / strip routes): same bits as the explicit upsample."""
    BT, Cin, H, W = 2, 256, 37, 37
    x, w = rnd(BT, Cin, H, W, seed=310), rnd(256, Cin, 3, 3, scale=(9 * Cin) ** -0.5, seed=311)
    r2 = rnd(BT, 256, 19, 19, seed=312)
    nh = lambda t: h(t.permute(0, 2, 3, 1).contiguous())
    xh, wh, r2h = nh(x), nh(w), nh(r2)
    y = ops.conv2d(xh, wh, res2=r2h)
    assert torch.equal(y, ops.conv2d(xh, wh, res2=ops.upsample_bilinear(r2h, H, W)))


@pytest.mark.parametrize("M,N,K", [(4001, 1024, 1024), (43840, 1024, 4096), (4001, 384, 1536), (5003, 768, 768),
                                   (300, 1024, 256), (4001, 1024, 512)])
def test_gemm_epilogue_row_stats(M, N, K):
    """proj / fc2 (x += ...) writing per-row partial (sum, sumsq) of their fp16 outputs over 256-column
    blocks (stats_out; the phased epilogue for the encoder shapes, the separate partial-sum pass for
    the others), and the next LN-folded GEMM consuming them (ln_parts = P): vs torch sums of the
    stored values and vs the same fold from vda_row_stats."""
    g = torch.Generator().manual_seed(M + N + K)
    x = (torch.randn(M, K, generator=g) * 0.5).half().float()
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = 0.1 * torch.randn(N, generator=g)
    r = (torch.randn(M, N, generator=g) * 2 + torch.randn(M, 1, generator=g)).half()
    P = (N + 255) // 256
    tok = r.to(DEV).contiguous()
    st = torch.full((M + 1, P, 2), float("nan"), device=DEV)  # spare row: 16-byte staging (vda.h ln_parts)
    ops.gemm(h(x), h(w), bias=f32(b), res=tok, out=tok, stats_out=st)
    y = tok.float().cpu()
    pad = torch.zeros(M, P * 256)
    pad[:, :N] = y
    ref_s = pad.view(M, P, 256).sum(2)
    ref_q = (pad * pad).view(M, P, 256).sum(2)
    stc = st[:M].cpu()
    assert torch.allclose(stc[..., 0], ref_s, rtol=1e-4, atol=1e-3)
    assert torch.allclose(stc[..., 1], ref_q, rtol=1e-4, atol=1e-3)
    # consumer: LN fold from the partials vs from vda_row_stats
    gam, bet = 1 + 0.2 * torch.randn(N, generator=g), 0.1 * torch.randn(N, generator=g)
    w2 = torch.randn(512, N, generator=g) * N ** -0.5
    wg = (w2 * gam[None, :]).half()
    c1, bb = f32(wg.float().sum(1)), f32(w2 @ bet)
    ya = ops.gemm(tok, wg.to(DEV), bias=bb, ln_stats=st, ln_parts=P, ln_eps=1e-6, ln_colsum=c1)
    yb = ops.gemm(tok, wg.to(DEV), bias=bb, ln_stats=ops.row_stats(tok, 1e-6), ln_colsum=c1)
    ref = F.linear(F.layer_norm(y, (N,), gam, bet, eps=1e-6), w2)
    assert rel(ya, ref) < 2e-3 and rel(ya, yb) < 1e-3
    # the register residual epilogue of the tuning build (vda_debug_gemm_epi(1), EK 2 for the phased
    # shapes): bit-identical outputs; the statistics sum in another order
    tok2, st2 = r.to(DEV).contiguous(), torch.full((M + 1, P, 2), float("nan"), device=DEV)
    xh, wh, bf = h(x), h(w), f32(b)
    e = Epilogue(rdiv=1, rmod=1, bias=bf.data_ptr(), res=tok2.data_ptr(), ldres=N, stats_out=st2.data_ptr())
    with tune_lib().route(gemm_epi=1) as T:
        T.gemm(xh, wh, tok2, e, M, N, K)
    torch.cuda.synchronize()
    assert torch.equal(tok2, tok)
    assert torch.allclose(st2[:M], st[:M], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M,P,rowbias,nobias", [(4097, 3, False, False), (4097, 1, False, False), (4097, 0, False, False),
                                                (4097, 3, False, True), (4097, 0, False, True), (4097, 1, True, False),
                                                (5003, 3, True, False)])
def test_gemm_layernorm_fold_odd_stats_exact_size(M, P, rowbias, nobias):
    """VERDICT r3 item 6 / ADVICE r2-r3: the phased LN-folded GEMM stages the statistics in 16-byte
    pieces; with M * P odd (or M odd for [M, 2] statistics) the last piece holds one valid entry.  The
    statistics buffer here is EXACTLY [M, P, 2] (no spare row), carved from the END of a larger
    allocation whose tail is NaN: a read past it would poison the last row.  Through the C ABI, vs
    torch fp32 LayerNorm -> Linear (+ the per-frame PE row bias on the EK 3 route); without a bias the
    staged epilogue's reader runs instead of the register epilogue's."""
    from vda_amd import _lib
    lib = _lib.lib()
    K = 256 * max(P, 1)
    N = 768 if rowbias else 512
    S, T = 1024, 4
    g = torch.Generator().manual_seed(M + P)
    x = (torch.randn(M, K, generator=g) * 2 + torch.randn(M, 1, generator=g)).half().float()
    gam, bet = 1 + 0.2 * torch.randn(K, generator=g), 0.1 * torch.randn(K, generator=g)
    w = torch.randn(N, K, generator=g) * K ** -0.5
    pe = torch.randn(T, K, generator=g) * 0.5
    ln = F.layer_norm(x, (K,), gam, bet, eps=1e-5)
    if rowbias:
        ln = ln + pe[(torch.arange(M) // S) % T]
    ref = F.linear(ln, w) - (w @ bet if nobias else 0)
    wg = (w * gam[None, :]).half()
    if P > 0:
        xf = x.view(M, P, 256)
        stats = torch.stack([xf.sum(2), (xf * xf).sum(2)], -1)  # [M, P, 2]
    else:
        mean, var = x.mean(1), x.var(1, unbiased=False)
        stats = torch.stack([mean, (var + 1e-5).rsqrt()], -1)  # [M, 2]
    n = stats.numel()
    big = torch.full((n + 64,), float("nan"), device=DEV)
    st = big[:n]  # exactly [M, P, 2]; NaN right behind it
    st.copy_(stats.reshape(-1).to(DEV))
    xd, wd = h(x), wg.to(DEV)
    y = torch.empty(M, N, dtype=torch.float16, device=DEV)
    bias, cs = f32(w @ bet), f32(wg.float().sum(1))
    rb = f32(pe @ w.t())
    e = Epilogue(bias=0 if nobias else bias.data_ptr(), ln_stats=st.data_ptr(), ln_colsum=cs.data_ptr(), ln_parts=P, ln_eps=1e-5,
                 rdiv=S if rowbias else 1, rmod=T if rowbias else 1, rowbias=rb.data_ptr() if rowbias else 0)
    stream = torch.cuda.current_stream().cuda_stream
    assert lib.vda_gemm(xd.data_ptr(), K, wd.data_ptr(), y.data_ptr(), N, M, N, K, e, stream) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    err = rel(y, ref)
    err_last = rel(y[-1:], ref[-1:])
    print(f"LN fold odd stats M={M} P={P} rowbias={rowbias}: rel-L1 {err:.2e}, last row {err_last:.2e}")
    assert err < 3e-3 and err_last < 5e-3


@pytest.mark.parametrize("kind", ["offset", "outlier_channels"])
@pytest.mark.parametrize("N2,act", [(3072, 0), (4096, ACT_GELU)])
def test_gemm_layernorm_fold_stress_statistics(kind, N2, act):
    """the LN fold's numerics on activation statistics like a trained DINOv2-L's
    (block.py:84,87; the reference's autocast LayerNorm runs in fp32).  The residual stream goes through
    the producer GEMM (proj / fc2: x += ..., stats_out partials over 256-column blocks) and then the
    LN-folded consumer (qkv / fc1) reads those partials; compared with torch fp32 LayerNorm -> Linear on
    the same stored fp16 residual values.  Rows carry either a common offset of 50-100 sigma (the
    E[x^2] - mean^2 cancellation) or a few channels at ~500 (DINOv2's massive activations)."""
    M, C, Kp = 8192, 1024, 1024
    g = torch.Generator().manual_seed(N2 + (1 if kind == "offset" else 2))
    if kind == "offset":
        sig = 0.5 + torch.rand(M, 1, generator=g)
        mu = (50 + 50 * torch.rand(M, 1, generator=g)) * sig * torch.sign(torch.randn(M, 1, generator=g))
        r = torch.randn(M, C, generator=g) * sig + mu
    else:
        r = torch.randn(M, C, generator=g)
        hot = torch.randint(0, C, (4,), generator=g)
        r[:, hot] = 400 + 200 * torch.rand(M, 4, generator=g)
    r = r.half()
    x = (torch.randn(M, Kp, generator=g) * 0.5).half()
    w = torch.randn(C, Kp, generator=g) * Kp ** -0.5 * 0.1
    b = 0.01 * torch.randn(C, generator=g)
    P = C // 256
    tok = r.to(DEV).contiguous()
    st = torch.empty(M, P, 2, device=DEV)
    ops.gemm(h(x.float()), h(w), bias=f32(b), res=tok, out=tok, stats_out=st)
    y = tok.float().cpu()  # the stored residual stream the consumer normalises
    gam, bet = 1 + 0.2 * torch.randn(C, generator=g), 0.1 * torch.randn(C, generator=g)
    w2 = torch.randn(N2, C, generator=g) * C ** -0.5
    b2 = 0.1 * torch.randn(N2, generator=g)
    wg = (w2 * gam[None, :]).half()
    c1, bb = f32(wg.float().sum(1)), f32(w2 @ bet + b2)
    ya = ops.gemm(tok, wg.to(DEV), bias=bb, act=act, ln_stats=st, ln_parts=P, ln_eps=1e-6, ln_colsum=c1)
    ref = F.linear(F.layer_norm(y, (C,), gam, bet, eps=1e-6), w2, b2)
    if act == ACT_GELU:
        ref = F.gelu(ref)
    # the per-row (mean, rstd) the partials imply, vs fp64 statistics of the stored values
    s = st.double().cpu().sum(1)
    mean = s[:, 0] / C
    rstd = ((s[:, 1] / C - mean * mean).clamp_min(0) + 1e-6).rsqrt()
    yd = y.double()
    rstd_ref = (yd.var(1, unbiased=False) + 1e-6).rsqrt()
    rstd_err = ((rstd - rstd_ref).abs() / rstd_ref).max().item()
    err = rel(ya, ref)
    print(f"LN fold stress {kind} N={N2} act={act}: rel-L1 {err:.2e}, max rstd rel err {rstd_err:.2e}")
    assert err < 1e-3


@pytest.mark.parametrize("M,N,K,kind", [(43840, 3072, 1024, "lnf"), (43840, 1024, 1024, "res"), (43840, 4096, 1024, "lnf_gelu"),
                                        (43840, 1024, 4096, "res"), (8192, 1024, 512, "plain"), (20000, 768, 256, "res")])
def test_gemm_dynamic_tile_schedule(M, N, K, kind):
    """the persistent GEMM taking its tiles beyond the first round by per-XCD atomic
    ticket (vda_epilogue.sched) computes every tile exactly as the fixed-stride schedule does
    (torch.equal, statistics too), leaves the counters zero for the next launch, and two streams with
    their own counter sets running the same GEMMs concurrently agree with it."""
    g = torch.Generator().manual_seed(M + N + K)
    x = (torch.randn(M, K, generator=g) * 0.5).half().to(DEV)
    w = (torch.randn(N, K, generator=g) * K ** -0.5).half().to(DEV)
    b = f32(0.1 * torch.randn(N, generator=g))
    kw = dict(bias=b)
    if kind.startswith("lnf"):
        xf = x.float().view(M, K // 256, 256)
        kw.update(ln_stats=torch.stack([xf.sum(2), (xf * xf).sum(2)], 2).contiguous(), ln_parts=K // 256, ln_eps=1e-6,
                  ln_colsum=w.float().sum(1).contiguous(), act=ACT_GELU if kind.endswith("gelu") else 0)
    res = (torch.randn(M, N, generator=g)).half().to(DEV) if kind == "res" else None
    P = (N + 255) // 256

    def run(sched, stream=None):
        out = res.clone() if res is not None else torch.empty(M, N, dtype=torch.float16, device=DEV)
        so = torch.full((M, P, 2), float("nan"), device=DEV) if res is not None else None
        ops.gemm(x, w, res=out if res is not None else None, out=out, stats_out=so, sched=sched, **kw)
        return out, so

    y0, s0 = run(None)
    sch = torch.zeros(16, dtype=torch.int32, device=DEV)
    for _ in range(3):
        y1, s1 = run(sch)
        torch.cuda.synchronize()
        assert torch.equal(y1, y0)
        if s0 is not None:
            assert torch.equal(s1, s0)
        assert int(sch.abs().sum()) == 0, "the last block must leave the counters zero"
    # two streams, own counters, interleaved launches
    st = [torch.cuda.Stream(), torch.cuda.Stream()]
    cs = [torch.zeros(16, dtype=torch.int32, device=DEV) for _ in st]
    torch.cuda.synchronize()
    outs = []
    for r in range(4):
        with torch.cuda.stream(st[r % 2]):
            outs.append(run(cs[r % 2])[0])
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, y0)
    assert all(int(c.abs().sum()) == 0 for c in cs)
    # the model's per-stream counter sets
    assert ops.sched_counters().dtype == torch.int32 and ops.sched_counters() is ops.sched_counters()


@pytest.mark.parametrize("BT,H,W", [(2, 70, 518), (3, 28, 924), (1, 14, 1036), (1, 518, 518), (32, 518, 518)])
def test_patch_im2col_exact(BT, H, W):
    """patch_embed.py:69-82 input: the [BT, 1 + np, Kp] fp16 patch matrix is the exact fp16 of the
    image's 14 x 14 patches (channel-major: k = c * 196 + ky * 14 + kx), zero cls rows and zero K padding."""
    img = rnd(BT, 3, H, W, seed=45)
    a = ops.patch_im2col(img.to(DEV).contiguous(), 640).cpu()
    np_ = (H // 14) * (W // 14)
    ref = torch.zeros(BT, np_ + 1, 640, dtype=torch.float16)
    ref[:, 1:, :588] = F.unfold(img, 14, stride=14).transpose(1, 2).half()
    assert torch.equal(a.view(BT, np_ + 1, 640), ref)

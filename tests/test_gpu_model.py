"""Whole clip forward on the MI355X path vs the reference's golden outputs and the CPU oracle.

Tolerance: relative L1 (sum|d - ref| / sum|ref|) <= 1e-3 for the fp16 path against the fp32
reference -- the north_star bar.  Measured on MI355X: 3.0e-4 .. 5.6e-4 on every golden case.
"""
import os

import pytest
import torch

import vda_amd
from helpers import GOLDEN_CASES, load_golden, recipe_state_dict, rel_l1, vda_oracle

pytestmark = pytest.mark.gpu
TOL_FP16 = 1e-3  # north_star bar (rel-L1 vs the fp32 reference)

_MODELS = {}


def model(enc):
    if enc not in _MODELS:
        _MODELS[enc] = vda_amd.build_model(enc, recipe_state_dict(enc), device="cuda")
    return _MODELS[enc]


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_forward_matches_reference_golden(name):
    x, depth, _, meta = load_golden(name)
    m = model(meta["encoder"])
    d = m(x.cuda(), skip_tmp_block=meta["skip_tmp_block"]).float().cpu()
    assert d.shape == depth.shape
    assert torch.isfinite(d).all()
    err = rel_l1(d, depth)
    print(f"{name}: rel-L1 vs reference = {err:.3e}")
    assert err <= TOL_FP16, f"{name}: rel-L1 {err:.3e}"


@pytest.mark.parametrize("enc,B,T,H,W", [("vits", 1, 32, 266, 266), ("vitl", 1, 6, 140, 196)])
def test_forward_matches_oracle(enc, B, T, H, W):
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, T, 3, H, W, generator=g)
    d = model(enc)(x.cuda()).float().cpu()
    ref = vda_oracle.forward(recipe_state_dict(enc), enc, x)
    err = rel_l1(d, ref)
    print(f"{enc} {B}x{T}x{H}x{W}: rel-L1 vs oracle = {err:.3e}")
    assert err <= TOL_FP16


@pytest.mark.parametrize("enc,T,H,W", [("vits", 32, 266, 266), ("vitl", 6, 140, 196)])
def test_forward_ff_norm_fold_matches_oracle(enc, T, H, W):
    """The model switch fold_ff_norm (off by default: slower in the forward A/B) folds each motion module's
    ff_norm into its GEGLU GEMM with statistics from the last to_out; the forward with it still meets the
    bar against the oracle, and differs from the unfolded forward only by fp16 rounding."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, T, 3, H, W, generator=g)
    m = model(enc)
    d0 = m(x.cuda()).float().cpu()
    m.fold_ff_norm = True
    try:
        d1 = m(x.cuda()).float().cpu()
    finally:
        m.fold_ff_norm = False
    ref = vda_oracle.forward(recipe_state_dict(enc), enc, x)
    err = rel_l1(d1, ref)
    print(f"{enc} 1x{T}x{H}x{W} with fold_ff_norm: rel-L1 vs oracle = {err:.3e} (unfolded {rel_l1(d0, ref):.3e})")
    assert err <= TOL_FP16
    assert rel_l1(d1, d0) < 1e-3


def test_forward_tap_norm_fold():
    """fold_tap_norm (on by default): each encoder tap's final LayerNorm folded into its DPT projects GEMM, the
    cls rows dropped in that GEMM's store (vda.h drop_period).  ViT-L at 12 x 266^2 (362 tokens per frame,
    4,344 rows: the phased route serves it); the forward with the fold differs from the LayerNorm + GEMM
    forward only by fp16 rounding (bar 1e-3 rel-L1; the full-size parity tests cover it against the oracle)."""
    g = torch.Generator().manual_seed(12)
    x = torch.randn(1, 12, 3, 266, 266, generator=g).cuda()
    m = model("vitl")
    P = m._pack(x.device)
    assert m._tap_fold(P, 12, 362) and not m._tap_fold(P, 4, 362)
    d1 = m(x).float().cpu()
    m.fold_tap_norm = False
    try:
        d0 = m(x).float().cpu()
    finally:
        m.fold_tap_norm = True
    err = rel_l1(d1, d0)
    print(f"vitl 1x12x266x266: fold_tap_norm vs LayerNorm + GEMM rel-L1 {err:.3e}")
    assert err < 1e-3


def test_forward_deterministic_and_batch_independent():
    """Clip-parallel sharding relies on per-clip independence: B=2 == two B=1 runs."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 4, 3, 70, 98, generator=g).cuda()
    m = model("vits")
    d2 = m(x)
    d0, d1 = m(x[:1]), m(x[1:])
    assert torch.equal(d2, m(x))
    assert rel_l1(d2[:1].cpu(), d0.cpu()) < 1e-6 and rel_l1(d2[1:].cpu(), d1.cpu()) < 1e-6


@pytest.mark.parametrize("fp32", [False, True])
def test_rope_variant_matches_reference_golden(fp32):
    """pe='rope': q/k rotated inside the temporal attention kernels (fp16 and fp32 paths)."""
    import json
    from vda_amd.weights import synthetic_state_dict
    from helpers import GOLDEN
    with open(os.path.join(GOLDEN, "state_dict_keys_vits_rope.json")) as f:
        keys = [(k, tuple(s)) for k, s in json.load(f)]
    m = vda_amd.build_model("vits", synthetic_state_dict(keys), device="cuda", pe="rope")
    x, depth, _, _ = load_golden("vits_t8_126_rope")
    d = m(x.cuda(), fp32=fp32).float().cpu()
    err = rel_l1(d, depth)
    print(f"rope fp32={fp32}: rel-L1 vs reference = {err:.3e}")
    assert err <= (1e-5 if fp32 else TOL_FP16)


@pytest.mark.parametrize("fp32", [False, True])
def test_bn_clstoken_variant_matches_reference_golden(fp32):
    """use_bn=True (BatchNorm folded into the RCU convs) + use_clstoken=True (readout as a per-frame
    fp32 row bias + GELU epilogue of the patch GEMM) vs the reference's output."""
    import json
    from vda_amd.weights import synthetic_state_dict
    from helpers import GOLDEN
    with open(os.path.join(GOLDEN, "state_dict_keys_vits_bn_cls.json")) as f:
        keys = [(k, tuple(s)) for k, s in json.load(f)]
    m = vda_amd.build_model("vits", synthetic_state_dict(keys), device="cuda", use_bn=True, use_clstoken=True)
    x, depth, _, _ = load_golden("vits_t4_70x98_bn_cls")
    d = m(x.cuda(), fp32=fp32).float().cpu()
    err = rel_l1(d, depth)
    print(f"bn+clstoken fp32={fp32}: rel-L1 vs reference = {err:.3e}")
    assert err <= (1e-5 if fp32 else TOL_FP16)


def test_forward_input_checks_mirror_reference_asserts():
    """The reference's shape asserts at the boundary: H, W multiples of 14 (patch_embed.py:73-74),
    T <= the temporal PE table (motion_module.py:198-206), 3 input channels (patch_embed.py:69)."""
    m = model("vits")
    with pytest.raises(AssertionError, match="multiple of the patch size"):
        m(torch.zeros(1, 2, 3, 70, 99, device="cuda"))
    with pytest.raises(ValueError, match="exceeds the temporal PE table"):
        m(torch.zeros(1, 33, 3, 28, 28, device="cuda"))
    with pytest.raises(ValueError, match="3 input channels"):
        m(torch.zeros(1, 2, 4, 28, 28, device="cuda"))
    # T = 1 (a single frame through the temporal blocks) is valid
    d = m(torch.randn(1, 1, 3, 28, 42, device="cuda"))
    assert d.shape == (1, 1, 28, 42) and torch.isfinite(d).all()


@pytest.mark.parametrize("big", [200.0, 600.0])
def test_forward_massive_residual_channels(big):
    """The residual stream is fp16 here, fp32 in the reference's autocast forward (x + pos_embed promotes
    to fp32 and every block's `x + ls(...)` stays fp32, block.py:104-106).  Trained DINOv2 weights carry a
    few "massive" residual channels (hundreds) beside O(1) ones, where fp16's absolute step grows (0.125
    at 200, 0.5 at 600).  Three channels are pushed to ~big by the patch-embed bias and every block's fc2
    bias adds to them; the fp16 path stays within the fp16 bar of the fp32 oracle."""
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    sd = {k: v.clone() for k, v in recipe_state_dict("vits").items()}
    ch = [7, 101, 250]
    sd["pretrained.patch_embed.proj.bias"][ch] += big
    depth = sum(1 for k in sd if k.startswith("pretrained.blocks.") and k.endswith(".mlp.fc2.bias"))
    for i in range(depth):
        sd[f"pretrained.blocks.{i}.mlp.fc2.bias"][ch] += big / 25
    m = vda_amd.build_model("vits", sd, device="cuda")
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, 8, 3, 140, 196, generator=g)
    d = m(x.cuda()).float().cpu()
    ref = vda_oracle.forward(sd, "vits", x)
    err = rel_l1(d, ref)
    print(f"massive residual channels at ~{big:.0f}: rel-L1 vs oracle = {err:.3e}")
    assert torch.isfinite(d).all()
    assert err <= TOL_FP16

"""The CPU oracle against golden vectors produced by the reference itself (tests/golden/)."""
import json
import os

import pytest
import torch

from helpers import GOLDEN, GOLDEN_CASES, load_golden, recipe_state_dict, rel_l1, vda_oracle


@pytest.mark.parametrize("enc", ["vits", "vitl"])
def test_state_dict_schema_matches_reference(enc):
    """Module tree key names / shapes == the reference's (strict checkpoint loading, run.py:80)."""
    import vda_amd
    with open(os.path.join(GOLDEN, f"state_dict_keys_{enc}.json")) as f:
        ref = [(k, tuple(s)) for k, s in json.load(f)]
    m = vda_amd.VideoDepthAnything.from_config(enc, device="meta")
    mine = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    assert sorted(mine) == sorted(ref)


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_reference_golden(name):
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    x, depth, tap_stats, meta = load_golden(name)
    sd = recipe_state_dict(meta["encoder"])
    d = vda_oracle.forward(sd, meta["encoder"], x, skip_tmp_block=meta["skip_tmp_block"])
    assert d.shape == depth.shape
    err = rel_l1(d, depth)
    assert err <= 1e-5, f"{name}: oracle vs reference rel-L1 {err:.3e}"


def test_oracle_taps_match_reference_stats():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    x, _, tap_stats, meta = load_golden("vits_t8_126")
    sd = {k: v.float() for k, v in recipe_state_dict("vits").items()}
    feats = vda_oracle.encoder_taps(sd, "vits", x.flatten(0, 1))
    for f, (mu, sd_, am) in zip(feats, tap_stats):
        assert abs(float(f.mean()) - mu) <= 1e-4 * max(1.0, abs(mu))
        assert abs(float(f.std()) - sd_) <= 1e-4 * sd_
        assert abs(float(f.abs().mean()) - am) <= 1e-4 * am


def test_rope_variant_schema_and_oracle():
    """pe='rope' (motion_module.py:238-242, 290-293): the module tree has no pos_encoder buffers, like
    the reference's; the oracle's rotary restatement matches the reference's output."""
    import vda_amd
    from vda_amd.weights import synthetic_state_dict
    with open(os.path.join(GOLDEN, "state_dict_keys_vits_rope.json")) as f:
        ref = [(k, tuple(s)) for k, s in json.load(f)]
    m = vda_amd.VideoDepthAnything.from_config("vits", device="meta", pe="rope")
    mine = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    assert sorted(mine) == sorted(ref)
    assert not any(k.endswith("pos_encoder.pe") for k, _ in mine)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    x, depth, _, meta = load_golden("vits_t8_126_rope")
    assert meta["pe"] == "rope"
    sd = synthetic_state_dict(ref)
    d = vda_oracle.forward(sd, "vits", x)
    assert rel_l1(d, depth) <= 1e-5


def test_bn_clstoken_variant_schema_and_oracle():
    """use_bn=True, use_clstoken=True: the same key schema as the reference's tree (BatchNorm buffers,
    readout projections) and the oracle reproduces the reference's output."""
    import vda_amd
    from vda_amd.weights import synthetic_state_dict
    with open(os.path.join(GOLDEN, "state_dict_keys_vits_bn_cls.json")) as f:
        ref = [(k, tuple(s)) for k, s in json.load(f)]
    with torch.device("meta"):
        m = vda_amd.VideoDepthAnything(**vda_amd.MODEL_CONFIGS["vits"], use_bn=True, use_clstoken=True)
    mine = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    assert sorted(mine) == sorted(ref)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    x, depth, _, meta = load_golden("vits_t4_70x98_bn_cls")
    d = vda_oracle.forward(synthetic_state_dict(ref), "vits", x)
    assert rel_l1(d, depth) <= 1e-5

"""Streaming mode (video_depth.py:91-327 ``infere_single_image``): schedule, feature store, parity.

CPU tests drive ``vda_amd.stream.infere_single_image`` with the oracle's fp32 engine and compare
with the reference's own outputs (tests/golden/stream_vits_50f.npz, made by
tests/golden/make_stream_golden.py); the GPU test runs the same video through libvda.
"""
import json
import os

import numpy as np
import pytest
import torch

from helpers import GOLDEN, recipe_state_dict, vda_oracle
from vda_amd import stream as S


def load_stream_golden():
    z = np.load(os.path.join(GOLDEN, "stream_vits_50f.npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return z["frames"], {k[6:]: z[k] for k in z.files if k.startswith("depth_")}, meta


def rel(a, b):
    return float(np.abs(a.astype(np.float64) - b).sum() / np.abs(b).sum())


def test_schedule_literal_values():
    sch = S.StreamSchedule.build(32, [2, 12])
    assert sch.n_slots == 43
    assert len(sch.contexts) == 13 and all(len(c) == 31 for c in sch.contexts)
    assert sch.contexts[0] == list(range(31))
    assert sch.align[0] == [0, 30, 20]
    # the default keyframes put slot 32 (never written before frame 32) into the first context
    d = S.StreamSchedule.build(32, [0, 12])
    assert d.contexts[0][1] == 32 and d.align[0][1] == 1
    with pytest.raises(AssertionError):
        S.StreamSchedule.build(32, [0, 0])  # duplicate fixed slots -> the reference assert (:170)

def test_feature_store_shift_is_a_remap():
    like = [torch.zeros(1, 2)]
    st = S.FeatureStore(5, like)
    for i in range(5):
        st.put(i, [torch.full((1, 2), float(i))])
    ref = torch.arange(5.0)[:, None].expand(5, 2).clone()
    st.shift_in([torch.full((1, 2), 9.0)])
    ref[:-1] = ref[[0, 2, 3, 4]].clone()
    ref[-1] = 9.0
    assert torch.equal(st.gather(range(5))[0], ref)
    with pytest.raises(IndexError):
        st.gather([5])


@pytest.mark.parametrize("case", ["noalign", "kf2_12", "kf4_12_skip", "kf2_12_len16"])
def test_stream_oracle_matches_reference(case):
    frames, depths, meta = load_stream_golden()
    eng = vda_oracle.StreamEngine(recipe_state_dict("vits"), "vits")
    d, fps = S.infere_single_image(eng, frames, 24, input_size=meta["input_size"], device="cpu",
                                   io=vda_oracle.TorchIO, **meta["cases"][case])
    assert fps == 24
    assert d.shape == depths[case].shape
    assert rel(d, depths[case]) <= 1e-5


def test_stream_default_raises_like_reference():
    frames, _, meta = load_stream_golden()
    assert meta["default_raises"].startswith("IndexError")
    eng = vda_oracle.StreamEngine(recipe_state_dict("vits"), "vits")
    with pytest.raises(IndexError):
        S.infere_single_image(eng, frames[:33], 24, input_size=56, device="cpu", io=vda_oracle.TorchIO)
    with pytest.raises(NotImplementedError):
        S.infere_single_image(eng, frames[:2], 24, input_size=56, device="cpu", warmup=False,
                              io=vda_oracle.TorchIO)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["noalign", "kf2_12", "kf4_12_skip", "kf2_12_len16"])
def test_stream_gpu_matches_reference(case):
    """libvda streaming vs the reference's infere_single_image output (north_star bar 1e-3)."""
    frames, depths, meta = load_stream_golden()
    m = vda_amd_model()
    d, _ = m.infere_single_image(frames, 24, input_size=meta["input_size"], device="cuda", **meta["cases"][case])
    err = rel(d, depths[case])
    print(f"stream {case}: rel-L1 {err:.3e}")
    assert d.shape == depths[case].shape and np.isfinite(d).all()
    assert err <= 1e-3


@pytest.mark.gpu
def test_forward_single_image_gpu_vs_oracle():
    """One streaming step at a non-square size with a shuffled context and alignment rows."""
    m = vda_amd_model()
    eng = vda_oracle.StreamEngine(recipe_state_dict("vits"), "vits")
    g = torch.Generator().manual_seed(5)
    T = 8
    xs = torch.randn(T, 3, 42, 70, generator=g)
    ctx_gpu = [m.get_motion_features(xs[i:i + 1].cuda()) for i in range(T - 1)]
    ctx_gpu = tuple(torch.cat([c[k] for c in ctx_gpu], 0) for k in range(4))
    ctx_cpu = [eng.motion_features(xs[i:i + 1]) for i in range(T - 1)]
    ctx_cpu = tuple(torch.cat([c[k] for c in ctx_cpu], 0) for k in range(4))
    for k in range(4):  # NHWC fp16 (libvda) vs NCHW fp32 (oracle)
        assert rel(ctx_gpu[k].float().permute(0, 3, 1, 2).cpu().numpy(), ctx_cpu[k].numpy()) <= 3e-3
    pred = [0, 5, 2]
    d, new = m.forward_single_image(xs[T - 1:].cuda()[None], ctx_gpu, list(pred), T)
    dr, _ = eng.predict(xs[T - 1:], ctx_cpu, list(pred), T)
    assert d.shape == (1, 4, 42, 70)
    assert rel(d[0].cpu().numpy(), dr.numpy()) <= 1e-3
    with pytest.raises(IndexError):
        m.forward_single_image(xs[T - 1:].cuda()[None], ctx_gpu, [T - 1], T)


_M = {}


def vda_amd_model():
    if "vits" not in _M:
        import vda_amd
        _M["vits"] = vda_amd.build_model("vits", state_dict=recipe_state_dict("vits"), device="cuda")
    return _M["vits"]

"""Weights for the Video-Depth-Anything module tree: reference checkpoints or a synthetic recipe.

No checkpoint can be downloaded here (``get_weights.sh`` needs the network), so tests, goldens
and the benchmark use a deterministic synthetic recipe keyed by the reference ``state_dict`` key
names.  The same function fills the reference model (in
``tests/golden/make_golden.py``, container only) and this package's model, so both sides see
bit-identical fp32 weights without sharing code or files.

Recipe, per key (generator seeded with crc32(key)):
  * ``*.pos_encoder.pe``           sinusoidal table (motion_module.py:189-203; a buffer, not random)
  * ``*.mask_token``               zeros (unused by the forward)
  * ``*norm*.weight``              1 + 0.1 N(0,1)      (LayerNorm / GroupNorm affine)
  * ``*.gamma``                    U(0.2, 0.6)         (LayerScale)
  * 1-D ``*.bias`` / cls / pos     0.02 N(0,1)
  * conv / linear weights          N(0,1) / sqrt(fan_in)
  * ``head.scratch.output_conv2.2`` weight |N(0,1)|/sqrt(32), bias 0.05: keeps the depth strictly
    positive so the final ReLUs (dpt.py:122, video_depth.py:64) do not zero most of the map.
  * BatchNorm (use_bn=True): running_mean 0.1 N(0,1), running_var U(0.5, 1.5), num_batches_tracked 0.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import torch


def _pe_table(C: int, max_len: int) -> torch.Tensor:
    pos = torch.arange(max_len).unsqueeze(1)
    div = torch.exp(torch.arange(0, C, 2) * (-math.log(10000.0) / C))
    pe = torch.zeros(1, max_len, C)
    pe[0, :, 0::2] = torch.sin(pos * div)
    pe[0, :, 1::2] = torch.cos(pos * div)
    return pe


def synthetic_tensor(key: str, shape: Tuple[int, ...]) -> torch.Tensor:
    g = torch.Generator().manual_seed(zlib.crc32(key.encode()) & 0x7FFFFFFF)
    shape = tuple(int(s) for s in shape)
    if key.endswith("pos_encoder.pe"):
        return _pe_table(shape[-1], shape[-2])
    if key.endswith("mask_token"):
        return torch.zeros(shape)
    if key == "head.scratch.output_conv2.2.weight":
        return torch.randn(shape, generator=g).abs() / math.sqrt(32.0)
    if key == "head.scratch.output_conv2.2.bias":
        return torch.full(shape, 0.05)
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":  # BatchNorm bookkeeping (use_bn=True trees)
        return torch.zeros(shape, dtype=torch.long)
    if leaf == "running_var":
        return 0.5 + torch.rand(shape, generator=g)
    if leaf == "running_mean":
        return 0.1 * torch.randn(shape, generator=g)
    if leaf == "gamma":
        return 0.2 + 0.4 * torch.rand(shape, generator=g)
    if leaf == "weight" and len(shape) == 1:  # norm affine
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    if leaf in ("bias", "cls_token", "pos_embed") or len(shape) == 1:
        return 0.02 * torch.randn(shape, generator=g)
    # conv / linear weight
    if key in ("head.resize_layers.0.weight", "head.resize_layers.1.weight"):
        fan_in = shape[0]  # ConvTranspose2d weight [in, out, k, k]: each output sums `in` taps
    else:
        fan_in = int(math.prod(shape[1:]))
    return torch.randn(shape, generator=g) / math.sqrt(fan_in)


def synthetic_state_dict(key_shapes: Iterable[Tuple[str, Tuple[int, ...]]]) -> Dict[str, torch.Tensor]:
    return {k: synthetic_tensor(k, s) for k, s in key_shapes}


def load_checkpoint(path: str) -> Dict[str, torch.Tensor]:
    """Load a reference checkpoint (video_depth_anything_{vits,vitl}.pth) without unpickling code."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "model" in sd and isinstance(sd["model"], dict):
        sd = sd["model"]
    return sd

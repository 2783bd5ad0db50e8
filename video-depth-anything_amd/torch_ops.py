"""``torch.ops.vda.*``: the libvda kernels as native PyTorch operators.

The operators are registered in C++ (``csrc/vda_torch.cpp``: ``TORCH_LIBRARY(vda, m)`` with CUDA =
HIP and Meta kernels, no CPU kernel) and live in ``libvda_torch.so``; importing this module loads
it.  ``vda_amd.ops`` and the model forward call the same operators, e.g.::

    import vda_amd.torch_ops  # loads the library once
    y = torch.ops.vda.gemm(x, w, bias, act=1)                       # fc1 + GELU (mlp.py:35-41)
    o = torch.ops.vda.temporal_attention(qkv, 1, 32, 1369, 8, 128, rope_theta=1e4)
"""
from __future__ import annotations

from ._lib import torch_ops

vda = torch_ops()

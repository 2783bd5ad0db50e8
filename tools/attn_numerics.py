"""Spatial-attention numerics across libvda builds (tuning tool): rel-L1 vs fp32 SDPA per shape / score range.
usage: python tools/attn_numerics.py LIB_A.so [LIB_B.so ...]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from vda_amd import _lib
libs = []
for p in sys.argv[1:]:
    l = ctypes.CDLL(os.path.abspath(p)); _lib._declare(l); libs.append((p, l))
st = torch.cuda.current_stream().cuda_stream
H, D = 6, 64
for N in (36, 71, 130, 1370):
    for sc in (1.0, 3.0, 6.0):
        B = 4 if N < 1000 else 2
        g = torch.Generator(device="cuda").manual_seed(N)
        qkv = (torch.randn(B * N, 3 * H * D, device="cuda", generator=g) * sc).half()
        q, k, v = qkv.view(B, N, 3, H, D).float().permute(2, 0, 3, 1, 4)
        ref = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B * N, H * D)
        line = f"N={N:5d} scale={sc}:"
        for p, l in libs:
            y = torch.empty(B * N, H * D, device="cuda", dtype=torch.float16)
            assert l.vda_spatial_attention(qkv.data_ptr(), y.data_ptr(), B, N, H, D, D ** -0.5, st) == 0
            torch.cuda.synchronize()
            err = float((y.float() - ref).abs().sum() / ref.abs().sum())
            line += f"  {os.path.basename(os.path.dirname(p))}: {err:.3e}"
        print(line, flush=True)

"""Fixed (prologue + epilogue) vs per-K-tile cost of the phased GEMM: time M x N x K for K = 64..2048."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops
from vda_amd._lib import ACT_GELU
M, N = 43840, 3072
for act in (0, ACT_GELU):
    res = []
    for K in (64, 128, 256, 512, 1024, 2048):
        x = torch.rand(M, K, device="cuda", dtype=torch.float16) * 2 - 1
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
        b = torch.randn(N, device="cuda") * 0.1
        y = torch.empty(M, N, device="cuda", dtype=torch.float16)
        for _ in range(3): ops.gemm(x, w, bias=b, act=act, out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): ops.gemm(x, w, bias=b, act=act, out=y)
        e1.record(); torch.cuda.synchronize()
        res.append((K, e0.elapsed_time(e1) / 20 * 1e3))
    print(f"act={act}: " + "  ".join(f"K={k}:{t:.1f}us" for k, t in res), flush=True)

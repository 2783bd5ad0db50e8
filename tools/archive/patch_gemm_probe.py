"""Where the patch-embed GEMM's time goes (GPU; tools only): M = 32 x 1370 tokens, K = 640, N = 1024
with the forward's per-token row bias vs a plain column bias, vs proj's K = 1024 plain GEMM."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops


def t(fn, iters=20, rounds=7):
    fn()
    torch.cuda.synchronize()
    xs = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        xs.append(e0.elapsed_time(e1) * 1e3 / iters)
    return statistics.median(xs)


dev = "cuda"
M, N = 32 * 1370, 1024
g = torch.Generator(device=dev).manual_seed(0)
for K in (640, 1024):
    a = torch.randn(M, K, device=dev, generator=g).half()
    w = (torch.randn(N, K, device=dev, generator=g) * 0.03).half()
    b = torch.randn(N, device=dev, generator=g)
    rb = torch.randn(1370, N, device=dev, generator=g)
    out = torch.empty(M, N, device=dev, dtype=torch.float16)
    fl = 2.0 * M * N * K
    for name, fn in [("rowbias", lambda: ops.gemm(a, w, rowbias=rb, rdiv=1, rmod=1370, out=out)),
                     ("bias", lambda: ops.gemm(a, w, bias=b, out=out)),
                     ("none", lambda: ops.gemm(a, w, out=out))]:
        us = t(fn)
        print(f"K {K} {name:8s} {us:7.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)

"""Time groupnorm_linear (fused GroupNorm -> proj_in, vda_groupnorm_linear) against the two-op composition
(vda_groupnorm + vda_gemm) at the ViT-L motion-module shapes (tuning tool, not product code).

usage: python tools/ab_gnl.py [iters] [S]
Prints per shape: fused and composed µs per call (HIP events, back-to-back launches), with and without the
stats_out epilogue, the rel-L1 between the two outputs, and the fused call's HBM rate (x in + y out)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
only_s = int(sys.argv[2]) if len(sys.argv) > 2 else None  # one frame size only (for rocprofv3 runs)
dev = "cuda"
torch.manual_seed(0)


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


for Fr, S, C in [(32, 5476, 256), (32, 1369, 256), (32, 361, 256), (32, 74 * 132, 256), (32, 1369, 128), (32, 1369, 64)]:
    if only_s is not None and S != only_s:
        continue
    M = Fr * S
    x = (torch.randn(M, C, device=dev) * 2 + 0.3).half()
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.1
    w = (torch.randn(C, C, device=dev) * C ** -0.5).half()
    bias = torch.randn(C, device=dev) * 0.1
    st = torch.empty(M + 1, 1, 2, device=dev)
    res = []
    for so in (None, st):
        tf = timeit(lambda: ops.groupnorm_linear(x, g, b, Fr, 32, 1e-6, w, bias=bias, stats_out=so))
        tc = timeit(lambda: ops.gemm(ops.groupnorm(x, g, b, Fr, 32, 1e-6), w, bias=bias, stats_out=so))
        res.append((tf, tc))
    yf = ops.groupnorm_linear(x, g, b, Fr, 32, 1e-6, w, bias=bias).double()
    yc = ops.gemm(ops.groupnorm(x, g, b, Fr, 32, 1e-6), w, bias=bias).double()
    r = float((yf - yc).abs().sum() / yc.abs().sum())
    gbs = 4.0 * M * C / (res[0][0] * 1e-6) / 1e9
    print(f"F={Fr} S={S} C={C}: fused {res[0][0]:7.1f} us (stats_out {res[1][0]:7.1f}), composed {res[0][1]:7.1f} us "
          f"(stats_out {res[1][1]:7.1f}); rel-L1 fused vs composed {r:.2e}; fused x+y {gbs:6.0f} GB/s", flush=True)

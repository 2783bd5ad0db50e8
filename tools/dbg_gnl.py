"""Debug: per-frame / per-row error of groupnorm_linear vs the composition (tuning tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops
dev = "cuda"
torch.manual_seed(0)
for Fr, S, C in [(32, 1369, 256), (2, 70, 256), (8, 1369, 256), (3, 12, 256)]:
    M = Fr * S
    x = (torch.randn(M, C, device=dev) + 0.3).half()
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev) * 0.1
    w = (torch.randn(C, C, device=dev) * C ** -0.5).half()
    yf = ops.groupnorm_linear(x, g, b, Fr, 32, 1e-6, w).float()
    yc = ops.gemm(ops.groupnorm(x, g, b, Fr, 32, 1e-6), w).float()
    err = (yf - yc).abs().sum(1) / yc.abs().sum(1)
    bad = (err > 1e-2).nonzero().flatten()
    print(f"F={Fr} S={S}: bad rows {bad.numel()} of {M}", flush=True)
    if bad.numel():
        rows = bad.tolist()
        print("  first bad rows", rows[:10], "last", rows[-5:], "tiles", sorted(set(r // 32 for r in rows))[:20], flush=True)
        print("  bad per frame", torch.bincount(bad // S, minlength=Fr).tolist(), flush=True)
        r = rows[0]
        print("  row", r, "fused", yf[r, :6].tolist(), "composed", yc[r, :6].tolist(), flush=True)

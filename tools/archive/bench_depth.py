"""Depth-head tail microbenchmark (ViT-L 32x518^2 shapes), per kernel config."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops, _lib
L = _lib.lib()
BT, C = 32, 128
x = (torch.randn(BT, 296, 296, C, device="cuda") * 0.5).half()
w = torch.randn(32, 3, 3, C, device="cuda") * (9 * C) ** -0.5
split = torch.cat([w.half(), (w - w.half().float()).half()], 0).contiguous()
b1 = torch.randn(32, device="cuda") * 0.1; w2 = torch.rand(32, device="cuda") * 0.2; b2 = torch.tensor([0.05], device="cuda")
ref = None
for cfg in (0, 1, 2, 3):
    L.vda_debug_force_tile(10 + cfg)
    y = ops.depth_head(x, split, b1, w2, b2, 518, 518)
    if ref is None: ref = y
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5): ops.depth_head(x, split, b1, w2, b2, 518, 518)
    e1.record(); torch.cuda.synchronize()
    print(f"depth cfg{cfg}: {e0.elapsed_time(e1)/5*1e3:.1f} us  maxdiff {float((y-ref).abs().max()):.2e}", flush=True)
L.vda_debug_force_tile(-1)

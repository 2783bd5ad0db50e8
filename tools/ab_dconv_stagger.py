"""Fused depth conv (depth_head at ViT-L's 296^2 -> 518^2, 32 frames) with the second half of its grid
started late by N x 1024 cycles (tuning build's vda_debug_dconv_stagger; tuning tool, not product code).
usage: VDA_LIB_OVERRIDE=build/tune/libvda.so python tools/ab_dconv_stagger.py [N ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd
from vda_amd import ops

lib = vda_amd._libvda()
vals = [int(v) for v in sys.argv[1:]] or [0, 1, 2, 4, 8]
dev = "cuda"
torch.manual_seed(0)
x = (torch.randn(32, 296, 296, 128, device=dev) * 0.5).half()
w1 = (torch.randn(64, 3, 3, 128, device=dev) * 0.03).half()
b1 = torch.randn(32, device=dev) * 0.1
w2 = torch.randn(32, device=dev) * 0.2
b2 = torch.randn(1, device=dev) * 0.1
ref = None
res = {v: [] for v in vals}
for rnd in range(4):
    for v in vals:
        assert lib.vda_debug_dconv_stagger(v) == 0
        for _ in range(2):
            d = ops.depth_head(x, w1, b1, w2, b2, 518, 518)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            d = ops.depth_head(x, w1, b1, w2, b2, 518, 518)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 10 * 1e3)
        if ref is None:
            ref = d.clone()
        assert torch.equal(d, ref)
lib.vda_debug_dconv_stagger(0)
for v in vals:
    r = sorted(res[v])
    print(f"stagger {v:3d} x 1024 cycles: median {r[len(r) // 2]:8.1f} us  (all {', '.join(f'{t:.1f}' for t in res[v])})", flush=True)

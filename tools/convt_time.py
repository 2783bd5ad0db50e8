"""Times the two DPT ConvTranspose(k = s) GEMMs of the ViT-L 32x518^2 forward (dpt.py:70-82): k4s4 256 ch
and k2s2 512 ch on the 37x37 token grid (tuning tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops
BT, h, w = 32, 37, 37
for k, c in ((4, 256), (2, 512)):
    x = torch.randn(BT * h * w, c, device="cuda").half()
    wp = (torch.randn(k * k * c, c, device="cuda") * c ** -0.5).half()
    b = torch.randn(k * k * c, device="cuda") * 0.1
    for _ in range(3):
        ops.conv_transpose_ks(x, wp, b, BT, h, w, k)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    s.record()
    for _ in range(n):
        ops.conv_transpose_ks(x, wp, b, BT, h, w, k)
    e.record()
    e.synchronize()
    us = s.elapsed_time(e) * 1000 / n
    flop = 2.0 * BT * h * w * k * k * c * c
    print(f"ConvT k{k}s{k} {c}ch BT={BT} {h}x{w}: {us:.1f} us  {flop / us / 1e6:.0f} TF/s")
    # the same GEMM with a plain row store (no pixel shuffle) and torch's copy rate for the output bytes
    y = torch.empty(BT * h * w, k * k * c, device="cuda", dtype=torch.float16)
    s.record()
    for _ in range(n):
        ops.gemm(x, wp, bias=b, out=y)
    e.record()
    e.synchronize()
    ug = s.elapsed_time(e) * 1000 / n
    z = torch.empty_like(y)
    s.record()
    for _ in range(n):
        z.copy_(y)
    e.record()
    e.synchronize()
    uc = s.elapsed_time(e) * 1000 / n
    print(f"   row-store GEMM {ug:.1f} us; output {y.numel() * 2 / 1e6:.0f} MB, a device copy of it {uc:.1f} us")

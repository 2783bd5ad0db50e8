"""Isolate the implicit-GEMM conv's K-step cost: the same M x N x K (M = 32*148^2, N = 256, K = 2304)
as a dense GEMM, a 1x1 conv (gather path, no tap re-reads) and the 3x3 conv (Cin = 256)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops, _lib
L = _lib.lib()
def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3
BT, H, W = 32, 148, 148
M, N, K = BT * H * W, 256, 2304
fl = 2.0 * M * N * K
a = (torch.randn(M, K, device="cuda") * 0.5).half()
w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
L.vda_debug_force_tile(-2)
us = t(lambda: ops.gemm(a, w)); print(f"dense GEMM      {us:7.0f} us {fl / us * 1e-6:5.0f} TF/s", flush=True)
x1 = a.view(BT, H, W, K)
us = t(lambda: ops.conv2d(x1, w.view(N, 1, 1, K), ks=1, pad=0)); print(f"1x1 conv (gather) {us:7.0f} us {fl / us * 1e-6:5.0f} TF/s", flush=True)
x3 = (torch.randn(BT, H, W, 256, device="cuda") * 0.5).half()
w3 = (torch.randn(N, 3, 3, 256, device="cuda") * K ** -0.5).half()
us = t(lambda: ops.conv2d(x3, w3)); print(f"3x3 conv Cin 256 {us:7.0f} us {fl / us * 1e-6:5.0f} TF/s", flush=True)
x3b = (torch.randn(BT, H, W, 256, device="cuda") * 0.5).half()
us = t(lambda: ops.conv2d(x3b, w3, pre_relu=True)); print(f"3x3 conv pre-ReLU {us:7.0f} us {fl / us * 1e-6:5.0f} TF/s", flush=True)
L.vda_debug_force_tile(-1)

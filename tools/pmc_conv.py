"""PMC subject: the 148^2 RCU conv (implicit GEMM, 32 x 148^2 x 256 -> 256, K = 2304) and the fc1 GEMM,
3 launches each, for L2 hit-rate passes (rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops, _lib
from vda_amd._lib import ACT_GELU
L = _lib.lib()
L.vda_debug_force_tile(-2)  # implicit GEMM for the Cout = 256 conv
x = (torch.randn(32, 148, 148, 256, device="cuda") * 0.5).half()
w = (torch.randn(256, 3, 3, 256, device="cuda") * 2304 ** -0.5).half()
for _ in range(3):
    ops.conv2d(x, w)
L.vda_debug_force_tile(-1)
a = torch.randn(43840, 1024, device="cuda").half()
w1 = (torch.randn(4096, 1024, device="cuda") * 1024 ** -0.5).half()
b1 = torch.randn(4096, device="cuda") * 0.1
for _ in range(3):
    ops.gemm(a, w1, bias=b1, act=ACT_GELU)
torch.cuda.synchronize()
print("done")

"""PMC subject (tuning tool): the 148^2 RCU conv (halo-tiled, 3x3 256 -> 256 + residual) and the plain fc1-shape
GEMM (bias only), each `reps` times through one library, so per-kernel counters can be set side by side.
usage: python tools/conv_gemm_only.py LIB.so [reps]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib
l = ctypes.CDLL(os.path.abspath(sys.argv[1])); _lib._declare(l)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
torch.manual_seed(0)
st = torch.cuda.current_stream().cuda_stream
BT, H, W, C = 32, 148, 148, 256
x = (torch.randn(BT, H, W, C, device="cuda") * 0.5).half()
w = (torch.randn(C, 3, 3, C, device="cuda") * (9 * C) ** -0.5).half()
b = torch.randn(C, device="cuda") * 0.1
r = torch.randn(BT, H, W, C, device="cuda").half()
y = torch.empty(BT, H, W, C, device="cuda", dtype=torch.float16)
ec = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr(), res=r.data_ptr(), ldres=C)
M, N, K = 43840, 4096, 1024
xg = (torch.randn(M, K, device="cuda")).half()
wg = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
bg = torch.randn(N, device="cuda") * 0.1
yg = torch.empty(M, N, device="cuda", dtype=torch.float16)
eg = _lib.Epilogue(rdiv=1, rmod=1, bias=bg.data_ptr())
for _ in range(reps):
    assert l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), BT, H, W, C, C, 3, 1, 1, 0, 0, 0, ctypes.byref(ec),
                        None, 0, st) == 0
    assert l.vda_gemm(xg.data_ptr(), K, wg.data_ptr(), yg.data_ptr(), N, M, N, K, ctypes.byref(eg), st) == 0
torch.cuda.synchronize()
print("ok")

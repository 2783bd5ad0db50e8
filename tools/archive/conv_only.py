"""Run output_conv1 (tools/ab_conv.py's oc1 case) a few times through one library: a PMC subject.
usage: python tools/conv_only.py LIB.so [reps]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib
l = ctypes.CDLL(os.path.abspath(sys.argv[1])); _lib._declare(l)
torch.manual_seed(0)
x = (torch.randn(32, 148, 148, 256, device="cuda") * 0.5).half()
w = (torch.randn(128, 3, 3, 256, device="cuda") * (9 * 256) ** -0.5).half()
b = torch.randn(128, device="cuda") * 0.1
y = torch.empty(32, 296, 296, 128, device="cuda", dtype=torch.float16)
e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr())
st = torch.cuda.current_stream().cuda_stream
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 2):
    assert l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 148, 148, 256, 128, 3, 1, 1, 0, 296, 296,
                        ctypes.byref(e), None, 0, st) == 0
torch.cuda.synchronize()
print("ok")

"""Run the spatial attention (ViT-L clip shape) a few times through one library: a PMC subject
(tuning tool).  usage: python tools/attn_only.py LIB.so [reps]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib
l = ctypes.CDLL(os.path.abspath(sys.argv[1])); _lib._declare(l)
B, N, H, D = 32, 1370, 16, 64
torch.manual_seed(0)
qkv = (torch.randn(B * N, 3 * H * D, device="cuda") * 1.5).half()
y = torch.empty(B * N, H * D, device="cuda", dtype=torch.float16)
st = torch.cuda.current_stream().cuda_stream
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    assert l.vda_spatial_attention(qkv.data_ptr(), y.data_ptr(), B, N, H, D, D ** -0.5, st) == 0
torch.cuda.synchronize()
print("ok")

"""In-process A/B of the spatial attention across libvda builds (tuning tool, not product code).

usage: python tools/ab_attn.py LIB_A.so[@K] [LIB_B.so[@K] ...] [--rounds R]
(@K: a tuning-build library with vda_debug_attn(K, 0) set, e.g. build/tune/libvda.so@2 = the v2 kernel)
ViT-L clip shape (32 frames x 1370 tokens x 16 heads x 64) through the C ABI (vda_spatial_attention)
on the current torch stream; rounds alternate the libraries; outputs compared bit-for-bit against the
first library's and (first 2 frames) against torch SDPA in fp32.
"""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from vda_amd import _lib

args = sys.argv[1:]
rounds = 7
libs = []
i = 0
while i < len(args):
    if args[i] == "--rounds":
        rounds = int(args[i + 1]); i += 2
    else:
        libs.append(args[i]); i += 1
L = []
for p in libs:
    path, _, knob = p.partition("@")
    l = ctypes.CDLL(os.path.abspath(path))
    _lib._declare(l)
    if knob:
        assert l.vda_debug_attn(int(knob), 0) == 0
    L.append(l)
B, N, H, D = 32, 1370, 16, 64
torch.manual_seed(0)
qkv = (torch.randn(B * N, 3 * H * D, device="cuda") * 1.5).half()
st = torch.cuda.current_stream().cuda_stream
scale = D ** -0.5
q, k, v = qkv.view(B, N, 3, H, D)[:2].float().permute(2, 0, 3, 1, 4)
ref = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(2 * N, H * D)
outs = []
for l in L:
    y = torch.empty(B * N, H * D, device="cuda", dtype=torch.float16)
    assert l.vda_spatial_attention(qkv.data_ptr(), y.data_ptr(), B, N, H, D, scale, st) == 0, l.vda_last_error()
    torch.cuda.synchronize()
    outs.append(y)
errs = [float((o[:2 * N].float() - ref).abs().sum() / ref.abs().sum()) for o in outs]
same = [bool(torch.equal(outs[0], o)) for o in outs[1:]]
times = [[] for _ in L]
n = 10
for r in range(rounds):
    for li, l in enumerate(L):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            l.vda_spatial_attention(qkv.data_ptr(), outs[li].data_ptr(), B, N, H, D, scale, st)
        e1.record()
        torch.cuda.synchronize()
        times[li].append(e0.elapsed_time(e1) / n * 1e3)
fl = 4.0 * B * H * N * N * D
for p, t, e in zip(libs, times, errs):
    print(f"{p}: med {statistics.median(t):6.1f} us  min {min(t):6.1f} us  {fl / statistics.median(t) / 1e6:6.1f} TF  rel-L1 vs SDPA {e:.2e}", flush=True)
print("bit-identical to the first:", same, flush=True)

"""Spatial / temporal attention microbenchmark (TFLOP/s, GB/s) at the ViT-L 32x518^2 shapes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops
def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n
B, N, H, D = 32, 1370, 16, 64
qkv = (torch.randn(B * N, 3 * H * D, device="cuda") * 0.5).half()  # NB: in-situ timings (rocprof of bench.py) are the ground truth
ms = t(lambda: ops.spatial_attention(qkv, B, N, H, D))
print(f"spatial B={B} N={N} H={H}: {ms*1e3:.1f} us  {4*B*H*N*N*D/ms/1e9:.1f} TFLOP/s", flush=True)
for (S, C) in [(1369, 1024), (361, 1024), (1369, 256), (5476, 256)]:
    T = 32
    qkv = torch.randn(T * S, 3 * C, device="cuda", dtype=torch.float16)
    ms = t(lambda: ops.temporal_attention(qkv, 1, T, S, 8, C // 8))
    byts = T * S * C * 2 * 4
    print(f"temporal S={S} C={C}: {ms*1e3:.1f} us  {byts/ms/1e6:.1f} GB/s", flush=True)

"""Spatial-attention microbenchmark at the ViT-L clip shape (32 frames x 1370 tokens x 16 heads x 64):
us per call, TFLOP/s (4·B·H·N²·D), and rel error vs torch SDPA on the same fp16 inputs.  With VDA_LIB_OVERRIDE=build/tune/libvda.so and
VDA_ATTN_OLD=1 the round-1 kernel (vda_debug_attn)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as F
from vda_amd import ops, _lib
if os.environ.get("VDA_ATTN_OLD"):
    _lib.lib().vda_debug_attn(1, 0)

B, N, H, D = 32, 1370, 16, 64
torch.manual_seed(0)
qkv = (torch.randn(B * N, 3 * H * D, device="cuda") * 1.5).half()
fn = lambda: ops.spatial_attention(qkv, B, N, H, D)
y = fn()
q, k, v = qkv.view(B, N, 3, H, D)[:2].float().permute(2, 0, 3, 1, 4)  # error on the first 2 frames
ref = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(2 * N, H * D)
err = ((y[:2 * N].float() - ref).abs().sum() / ref.abs().sum()).item()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3): fn()
e0.record()
for _ in range(20): fn()
e1.record(); torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
print(f"{'old' if os.environ.get('VDA_ATTN_OLD') else 'new'}: {us:.1f} us  {4 * B * H * N * N * D / us * 1e-6:.0f} TF/s  rel-L1 {err:.2e}", flush=True)
for (S, C) in [(1369, 1024), (361, 1024), (1369, 256), (5476, 256)]:
    T = 32
    qkv = torch.randn(T * S, 3 * C, device="cuda", dtype=torch.float16)
    fn = lambda: ops.temporal_attention(qkv, 1, T, S, 8, C // 8)
    fn(); torch.cuda.synchronize()
    e0.record()
    for _ in range(10): fn()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    print(f"temporal S={S} C={C}: {us:.1f} us  {T * S * C * 2 * 4 / us * 1e-3:.1f} GB/s", flush=True)

"""Temporal attention (motion_module.py:302-322) at the ViT-L 32x518^2 motion-module shapes: us per
call and HBM GB/s (q, k, v read + o written).  VDA_TA_OLD=1 selects the direct-load kernel (A/B; tuning build: VDA_LIB_OVERRIDE=build/tune/libvda.so)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops, _lib
if os.environ.get("VDA_TA_OLD"):
    _lib.lib().vda_debug_attn(0, 1)


def t(fn, n=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


tag = "direct-load" if os.environ.get("VDA_TA_OLD") else "lds-staged"
for name, S, C in [("mm0 37^2 C=1024", 37 * 37, 1024), ("mm1 19^2 C=1024", 19 * 19, 1024),
                   ("mm2 37^2 C=256", 37 * 37, 256), ("mm3 74^2 C=256", 74 * 74, 256)]:
    T, H = 32, 8
    qkv = torch.randn(T * S, 3 * C, device="cuda", dtype=torch.float16)
    us = min(t(lambda: ops.temporal_attention(qkv, 1, T, S, H, C // H)) for _ in range(3))
    gb = (T * S * 3 * C + T * S * C) * 2 / 1e9
    print(f"{tag} {name}: {us:.1f} us, {gb / (us * 1e-6) / 1e3:.2f} TB/s", flush=True)

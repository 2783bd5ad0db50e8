"""Upsample microbenchmark: the ViT-L head's bilinear (align_corners=True) resizes, NHWC fp16, 32
frames: 148^2 -> 296^2 (256 ch, refinenet1) and 296^2 -> 518^2 (128 ch, output_conv2 input).
Prints us per call and GB/s of (output + input) bytes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops
for (hi, ho, c) in [(148, 296, 256), (296, 518, 128), (74, 148, 256)]:
    x = torch.randn(32, hi, hi, c, device="cuda").half()
    ops.upsample_bilinear(x, ho, ho)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.upsample_bilinear(x, ho, ho)
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 10 * 1e3
    by = 32 * (ho * ho + hi * hi) * c * 2
    print(f"{hi}->{ho} C={c}: {us:7.1f} us  {by / us * 1e-3:6.0f} GB/s", flush=True)

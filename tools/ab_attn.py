"""In-process A/B of the spatial attention kernels (tuning tool): v2 (4 waves, 2 blocks per CU) vs the
8-wave ping-pong kernel, at the encoder shapes (B = 32 frames, H = 16, N = 1370 / 2443 tokens)."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd
from vda_amd import ops
lib = vda_amd._libvda()
for (B, N, H) in [(32, 1370, 16), (32, 2443, 16), (32, 1370, 6)]:
    D = 64
    qkv = (torch.randn(B * N, 3 * H * D, device="cuda") * 1.5).half()
    outs = {}
    t = {0: [], 1: []}
    for mode in (0, 1):
        lib.vda_debug_attn(mode)
        outs[mode] = ops.spatial_attention(qkv, B, N, H, D)
    for r in range(7):
        for mode in (0, 1):
            lib.vda_debug_attn(mode)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.spatial_attention(qkv, B, N, H, D)
            e1.record(); torch.cuda.synchronize()
            t[mode].append(e0.elapsed_time(e1) / 10 * 1e3)
    lib.vda_debug_attn(0)
    fl = 4.0 * B * H * N * N * D
    print(f"B={B} N={N} H={H}: " + " | ".join(f"mode{m}: med {statistics.median(v):7.1f}us min {min(v):7.1f}us "
                                              f"{fl / statistics.median(v) / 1e6:6.1f}TF" for m, v in t.items())
          + f" | bit-identical {bool(torch.equal(outs[0], outs[1]))}", flush=True)

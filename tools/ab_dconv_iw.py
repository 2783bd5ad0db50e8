"""The fused depth conv (depth_head at ViT-L's 296^2 -> 518^2 and config 5's 296 x 528 -> 518 x 924, 32 frames):
the two-blocks-per-CU kernel vs its interpolation-wave variant (tuning build, vda_debug_dconv(3)), alternating
rounds, outputs compared bitwise.  Tuning tool.  usage: VDA_LIB_OVERRIDE=build/tune/libvda.so python tools/ab_dconv_iw.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd
from vda_amd import ops

lib = vda_amd._libvda()
dev = "cuda"
torch.manual_seed(0)
for (hs, ws, ho, wo) in ((296, 296, 518, 518), (296, 528, 518, 924)):
    x = (torch.randn(32, hs, ws, 128, device=dev) * 0.5).half()
    w1 = (torch.randn(64, 3, 3, 128, device=dev) * 0.03).half()
    b1 = torch.randn(32, device=dev) * 0.1
    w2 = torch.randn(32, device=dev) * 0.2
    b2 = torch.randn(1, device=dev) * 0.1
    res = {-1: [], 3: []}
    outs = {}
    for rnd in range(4):
        for mode in (-1, 3):
            assert lib.vda_debug_dconv(mode) == 0
            for _ in range(2):
                d = ops.depth_head(x, w1, b1, w2, b2, ho, wo)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                d = ops.depth_head(x, w1, b1, w2, b2, ho, wo)
            e1.record()
            torch.cuda.synchronize()
            res[mode].append(e0.elapsed_time(e1) / 10 * 1e3)
            outs[mode] = d.clone()
    lib.vda_debug_dconv(-1)
    same = torch.equal(outs[-1], outs[3])
    for mode, name in ((-1, "2 blocks x 4 waves (product)"), (3, "interpolation waves")):
        r = sorted(res[mode])
        print(f"{hs}x{ws} -> {ho}x{wo}: {name:30s} median {r[len(r) // 2]:8.1f} us  (all {', '.join(f'{t:.1f}' for t in res[mode])})",
              flush=True)
    print(f"  bit-identical: {same}", flush=True)

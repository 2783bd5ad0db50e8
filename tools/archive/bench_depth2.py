"""Depth tail at ViT-L 32 x 296^2 x 128 -> 518^2: the depth conv of vda_dconv.hip with the resize fused
(default), on a materialised resize (vda_debug_dconv(2)), and the older fused halo conv (vda_debug_dconv(0));
us per call, interleaved rounds, same process."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops, _lib
L = _lib.lib()
torch.manual_seed(0)


def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


x1 = (torch.randn(32, 296, 296, 128, device="cuda") * 0.5).half()
w1 = torch.randn(32, 3, 3, 128, device="cuda") * (9 * 128) ** -0.5
split = torch.cat([w1.half(), (w1 - w1.half().float()).half()], 0).contiguous()
b1 = torch.randn(32, device="cuda") * 0.1; w2 = torch.rand(32, device="cuda") * 0.2; b2 = torch.tensor([0.05], device="cuda")
res = {"dconv": [], "dconv_mat": [], "fused": [], "resize": []}
for rnd in range(3):
    L.vda_debug_dconv(-1)
    res["dconv"].append(t(lambda: ops.depth_head(x1, split, b1, w2, b2, 518, 518)))
    L.vda_debug_dconv(2)
    res["dconv_mat"].append(t(lambda: ops.depth_head(x1, split, b1, w2, b2, 518, 518)))
    L.vda_debug_dconv(0)
    res["fused"].append(t(lambda: ops.depth_head(x1, split, b1, w2, b2, 518, 518)))
    res["resize"].append(t(lambda: ops.upsample_bilinear(x1, 518, 518)))
L.vda_debug_dconv(-1)
fl = 2.0 * 32 * 518 * 518 * 64 * 9 * 128
d, dm, f, r = min(res["dconv"]), min(res["dconv_mat"]), min(res["fused"]), min(res["resize"])
print(f"depth tail: dconv (resize fused) {d:.0f} us ({fl / d / 1e6:.0f} TF/s fp16 MFMA) | resize+dconv {dm:.0f} us "
      f"(conv ~{dm - r:.0f} us, {fl / (dm - r) / 1e6:.0f} TF/s) | old fused halo {f:.0f} us | resize alone {r:.0f} us", flush=True)

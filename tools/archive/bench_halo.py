"""Halo-kernel microbenchmark: output_conv1 (conv3x3 256->128 at 32x296^2) and the depth tail
(resize to 518^2 + halo conv), each vs its implicit-GEMM fallback.  us per call, same process."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops, _lib
L = _lib.lib()
torch.manual_seed(0)


def t(fn, n=5):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


x = (torch.randn(32, 296, 296, 256, device="cuda") * 0.5).half()
w = (torch.randn(128, 3, 3, 256, device="cuda") * (9 * 256) ** -0.5).half()
b = torch.randn(128, device="cuda") * 0.1
x1 = (torch.randn(32, 296, 296, 128, device="cuda") * 0.5).half()
w1 = torch.randn(32, 3, 3, 128, device="cuda") * (9 * 128) ** -0.5
split = torch.cat([w1.half(), (w1 - w1.half().float()).half()], 0).contiguous()
b1 = torch.randn(32, device="cuda") * 0.1; w2 = torch.rand(32, device="cuda") * 0.2; b2 = torch.tensor([0.05], device="cuda")
for tag in sys.argv[1:] or ["cur"]:
    tc = t(lambda: ops.conv2d(x, w, bias=b))
    tu = t(lambda: ops.upsample_bilinear(x1, 518, 518))
    td = t(lambda: ops.depth_head(x1, split, b1, w2, b2, 518, 518))
    L.vda_debug_force_tile(3)
    tc0 = t(lambda: ops.conv2d(x, w, bias=b))
    L.vda_debug_force_tile(13)
    td0 = t(lambda: ops.depth_head(x1, split, b1, w2, b2, 518, 518))
    L.vda_debug_force_tile(-1)
    print(f"{os.environ.get('VDA_LIB_OVERRIDE', 'in-tree')}: conv128 halo {tc:.0f} us (implicit {tc0:.0f}) | "
          f"depth halo {td - tu:.0f} us (implicit {td0 - tu:.0f}) | upsample {tu:.0f} us", flush=True)

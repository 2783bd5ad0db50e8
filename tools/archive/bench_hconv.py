"""Halo-tiled phased 3x3 conv (csrc/vda_hconv.hip) vs the implicit-GEMM / strip conv on the decoder's
Cout = 256 shapes (32 frames).  us per call, same process, interleaved rounds; TF/s on 2*M*256*9*Cin."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops, _lib
from vda_amd._lib import ACT_RELU
L = _lib.lib()
torch.manual_seed(0)


def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


for (BT, H, W, Cin) in [(32, 148, 148, 256), (32, 74, 74, 256), (32, 148, 264, 256), (32, 37, 37, 256)]:
    x = (torch.randn(BT, H, W, Cin, device="cuda") * 0.5).half()
    w = (torch.randn(256, 3, 3, Cin, device="cuda") * (9 * Cin) ** -0.5).half()
    b = torch.randn(256, device="cuda") * 0.1
    r1 = torch.randn(BT, H, W, 256, device="cuda").half()
    r2 = torch.randn(BT, H, W, 256, device="cuda").half()
    fl = 2.0 * BT * H * W * 256 * 9 * Cin
    cases = {"plain": dict(), "rcu1": dict(bias=b, pre_relu=True, act=ACT_RELU), "rcu2": dict(bias=b, res=r1, res2=r2)}
    for name, kw in cases.items():
        res = {"hconv": [], "old": []}
        for rnd in range(3):
            for mode in ("hconv", "old"):
                L.vda_debug_hconv(1 if mode == "hconv" else 0)
                res[mode].append(t(lambda: ops.conv2d(x, w, **kw)))
        L.vda_debug_hconv(-1)
        hc, old = min(res["hconv"]), min(res["old"])
        print(f"{BT}x{H}x{W} Cin {Cin} {name}: hconv {hc:.0f} us ({fl / hc / 1e6:.0f} TF/s)  old {old:.0f} us "
              f"({fl / old / 1e6:.0f} TF/s)  {old / hc:.2f}x", flush=True)

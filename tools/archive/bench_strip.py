"""Strip-conv microbenchmark: the ViT-L head's 3x3 convs with 256 outputs (layerN_rn and the fusion
RCU convs, 32 frames at 518^2) on the strip-tiled halo kernel vs the implicit GEMM
(vda_debug_force_tile(-2)).  us per call and TFLOP/s, same process."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
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


BT = 32
for name, cin, hw, rcu in [("layer1_rn", 256, 148, False), ("rcu@148", 256, 148, True), ("layer2_rn", 512, 74, False),
                           ("rcu@74", 256, 74, True), ("layer3_rn", 1024, 37, False), ("rcu@37", 256, 37, True),
                           ("layer4_rn", 1024, 19, False), ("rcu@19", 256, 19, True)]:
    x = (torch.randn(BT, hw, hw, cin, device="cuda") * 0.5).half()
    w = (torch.randn(256, 3, 3, cin, device="cuda") * (9 * cin) ** -0.5).half()
    b = torch.randn(256, device="cuda") * 0.1
    kw = dict(bias=b, res=x, pre_relu=True) if rcu else {}
    L.vda_debug_force_tile(-3)
    ts = t(lambda: ops.conv2d(x, w, **kw))
    L.vda_debug_force_tile(-2)
    ti = t(lambda: ops.conv2d(x, w, **kw))
    L.vda_debug_force_tile(-1)
    fl = 2.0 * BT * hw * hw * 256 * 9 * cin
    print(f"{name:10s} Cin={cin:4d} {hw:3d}^2: strip {ts:7.0f} us ({fl / ts * 1e-6:4.0f} TF/s) | implicit {ti:7.0f} us "
          f"({fl / ti * 1e-6:4.0f} TF/s)", flush=True)

"""Small-M GEMM tile configs (the streaming mode's one-frame encoder, M = 1,370): time per config
(vda_debug_force_tile) and error vs torch fp32.  Diagnostic."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd
from vda_amd import ops, _lib
from vda_amd._lib import ACT_GELU
L = _lib.lib()
torch.manual_seed(0)
cfgs = [int(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "2", "6", "7"])]
for name, M, N, K, act in [("qkv", 1370, 3072, 1024, 0), ("proj", 1370, 1024, 1024, 0), ("fc1", 1370, 4096, 1024, ACT_GELU),
                           ("fc2", 1370, 1024, 4096, 0), ("vits_fc1", 1370, 1536, 384, ACT_GELU), ("vits_qkv", 1370, 1152, 384, 0)]:
    x = torch.rand(M, K, device="cuda", dtype=torch.float16) * 2 - 1
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
    b = torch.randn(N, device="cuda") * 0.1
    r = x.float() @ w.float().t() + b
    ref = torch.nn.functional.gelu(r) if act == ACT_GELU else r
    out = []
    for c in cfgs:
        L.vda_debug_force_tile(c)
        y = ops.gemm(x, w, bias=b, act=act)
        err = float((y.float() - ref).abs().sum() / ref.abs().sum())
        for _ in range(5):
            ops.gemm(x, w, bias=b, act=act, out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ops.gemm(x, w, bias=b, act=act, out=y)
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        out.append(f"cfg{c} {us:6.1f}us err {err:.1e}")
    print(f"{name:9s} {M}x{N}x{K}: " + " | ".join(out), flush=True)
L.vda_debug_force_tile(-1)

"""GEMM / conv tile-config microbenchmark on the GPU (correctness vs torch + TFLOP/s per config)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd
from vda_amd import ops, _lib
from vda_amd._lib import ACT_GELU

L = _lib.lib()
dev = "cuda"
torch.manual_seed(0)
shapes = [("sq4k", 4096, 4096, 4096, 0), ("sq8k", 8192, 8192, 8192, 0)] if os.environ.get("SQ") else []
shapes += [("qkv", 43840, 3072, 1024, 0), ("proj", 43840, 1024, 1024, 0), ("fc1", 43840, 4096, 1024, ACT_GELU),
          ("fc2", 43840, 1024, 4096, 0), ("mm0_qkv", 43808, 3072, 1024, 0), ("mm3_ff1", 175232, 2048, 256, 0),
          ("mm3_ff2", 175232, 256, 1024, 0)]
cfgs = [int(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2", "3"])]
for name, M, N, K, act in shapes:
    x = torch.rand(M, K, device=dev, dtype=torch.float16) * 2 - 1
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    ref = torch.nn.functional.gelu((x.float() @ w.float().t()) + b) if act == ACT_GELU else (x.float() @ w.float().t()) + b
    res = []
    for c in cfgs:
        L.vda_debug_force_tile(c)
        y = ops.gemm(x, w, bias=b, act=act)
        err = float((y.float() - ref).abs().sum() / ref.abs().sum())
        for _ in range(3):
            ops.gemm(x, w, bias=b, act=act, out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            ops.gemm(x, w, bias=b, act=act, out=y)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        res.append(f"cfg{c}: {ms*1e3:8.1f}us {2*M*N*K/ms/1e9:7.1f}TF err={err:.1e}")
    print(f"{name:8s} M={M} N={N} K={K}: " + " | ".join(res), flush=True)
L.vda_debug_force_tile(-1)
# convs
for (BT, H, W, Cin, Cout, st) in [(32, 148, 148, 256, 256, 1), (32, 74, 74, 512, 256, 1), (32, 296, 296, 256, 128, 1),
                                  (32, 37, 37, 1024, 1024, 2)]:
    x = torch.randn(BT, H, W, Cin, device=dev, dtype=torch.float16)
    wt = (torch.randn(Cout, 3, 3, Cin, device=dev) * (9 * Cin) ** -0.5).half()
    res = []
    for c in cfgs:
        L.vda_debug_force_tile(c)
        y = ops.conv2d(x, wt, stride=st)
        for _ in range(2): ops.conv2d(x, wt, stride=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5): ops.conv2d(x, wt, stride=st)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        Ho, Wo = y.shape[1:3]
        fl = 2 * BT * Ho * Wo * Cout * 9 * Cin
        res.append(f"cfg{c}: {ms*1e3:8.1f}us {fl/ms/1e9:7.1f}TF")
    print(f"conv {H}x{W} {Cin}->{Cout} s{st}: " + " | ".join(res), flush=True)
L.vda_debug_force_tile(-1)

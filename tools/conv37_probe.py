"""Under-filled decoder convs at 37^2 (tuning build): the four refinenet RCU convs (3x3 256 -> 256, 172
implicit-GEMM tiles for 256 CUs) and resize_layers[3] (3x3 stride-2 1024 -> 1024 onto 19^2, 184 tiles)
through each route the tuning library offers: default, the strip conv with its own or a forced split count,
and the phased / generic implicit-GEMM tile configurations.  Tuning tool, not product code.

usage: python tools/conv37_probe.py build/tune/libvda.so"""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
_lib._declare(L)
dev = "cuda"
torch.manual_seed(0)
st = torch.cuda.current_stream().cuda_stream


def run_case(name, BT, H, W, Cin, Cout, stride, pre_relu, act, routes):
    x = (torch.randn(BT, H, W, Cin, device=dev) * 0.5).half()
    w = (torch.randn(Cout, 3, 3, Cin, device=dev) * (9 * Cin) ** -0.5).half()
    b = torch.randn(Cout, device=dev) * 0.1
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    y = torch.empty(BT, Ho, Wo, Cout, device=dev, dtype=torch.float16)
    e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr(), act=act)
    fl = 2.0 * BT * Ho * Wo * Cout * 9 * Cin
    ref, out = None, []
    for label, force, split in routes:
        L.vda_debug_force_tile(force)
        L.vda_debug_strip_split(split)
        nb = L.vda_conv2d_workspace(BT, H, W, Cin, Cout, 3, stride, 1)
        ws = torch.empty(max(nb, 16), device=dev, dtype=torch.uint8)
        call = lambda: L.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), BT, H, W, Cin, Cout, 3, stride, 1, pre_relu,
                                    0, 0, ctypes.byref(e), ws.data_ptr(), nb, st)
        rc = call()
        if rc != 0:
            out.append(f"{label}: rc {rc} {L.vda_last_error().decode()[:60]}")
            continue
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        err = float((y.float() - ref.float()).abs().sum() / ref.float().abs().sum())
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10 * 1e3)
        t = statistics.median(ts)
        out.append(f"{label}: {t:6.1f}us {fl / t / 1e6:6.1f}TF d={err:.1e} ws={nb >> 20}MB")
    L.vda_debug_force_tile(-1)
    L.vda_debug_strip_split(0)
    print(f"{name}: " + " | ".join(out), flush=True)


rcu = [("default", -1, 0), ("strip", -3, 0), ("strip/2", -3, 2), ("strip/4", -3, 4), ("strip/8", -3, 8),
       ("cfg0", 0, 0), ("cfg1", 1, 0), ("cfg2", 2, 0), ("cfg3", 3, 0)]
run_case("rcu37 256->256", 32, 37, 37, 256, 256, 1, 1, _lib.ACT_RELU, rcu)
s2 = [("default", -1, 0), ("cfg0", 0, 0), ("cfg1", 1, 0), ("cfg2", 2, 0), ("cfg3", 3, 0), ("cfg5", 5, 0)]
run_case("rl3 1024->1024 s2", 32, 37, 37, 1024, 1024, 2, 0, _lib.ACT_NONE, s2)

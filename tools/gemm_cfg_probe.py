"""The decoder's narrow / short-K GEMMs through every tile configuration of the tuning build (tuning
tool, not product code): the DPT projects (1x1 conv 1024 -> 256 / 512 at 37^2, 32 frames) and the
fusion blocks' out_conv (1x1 256 -> 256 at 148^2 / 74^2).  Bias epilogue, row-store output.

usage: python tools/gemm_cfg_probe.py build/tune/libvda.so"""
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
cases = [("project N=256", 32 * 37 * 37, 1024, 256), ("project N=512", 32 * 37 * 37, 1024, 512),
         ("out_conv 148^2", 32 * 148 * 148, 256, 256), ("out_conv 74^2", 32 * 74 * 74, 256, 256)]
for name, M, K, N in cases:
    x = (torch.randn(M, K, device=dev) * 0.5).half()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr())
    fl = 2.0 * M * N * K
    out, ref = [], None
    for cfg in (-1, 0, 1, 2, 3, 4):
        L.vda_debug_force_tile(cfg)
        call = lambda: L.vda_gemm(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), N, M, N, K, ctypes.byref(e), st)
        if call() != 0:
            out.append(f"cfg{cfg}: rc"); continue
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        d = float((y.float() - ref.float()).abs().max())
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
        out.append(f"{'auto' if cfg < 0 else 'cfg%d' % cfg}: {t:6.1f}us {fl / t / 1e6:5.0f}TF d={d:.0e}")
    L.vda_debug_force_tile(-1)
    print(f"{name} (M={M} K={K} N={N}): " + " | ".join(out), flush=True)

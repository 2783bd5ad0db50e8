"""Tile configurations on the motion modules' short-K GEMMs (K = 256, mm2 / mm3 at C = 256), through
the tuning build's vda_debug_force_tile (tuning tool).  usage: python tools/bench_small_k.py [M]
Prints us per call per configuration (-1 = the automatic choice) and checks every configuration's
output against the automatic one (rel-L1)."""
import ctypes, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import _lib
L = ctypes.CDLL(_lib.TUNE_LIB_PATH); _lib._declare(L)
M = int(sys.argv[1]) if len(sys.argv) > 1 else 175232
T, S = 32, M // 32
dev = "cuda"
torch.manual_seed(0)
st = torch.cuda.current_stream().cuda_stream


def case(name):
    C = 256
    K, N = (C, 3 * C) if name == "qkv" else (C, 8 * C) if name == "ff1" else (4 * C, C) if name == "ff2" else (C, C)
    x = (torch.randn(M, K, device=dev) * 0.5).half()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    e = _lib.Epilogue(rdiv=1, rmod=1)
    keep = [x, w, b]
    if name == "qkv":
        rb = torch.randn(T, N, device=dev) * 0.1; keep.append(rb)
        e.rowbias, e.rdiv, e.rmod = rb.data_ptr(), S, T
    else:
        e.bias = b.data_ptr()
    if name == "ff1":
        e.act = _lib.ACT_GEGLU
    y = torch.empty(M, N // 2 if name == "ff1" else N, device=dev, dtype=torch.float16)
    if name in ("out", "ff2"):
        r = torch.randn(M, N, device=dev).half(); so = torch.empty(M + 1, (N + 255) // 256, 2, device=dev)
        keep += [r, so]
        e.res, e.ldres, e.stats_out = r.data_ptr(), N, so.data_ptr()
    fl = 2.0 * M * N * K
    return x, w, y, e, K, N, fl, keep


for name in ["pin", "out", "qkv", "ff1", "ff2"]:
    x, w, y, e, K, N, fl, keep = case(name)
    res = {}
    ref = None
    for cfg in [-1, 0, 1, 2, 3, 4, 7]:
        L.vda_debug_force_tile(cfg)
        rc = L.vda_gemm(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), y.shape[1], M, N, K, ctypes.byref(e), st)
        if rc != 0:
            res[cfg] = "rc"; continue
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        err = float((y.float() - ref.float()).abs().sum() / ref.float().abs().sum().clamp_min(1e-30))
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                L.vda_gemm(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), y.shape[1], M, N, K, ctypes.byref(e), st)
            e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 5 * 1e3)
        res[cfg] = f"{statistics.median(ts):.1f}us ({fl / statistics.median(ts) / 1e6:.0f}TF, {err:.0e})"
    L.vda_debug_force_tile(-1)
    print(f"{name} M={M} N={N} K={K}: " + " | ".join(f"{k}: {v}" for k, v in res.items()), flush=True)

"""Per-phase timing of every tile of the phased encoder GEMMs (tuning tool, not product code).

usage: bash tools/build_ts.sh && python tools/ts_probe2.py build/ts/libvda.so
The -DVDA_TS build stamps s_memrealtime (100 MHz) at the phase boundaries of every tile (g_ts[tile][k]):
0 tile start, 2 main loop start (prologue wait done), 3 main loop end, 4 epilogue phase 1 done,
5 stores issued, 7 tile end.  Printed: medians per persistent round (round r = tiles r*grid ..).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from vda_amd import _lib

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
_lib._declare(L)
L.vda_debug_timestamps.argtypes = [ctypes.c_void_p]
dev = "cuda"
torch.manual_seed(0)
M, C = 43840, 1024
tok = (torch.randn(M, C, device=dev) * 2).half()
st = torch.cuda.current_stream().cuda_stream
grid = torch.cuda.get_device_properties(0).multi_processor_count


def row_partials(y):
    yf = y.float().view(y.shape[0], -1, 256)
    return torch.stack([yf.sum(-1), (yf * yf).sum(-1)], -1).contiguous()


for name in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["qkv", "proj", "fc1", "fc2"]):
    K, N = (C, 3 * C) if name == "qkv" else (C, C) if name == "proj" else (C, 4 * C) if name == "fc1" else (4 * C, C)
    x = tok if K == C else (torch.randn(M, K, device=dev) * 0.5).half()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    e = _lib.Epilogue()
    e.bias = b.data_ptr(); e.rdiv = 1; e.rmod = 1
    keep = []
    if name in ("qkv", "fc1"):
        stats = row_partials(x); cs = w.float().sum(1).contiguous(); keep += [stats, cs]
        e.ln_stats = stats.data_ptr(); e.ln_colsum = cs.data_ptr(); e.ln_parts = 4; e.ln_eps = 1e-6
        e.act = _lib.ACT_GELU if name == "fc1" else _lib.ACT_NONE
    y = torch.randn(M, N, device=dev).half()
    if name in ("proj", "fc2"):
        so = torch.empty(M + 1, (N + 255) // 256, 2, device=dev); keep.append(so)
        e.res = y.data_ptr(); e.ldres = N; e.stats_out = so.data_ptr()
    for _ in range(4):
        assert L.vda_gemm(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), N, M, N, K, ctypes.byref(e), st) == 0
    torch.cuda.synchronize()
    buf = np.zeros((4096, 8), dtype=np.uint64)
    L.vda_debug_timestamps(ctypes.c_void_p(buf.ctypes.data))
    ntiles = ((M + 255) // 256) * (N // 256)
    ts = buf[:ntiles].astype(np.float64) / 100.0  # us
    t0 = ts[:, 0].min()
    rounds = (ntiles + grid - 1) // grid
    print(f"{name} {M}x{N}x{K}: {ntiles} tiles, {rounds} rounds, kernel span {ts[:, 7].max() - t0:.1f} us", flush=True)
    for r in range(rounds):
        v = ts[r * grid:(r + 1) * grid]
        d = lambda a, b: np.median(v[:, b] - v[:, a])
        print(f"  round {r:2d} ({len(v):3d} tiles): start {np.median(v[:, 0]) - t0:6.1f}  prologue-wait {d(0, 2):5.2f}  "
              f"main {d(2, 3):6.2f}  epi1 {d(3, 4):5.2f}  stores {d(4, 5):5.2f}  tail {d(5, 7):5.2f}  tile {d(0, 7):6.2f}  "
              f"spread(start) {v[:, 0].max() - v[:, 0].min():5.1f}", flush=True)

"""Per-block phase timing of the halo-tiled 256-channel conv (tuning tool, not product code).

usage: bash tools/build_ts.sh && python tools/ts_hconv.py build/ts/libvda.so
The -DVDA_TS build keeps s_memrealtime stamps (100 MHz) in registers and stores them at each block's end:
0 block start, 1 prologue landed (patch slab 0 + W, after the barrier), 2 main loop end, 3 epilogue LDS
image written, 4 stores issued, 5 stores retired.  Printed: medians over the blocks, and the gap between a
block's end and the next block's start on the same CU slot (approximated per blockIdx + grid stride).
Shape: refinenet1's RCU conv2 at 148^2 (3x3 256 -> 256, bias, residual), 32 frames."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from vda_amd import _lib

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
_lib._declare(L)
L.vda_debug_hconv_timestamps.argtypes = [ctypes.c_void_p]
dev = "cuda"
torch.manual_seed(0)
st = torch.cuda.current_stream().cuda_stream
for name, pre, relu, with_res in (("rcu148 conv1 (pre-relu, relu)", 1, 1, False), ("rcu148 conv2 (+res)", 0, 0, True)):
    BT, H, W, C = 32, 148, 148, 256
    x = (torch.randn(BT, H, W, C, device=dev) * 0.5).half()
    w = (torch.randn(C, 3, 3, C, device=dev) * (9 * C) ** -0.5).half()
    b = torch.randn(C, device=dev) * 0.1
    r = torch.randn(BT, H, W, C, device=dev).half()
    y = torch.empty(BT, H, W, C, device=dev, dtype=torch.float16)
    e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr(), act=_lib.ACT_RELU if relu else 0)
    if with_res:
        e.res = r.data_ptr(); e.ldres = C
    for _ in range(3):
        assert L.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), BT, H, W, C, C, 3, 1, 1, pre, 0, 0,
                            ctypes.byref(e), None, 0, st) == 0, L.vda_last_error()
    torch.cuda.synchronize()
    buf = np.zeros((8192, 6), dtype=np.uint64)
    L.vda_debug_hconv_timestamps(ctypes.c_void_p(buf.ctypes.data))
    ntiles = BT * ((H + 7) // 8) * ((W + 31) // 32)
    n = min(ntiles, 8192)
    ts = buf[:n].astype(np.float64) / 100.0
    t0 = ts[:, 0].min()
    d = lambda a, c: np.median(ts[:, c] - ts[:, a])
    print(f"{name}: {ntiles} blocks, span {ts[:, 5].max() - t0:.1f} us | prologue {d(0, 1):.2f}  main {d(1, 2):.2f}  "
          f"epi-stage {d(2, 3):.2f}  epi-store-issue {d(3, 4):.2f}  store-drain {d(4, 5):.2f}  block {d(0, 5):.2f} us",
          flush=True)
    # start gaps: sort block starts; per CU slot the next block starts after some block ends
    starts = np.sort(ts[:, 0]) - t0
    ends = np.sort(ts[:, 5]) - t0
    g = 256
    gaps = starts[g:] - ends[:len(starts) - g]
    print(f"   block start after the matching earlier block end (k-th start vs k-th end): median {np.median(gaps):.2f} us, "
          f"p90 {np.percentile(gaps, 90):.2f} us", flush=True)

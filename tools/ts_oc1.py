"""Step-class cycle sums of output_conv1's halo conv (tuning tool, not product code).

usage: bash tools/build_ts.sh && python tools/ts_oc1.py build/ts/libvda.so
The -DVDA_TS build sums s_memtime deltas between consecutive end-of-step barriers per step class (the
step's tap 0..8 within a 64-channel slab, 9 = a tile's last step, which carries the epilogue) and
stores them per block.  Printed: cycles per step of each class (median over blocks), the share of
the kernel each class takes, and the in-kernel clock (s_memtime / s_memrealtime)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from vda_amd import _lib

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
_lib._declare(L)
L.vda_debug_oc1_timestamps.argtypes = [ctypes.c_void_p]
dev = "cuda"
torch.manual_seed(0)
st = torch.cuda.current_stream().cuda_stream
x = (torch.randn(32, 148, 148, 256, device=dev) * 0.5).half()
w = (torch.randn(128, 3, 3, 256, device=dev) * (9 * 256) ** -0.5).half()
b = torch.randn(128, device=dev) * 0.1
y = torch.empty(32, 296, 296, 128, device=dev, dtype=torch.float16)
e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr())
for _ in range(5):
    assert L.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 148, 148, 256, 128, 3, 1, 1, 0, 296, 296,
                        ctypes.byref(e), None, 0, st) == 0, L.vda_last_error()
torch.cuda.synchronize()
buf = np.zeros((1024, 24), dtype=np.uint64)
L.vda_debug_oc1_timestamps(ctypes.c_void_p(buf.ctypes.data))
used = buf[:, 20] > 0
B = buf[used].astype(np.float64)
print(f"blocks {int(used.sum())}, clock {np.median(B[:, 21] / (B[:, 20] / 100.0)) / 1e3:.3f} GHz, "
      f"kernel {np.median(B[:, 20]) / 100.0:.1f} us per block", flush=True)
tot = B[:, :10].sum(1)
print(f"  end-of-step vmcnt wait + barrier: {np.median(B[:, 22] / tot):.3f} of the step cycles", flush=True)
for c in range(10):
    n = B[:, 10 + c]
    if n.sum() == 0:
        continue
    per = np.median(B[:, c] / np.maximum(n, 1))
    share = np.median(B[:, c] / tot)
    name = "tile end (last step)" if c == 9 else f"tap {c}" + (" (+source DMA)" if c == 0 else "") + (" (+interp)" if c == 8 else "")
    print(f"  {name:24s}: {per:8.0f} cycles/step  n/block {np.median(n):5.0f}  share {share:.3f}", flush=True)

"""Phase-class cycle sums of the fused depth conv (tuning tool, not product code).

usage: bash tools/build_ts.sh && python tools/ts_dconv.py build/ts/libvda.so
The -DVDA_TS build sums s_memtime deltas between the phase-start barriers of depth_conv_kernel<true>
per phase class (the kernel row dy = 0..2 of a 32-channel unit; 3 = a tile's last phase, which carries
the epilogue; row 1 also interpolates the next unit's patch) and stores them per block.  Printed:
cycles per phase of each class (median over blocks), the share of the kernel, the end-of-phase wait +
barrier share and the in-kernel clock.  Shape: the ViT-L depth tail at 518^2 (resize from 296^2)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from vda_amd import _lib

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
_lib._declare(L)
L.vda_debug_dconv_timestamps.argtypes = [ctypes.c_void_p]
dev = "cuda"
torch.manual_seed(0)
st = torch.cuda.current_stream().cuda_stream
x = (torch.randn(32, 296, 296, 128, device=dev) * 0.5).half()
w32 = torch.randn(32, 3, 3, 128, device=dev) * (9 * 128) ** -0.5
w1 = torch.cat([w32.half(), (w32 - w32.half().float()).half()], 0).contiguous()
b1, w2, b2 = torch.randn(32, device=dev) * 0.1, torch.rand(32, device=dev) * 0.2, torch.tensor([0.05], device=dev)
d = torch.empty(32, 518, 518, device=dev)
for _ in range(5):
    assert L.vda_depth_head(x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), d.data_ptr(),
                            None, 32, 296, 296, 128, 518, 518, st) == 0, L.vda_last_error()
torch.cuda.synchronize()
buf = np.zeros((1024, 12), dtype=np.uint64)
L.vda_debug_dconv_timestamps(ctypes.c_void_p(buf.ctypes.data))
used = buf[:, 8] > 0
B = buf[used].astype(np.float64)
print(f"blocks {int(used.sum())}, clock {np.median(B[:, 9] / (B[:, 8] / 100.0)) / 1e3:.3f} GHz, "
      f"kernel {np.median(B[:, 8]) / 100.0:.1f} us per block", flush=True)
tot = B[:, :4].sum(1)
print(f"  end-of-phase wait + barrier: {np.median(B[:, 10] / tot):.3f} of the phase cycles", flush=True)
names = ["row 0 (+source DMA at row 2 of the unit before)", "row 1 (+interp)", "row 2", "tile end (row 2 + epilogue)"]
for c in range(4):
    n = B[:, 4 + c]
    if n.sum() == 0:
        continue
    print(f"  {names[c]:48s}: {np.median(B[:, c] / np.maximum(n, 1)):8.0f} cycles/phase  n/block {np.median(n):5.0f}  "
          f"share {np.median(B[:, c] / tot):.3f}", flush=True)

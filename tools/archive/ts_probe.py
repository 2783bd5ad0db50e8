"""Per-phase timing of the phased GEMM's first tile on every block (needs the -DVDA_TS build:
VDA_LIB_OVERRIDE=build/ts/libvda_ts.so).  100 MHz s_memrealtime stamps -> microseconds."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from vda_amd import ops, _lib
from vda_amd._lib import ACT_GELU
L = _lib.lib()
def probe(M, N, K, act, sched=(-1, 0)):
    L.vda_debug_gemm_sched(*sched)
    x = torch.rand(M, K, device="cuda", dtype=torch.float16) * 2 - 1
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
    b = torch.randn(N, device="cuda") * 0.1
    y = torch.empty(M, N, device="cuda", dtype=torch.float16)
    for _ in range(3): ops.gemm(x, w, bias=b, act=act, out=y)
    torch.cuda.synchronize()
    buf = np.zeros((1024, 8), dtype=np.uint64)
    ops.gemm(x, w, bias=b, act=act, out=y); torch.cuda.synchronize()
    L.vda_debug_timestamps(ctypes.c_void_p(buf.ctypes.data))
    ts = buf[:256].astype(np.float64) / 100.0  # us
    v = ts[(ts[:, 0] > 0)]
    d = np.diff(v, axis=1)
    names = ["stagger", "prologue", "mainloop", "epi-ph1", "epi-ph2", "drain", "tail"]
    med = np.median(d, axis=0)
    print(f"{M}x{N}x{K} act{act} sched{sched}: blocks {len(v)}  start spread {v[:,0].max()-v[:,0].min():.1f}us  "
          + "  ".join(f"{n}={m:.2f}" for n, m in zip(names, med)) + f"  tile={np.median(v[:,7]-v[:,0]):.2f}", flush=True)
probe(43840, 3072, 1024, 0)
probe(43840, 4096, 1024, ACT_GELU)
probe(43840, 1024, 4096, 0)
probe(43840, 1024, 1024, 0)

"""Persistent-grid / start-stagger probe for the phased GEMM (qkv and fc1 shapes)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops, _lib
from vda_amd._lib import ACT_GELU
L = _lib.lib()
def run(M, N, K, act):
    x = torch.rand(M, K, device="cuda", dtype=torch.float16) * 2 - 1
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
    b = torch.randn(N, device="cuda") * 0.1
    y = torch.empty(M, N, device="cuda", dtype=torch.float16)
    ref = None
    out = []
    for persist, stag in [(0, 0), (0, 0), (-1, 0), (-1, -1), (-1, 500), (-1, 1000), (-1, 1500), (-1, 2000)]:
        L.vda_debug_gemm_sched(persist, stag)
        ops.gemm(x, w, bias=b, act=act, out=y); torch.cuda.synchronize()
        if ref is None: ref = y.clone()
        ok = torch.equal(ref, y)
        for _ in range(3): ops.gemm(x, w, bias=b, act=act, out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): ops.gemm(x, w, bias=b, act=act, out=y)
        e1.record(); torch.cuda.synchronize()
        out.append(f"p{persist}s{stag}:{e0.elapsed_time(e1) / 20 * 1e3:.1f}{'' if ok else '!'}")
    L.vda_debug_gemm_sched(-1, -1)
    print(f"{M}x{N}x{K} act{act}: " + " ".join(out), flush=True)
run(43840, 3072, 1024, 0)
run(43840, 4096, 1024, ACT_GELU)
run(43840, 1024, 4096, 0)
run(43840, 1024, 1024, 0)

"""Desynchronised-start probe for the phased GEMM: do the CUs' epilogue store bursts cost time when
every block runs its tiles in lockstep?  (vda_debug_gemm_desync; encoder GEMM shapes, random data)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops, _lib
from vda_amd._lib import ACT_GELU
L = _lib.lib()


def run(M, N, K, act, cfgs):
    x = torch.rand(M, K, device="cuda", dtype=torch.float16) * 2 - 1
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
    b = torch.randn(N, device="cuda") * 0.1
    y = torch.empty(M, N, device="cuda", dtype=torch.float16)
    res = {c: [] for c in cfgs}
    ref = None
    for rnd in range(3):  # interleaved rounds
        for (g, t) in cfgs:
            L.vda_debug_gemm_desync(g)
            L.vda_debug_gemm_sched(-1, t)
            ops.gemm(x, w, bias=b, act=act, out=y)
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            assert torch.equal(ref, y)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.gemm(x, w, bias=b, act=act, out=y)
            e1.record()
            torch.cuda.synchronize()
            res[(g, t)].append(e0.elapsed_time(e1) / 10 * 1e3)
    L.vda_debug_gemm_desync(0)
    L.vda_debug_gemm_sched(-1, -1)
    print(f"{M}x{N}x{K} act{act}: " + "  ".join(f"g{g}t{t}:{min(v):.1f}" for (g, t), v in res.items()), flush=True)


cfgs = [(0, -1), (2, 1500), (2, 3000), (4, 3000), (4, 1500), (8, 3000)]
run(43840, 4096, 1024, ACT_GELU, cfgs)
run(43840, 3072, 1024, 0, cfgs)
run(43840, 1024, 4096, 0, cfgs)
run(43840, 1024, 1024, 0, cfgs)

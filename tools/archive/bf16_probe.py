"""Power/clock probe: the phased GEMM on fp16 vs bf16-bit-pattern operands (experimental lib built with
-DVDA_MFMA_BF16 multiplies bf16).  usage: VDA_LIB_OVERRIDE=... python tools/bf16_probe.py [bf16]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops, _lib
L = _lib.lib(); L.vda_debug_force_tile(4)
dt = torch.bfloat16 if (len(sys.argv) > 1 and sys.argv[1] == "bf16") else torch.float16
for M, N, K in [(8192, 8192, 8192), (4096, 4096, 4096), (43840, 3072, 1024)]:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(dt).view(torch.float16)
    w = (torch.rand(N, K, device="cuda") * 2 - 1).to(dt).view(torch.float16)
    y = torch.empty(M, N, device="cuda", dtype=torch.float16)
    for _ in range(3): ops.gemm(x, w, out=y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): ops.gemm(x, w, out=y)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"{dt} {M}x{N}x{K}: {ms*1e3:.1f} us {2*M*N*K/ms/1e9:.1f} TF", flush=True)

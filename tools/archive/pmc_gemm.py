"""Run one GEMM shape repeatedly (PMC subject).  usage: pmc_gemm.py M N K [act] [reps]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops
M, N, K = (int(a) for a in sys.argv[1:4])
act = int(sys.argv[4]) if len(sys.argv) > 4 else 0
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
x = torch.randn(M, K, device="cuda", dtype=torch.float16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
b = torch.randn(N, device="cuda") * 0.1
y = torch.empty(M, N // (2 if act == 2 else 1), device="cuda", dtype=torch.float16)
for _ in range(reps):
    ops.gemm(x, w, bias=b, act=act, out=y)
torch.cuda.synchronize()

"""Run one encoder GEMM (tools/ab_gemm.py's exact operands / epilogues) a few times through the C ABI
of the given library: a PMC subject that does not depend on libvda_torch.so (tuning tool).
usage: python tools/gemm_only.py LIB.so [qkv|proj|fc1|fc2] [reps]"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib
l = ctypes.CDLL(os.path.abspath(sys.argv[1])); _lib._declare(l)
name = sys.argv[2] if len(sys.argv) > 2 else "fc1"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
M, C = 43840, 1024
torch.manual_seed(0)
K, N = (C, 3 * C) if name == "qkv" else (C, C) if name == "proj" else (C, 4 * C) if name == "fc1" else (4 * C, C)
x = (torch.randn(M, K, device="cuda") * (2 if K == C else 0.5)).half()
w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
b = torch.randn(N, device="cuda") * 0.1
e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr())
keep = []
if name in ("qkv", "fc1"):
    xf = x.float().view(M, -1, 256)
    stats = torch.stack([xf.sum(-1), (xf * xf).sum(-1)], -1).contiguous()
    cs = w.float().sum(1).contiguous()
    keep += [stats, cs]
    e.ln_stats, e.ln_colsum, e.ln_parts, e.ln_eps = stats.data_ptr(), cs.data_ptr(), 4, 1e-6
    e.act = _lib.ACT_GELU if name == "fc1" else _lib.ACT_NONE
y = torch.randn(M, N, device="cuda").half()
if name in ("proj", "fc2"):
    so = torch.empty(M + 1, (N + 255) // 256, 2, device="cuda"); keep.append(so)
    e.res, e.ldres, e.stats_out = y.data_ptr(), N, so.data_ptr()
st = torch.cuda.current_stream().cuda_stream
for _ in range(reps):
    assert l.vda_gemm(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), N, M, N, K, ctypes.byref(e), st) == 0
torch.cuda.synchronize()
print("ok", name, (M * K + N * K + M * N) * 2, "algorithmic bytes")

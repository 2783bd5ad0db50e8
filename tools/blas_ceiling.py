"""Calibration: the vendor library's fp16 GEMM (torch.matmul -> hipBLASLt) on the four encoder shapes,
beside this repo's dense GEMM (ops.gemm, bias only, no LN fold) on the same operands.  Tells how far the
phased 256x256 kernel sits from what the platform's own GEMM reaches on these shapes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd
from vda_amd import ops

dev = "cuda"
torch.manual_seed(0)
shapes = [("qkv", 43840, 3072, 1024), ("proj", 43840, 1024, 1024), ("fc1", 43840, 4096, 1024), ("fc2", 43840, 1024, 4096)]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for name, M, N, K in shapes:
    x = torch.rand(M, K, device=dev, dtype=torch.float16) * 2 - 1
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = (torch.randn(N, device=dev) * 0.1)
    wt = w.t()
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    fl = 2 * M * N * K
    t_blas = timeit(lambda: torch.matmul(x, wt, out=y))
    t_blas_b = timeit(lambda: torch.addmm(b.half(), x, wt, out=y))
    t_ours = timeit(lambda: ops.gemm(x, w, bias=b, out=y))
    print(f"{name:5s} M={M} N={N} K={K}: hipBLASLt {t_blas*1e3:7.1f} us {fl/t_blas/1e9:7.1f} TF | "
          f"addmm {t_blas_b*1e3:7.1f} us {fl/t_blas_b/1e9:7.1f} TF | vda {t_ours*1e3:7.1f} us {fl/t_ours/1e9:7.1f} TF",
          flush=True)

"""Vendor-library reference points on the same shapes (hipBLASLt via torch.matmul, SDPA attention),
next to libvda's own kernels, random fp16 data.  Diagnostic only: tells how far from the library
ceiling each libvda kernel is."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
import vda_amd
from vda_amd import ops
from vda_amd._lib import ACT_GELU

dev = "cuda"
torch.manual_seed(0)


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


for name, M, N, K in [("qkv", 43840, 3072, 1024), ("fc1", 43840, 4096, 1024), ("fc2", 43840, 1024, 4096),
                      ("sq8k", 8192, 8192, 8192)]:
    x = torch.rand(M, K, device=dev, dtype=torch.float16) * 2 - 1
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    fl = 2 * M * N * K
    t_lib = timeit(lambda: torch.matmul(x, w.t()))
    t_lin = timeit(lambda: F.linear(x, w, b.half()))
    t_vda = timeit(lambda: ops.gemm(x, w, bias=b))
    print(f"{name:5s} M={M} N={N} K={K}: hipBLASLt matmul {fl / t_lib / 1e9:7.1f} TF | F.linear+bias "
          f"{fl / t_lin / 1e9:7.1f} TF | libvda {fl / t_vda / 1e9:7.1f} TF", flush=True)

B, N, H, D = 32, 1370, 16, 64
qkv = torch.randn(B * N, 3 * H * D, device=dev, dtype=torch.float16)
q, k, v = qkv.view(B, N, 3, H, D).permute(2, 0, 3, 1, 4).contiguous().unbind(0)
fl = 4 * B * H * N * N * D
for be, name in ((torch.nn.attention.SDPBackend.FLASH_ATTENTION, "flash"),
                 (torch.nn.attention.SDPBackend.EFFICIENT_ATTENTION, "efficient")):
    try:
        with torch.nn.attention.sdpa_kernel(be):
            t = timeit(lambda: F.scaled_dot_product_attention(q, k, v))
        print(f"SDPA {name}: {t * 1e3:.1f} us {fl / t / 1e9:.1f} TF", flush=True)
    except Exception as e:
        print(f"SDPA {name}: unavailable ({type(e).__name__}: {str(e)[:80]})")
t = timeit(lambda: ops.spatial_attention(qkv, B, N, H, D))
print(f"libvda spatial_attention: {t * 1e3:.1f} us {fl / t / 1e9:.1f} TF", flush=True)

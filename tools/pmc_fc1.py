"""Run the encoder fc1 GEMM of ViT-L 32x518x518 as the forward runs it (norm2 folded in: partial row
statistics from the proj epilogue, + GELU) a few times: the PMC subject for bench.py's roofline.traffic
(rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, tools/refresh_profiles.sh)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops
from vda_amd._lib import ACT_GELU
M, N, K = 32 * 1370, 4096, 1024
x = torch.randn(M, K, device="cuda", dtype=torch.float16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).half()
b = torch.randn(N, device="cuda") * 0.1
c1 = w.float().sum(1)
xf = x.float().view(M, 4, 256)
st = torch.stack([xf.sum(2), (xf * xf).sum(2)], 2).contiguous()  # [M, 4, 2] partial (sum, sumsq)
y = torch.empty(M, N, device="cuda", dtype=torch.float16)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    ops.gemm(x, w, bias=b, act=ACT_GELU, ln_stats=st, ln_parts=4, ln_eps=1e-6, ln_colsum=c1, out=y)
torch.cuda.synchronize()
print("alg bytes per launch", (M * K + N * K + M * N) * 2 + M * 4 * 2 * 4)

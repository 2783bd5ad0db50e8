import os, sys, statistics, torch
sys.path.insert(0, "/root/repo")
from vda_amd import ops
dev = "cuda"
torch.manual_seed(0)
BT, H, W, C = 32, 37, 37, 1024
x = (torch.randn(BT, H, W, C, device=dev) * 0.5).half()
w = (torch.randn(C, 3, 3, C, device=dev) * (9 * C) ** -0.5).half()
b = torch.randn(C, device=dev) * 0.1
Ho = (H + 2 - 3) // 2 + 1
M, K = BT * Ho * Ho, 9 * C
a = torch.randn(M, K, device=dev).half()
wk = w.reshape(C, K)
def t(fn, n=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / n * 1e3
# the explicit im2col in torch (unfold) for the copy cost estimate
def im2col():
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1))
    cols = xp.unfold(1, 3, 2).unfold(2, 3, 2)  # [BT, Ho, Wo, C, 3, 3]
    return cols.permute(0, 1, 2, 4, 5, 3).reshape(M, K).contiguous()
for r in range(3):
    tc = t(lambda: ops.conv2d(x, w, ks=3, stride=2, pad=1, bias=b))
    tg = t(lambda: ops.gemm(a, wk, bias=b))
    ti = t(im2col)
    print(f"conv s2 implicit {tc:7.1f} us | dense GEMM M={M} N={C} K={K} {tg:7.1f} us | torch im2col copy {ti:7.1f} us", flush=True)
y1 = ops.conv2d(x, w, ks=3, stride=2, pad=1, bias=b)
y2 = ops.gemm(im2col(), wk, bias=b).reshape(BT, Ho, Ho, C)
print("equal:", torch.equal(y1, y2), float((y1.float() - y2.float()).abs().max()))

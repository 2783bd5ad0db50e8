"""What each epilogue costs on the encoder GEMM shapes (product library, C ABI): the same operands
through the forward's epilogue and through reduced ones (LN fold without GELU, bias + GELU, bias only),
rounds interleaved in one process.  Tuning tool, not product code."""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib

L = _lib.lib()
dev = "cuda"
torch.manual_seed(0)
M, C = 43840, 1024
st = torch.cuda.current_stream().cuda_stream
rounds = int(os.environ.get("ROUNDS", "5"))


def row_partials(y):
    yf = y.float().view(y.shape[0], -1, 256)
    return torch.stack([yf.sum(-1), (yf * yf).sum(-1)], -1).contiguous()


def run(name, K, N, cfgs):
    x = (torch.randn(M, K, device=dev) * (2 if K == C else 0.5)).half()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    stats = row_partials(x) if K == C else None
    xf = x.float()
    mr = torch.stack([xf.mean(1), torch.rsqrt(xf.var(1, unbiased=False) + 1e-6)], 1).contiguous() if K == C else None
    cs = w.float().sum(1).contiguous()
    res = torch.randn(M, N, device=dev).half()
    so = torch.empty(M, (N + 255) // 256, 2, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    eps = {}
    for c in cfgs:
        e = _lib.Epilogue()
        e.bias = b.data_ptr(); e.rdiv = 1; e.rmod = 1
        if c.startswith("ln0"):  # finalized [M, 2] (mean, rstd)
            e.ln_stats = mr.data_ptr(); e.ln_colsum = cs.data_ptr(); e.ln_parts = 0; e.ln_eps = 1e-6
        elif "ln" in c:  # [M, 4, 2] partial sums, as the forward
            e.ln_stats = stats.data_ptr(); e.ln_colsum = cs.data_ptr(); e.ln_parts = 4; e.ln_eps = 1e-6
        if "gelu" in c:
            e.act = _lib.ACT_GELU
        if "res" in c:
            e.res = y.data_ptr(); e.ldres = N
        if "stats" in c:
            e.stats_out = so.data_ptr()
        eps[c] = e
    call = lambda e: L.vda_gemm(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), N, M, N, K, ctypes.byref(e), st)
    for c in cfgs:
        y.copy_(res)
        assert call(eps[c]) == 0, L.vda_last_error()
    torch.cuda.synchronize()
    times = {c: [] for c in cfgs}
    for _ in range(rounds):
        for c in cfgs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                call(eps[c])
            e1.record()
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / 10 * 1e3)
    fl = 2.0 * M * N * K
    print(f"{name:5s} N={N} K={K}: " + " | ".join(f"{c}: {statistics.median(t):6.1f}us {fl / statistics.median(t) / 1e6:6.1f}TF"
                                                for c, t in times.items()), flush=True)


run("fc1", C, 4 * C, ["ln+gelu", "ln0+gelu", "ln", "ln0", "gelu", "bias"])
run("qkv", C, 3 * C, ["ln", "ln0", "bias"])
run("proj", C, C, ["res+stats", "res", "bias"])
run("fc2", 4 * C, C, ["res+stats", "res", "bias"])

"""In-process A/B of the encoder GEMMs across libvda builds (tuning tool, not product code).

usage: python tools/ab_gemm.py LIB_A.so [LIB_B.so[@tile=N] ...] [--rounds R] [--shapes qkv,proj,fc1,fc2,patch] [--m M]

Each library is loaded through ctypes and called through the C ABI (vda_gemm) on the current torch
stream with the forward's exact epilogues (LN fold from [M, 4, 2] partials for qkv / fc1, residual +
row statistics for proj / fc2).  `--m` changes the token count (default 43,840 = the forward's; e.g.
32,768 makes proj / fc2 exactly two rounds of 256x256 tiles on 256 CUs).  Rounds alternate the libraries (one process, one device), and every
output is compared bit-for-bit against the first library's.
"""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib

args = sys.argv[1:]
rounds, shapes, M = 7, ["qkv", "proj", "fc1", "fc2"], 43840
libs = []
i = 0
while i < len(args):
    if args[i] == "--rounds":
        rounds = int(args[i + 1]); i += 2
    elif args[i] == "--m":
        M = int(args[i + 1]); i += 2
    elif args[i] == "--shapes":
        shapes = args[i + 1].split(","); i += 2
    else:
        libs.append(args[i]); i += 1
L = []
for k, p in enumerate(libs):
    path, _, opt = p.partition("@")
    if opt:  # LIB@tile=N: a private copy of a tuning build with vda_debug_force_tile(N)
        import shutil, tempfile
        cp = os.path.join(tempfile.mkdtemp(), "libvda.so")
        shutil.copy(path, cp)
        path = cp
    l = ctypes.CDLL(os.path.abspath(path))
    _lib._declare(l)
    if opt:
        key, _, val = opt.partition("=")
        assert key == "tile", opt
        l.vda_debug_force_tile(int(val))
    L.append(l)

dev = "cuda"
torch.manual_seed(0)
C = 1024
tok = (torch.randn(M, C, device=dev) * 2).half()
st = torch.cuda.current_stream().cuda_stream


def row_partials(y):  # [M, N] fp16 -> [M, ceil(N/256), 2] (sum, sumsq) fp32, as the proj/fc2 epilogues write
    yf = y.float().view(y.shape[0], -1, 256)
    return torch.stack([yf.sum(-1), (yf * yf).sum(-1)], -1).contiguous()


def mk(name):
    if name == "patch":  # the patch embed: K 588 -> 640, per-token fp32 row bias (pos embed + bias)
        K, N, ntok = 640, C, 1370
        x = (torch.randn(M, K, device=dev)).half()
        w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        rb = torch.randn(ntok, N, device=dev)
        e = _lib.Epilogue()
        e.rowbias = rb.data_ptr(); e.rdiv = 1; e.rmod = ntok
        y = torch.empty(M, N, device=dev, dtype=torch.float16)
        return dict(x=x, w=w, y=y, e=e, K=K, N=N, keep=[x, w, rb], res=None, ldy=N)
    if name == "ff1":  # a motion module's GEGLU feed-forward (the [h | g] interleaved W, N/2 outputs)
        K, N = C, 8 * C
        x = tok
        w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        b = torch.randn(N, device=dev) * 0.1
        e = _lib.Epilogue()
        e.bias = b.data_ptr(); e.rdiv = 1; e.rmod = 1; e.act = _lib.ACT_GEGLU
        y = torch.empty(M, N // 2, device=dev, dtype=torch.float16)
        return dict(x=x, w=w, y=y, e=e, K=K, N=N, keep=[x, w, b], res=None, ldy=N // 2)
    K, N = (C, 3 * C) if name == "qkv" else (C, C) if name == "proj" else (C, 4 * C) if name == "fc1" else (4 * C, C)
    x = tok if K == C else (torch.randn(M, K, device=dev) * 0.5).half()
    w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    e = _lib.Epilogue()
    e.bias = b.data_ptr(); e.rdiv = 1; e.rmod = 1
    keep = [x, w, b]
    res = None
    if name in ("qkv", "fc1"):
        stats = row_partials(x)
        cs = w.float().sum(1).contiguous()
        keep += [stats, cs]
        e.ln_stats = stats.data_ptr(); e.ln_colsum = cs.data_ptr(); e.ln_parts = 4; e.ln_eps = 1e-6
        e.act = _lib.ACT_GELU if name == "fc1" else _lib.ACT_NONE
    else:
        res = torch.randn(M, N, device=dev).half()
        so = torch.empty(M, (N + 255) // 256, 2, device=dev)
        keep += [res, so]
        e.res = res.data_ptr(); e.ldres = N; e.stats_out = so.data_ptr()
    y = torch.empty(M, N, device=dev, dtype=torch.float16)
    return dict(x=x, w=w, y=y, e=e, K=K, N=N, keep=keep, res=res, ldy=N)


for name in shapes:
    s = mk(name)
    outs = []
    for l in L:
        if s["res"] is not None:
            s["y"].copy_(s["res"]); s["e"].res = s["y"].data_ptr()  # in place, like the encoder
        rc = l.vda_gemm(s["x"].data_ptr(), s["K"], s["w"].data_ptr(), s["y"].data_ptr(), s["ldy"], M, s["N"], s["K"],
                        ctypes.byref(s["e"]), st)
        assert rc == 0, l.vda_last_error()
        torch.cuda.synchronize()
        outs.append(s["y"].clone())
    same = [bool(torch.equal(outs[0], o)) or f"rel {float((o.float() - outs[0].float()).abs().sum() / outs[0].float().abs().sum()):.1e}"
            for o in outs[1:]]
    times = [[] for _ in L]
    n = 10
    for r in range(rounds):
        for li, l in enumerate(L):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                l.vda_gemm(s["x"].data_ptr(), s["K"], s["w"].data_ptr(), s["y"].data_ptr(), s["ldy"], M, s["N"], s["K"],
                           ctypes.byref(s["e"]), st)
            e1.record()
            torch.cuda.synchronize()
            times[li].append(e0.elapsed_time(e1) / n * 1e3)
    fl = 2.0 * M * s["N"] * s["K"]
    line = f"{name:5s} M={M} N={s['N']} K={s['K']}: "
    line += " | ".join(f"{(os.path.basename(os.path.dirname(p.partition('@')[0])) or p) + p.partition('@')[2]}: med {statistics.median(t):7.1f}us min {min(t):7.1f}us "
                       f"{fl / statistics.median(t) / 1e6:6.1f}TF" for p, t in zip(libs, times))
    print(line + f" | bit-identical {same}", flush=True)

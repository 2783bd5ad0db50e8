"""GEMM structure lab driver (tuning tool): the lab kernels (build/lab/liblab.so, tools/gemm_lab/lab.hip)
beside the product's phased GEMM (ops.gemm, bias-only epilogue) on the encoder shapes, random data,
one process, alternating rounds; each output is checked against torch fp32.

usage: python tools/gemm_lab/run_lab.py [--variants 0,2,3] [--shapes qkv,proj,fc1,fc2] [--rounds 5] [--m 43840]
"""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from vda_amd import ops

args = sys.argv[1:]
opt = {"--variants": "0,2,3", "--shapes": "qkv,proj,fc1,fc2", "--rounds": "5", "--m": "43840", "--reps": "10",
       "--lib": "build/lab/liblab.so"}
for i in range(0, len(args), 2):
    opt[args[i]] = args[i + 1]
variants = [int(v) for v in opt["--variants"].split(",") if v != ""]
M, rounds, reps = int(opt["--m"]), int(opt["--rounds"]), int(opt["--reps"])
lab = ctypes.CDLL(os.path.abspath(opt["--lib"]))
lab.lab_gemm.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
lab.lab_gemm.restype = ctypes.c_int
dev = "cuda"
SH = {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096), "sq8k": (8192, 8192)}


def timeit(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


for name in opt["--shapes"].split(","):
    N, K = SH[name]
    m = M if name != "sq8k" else 8192
    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.rand(m, K, device=dev, generator=g) * 2 - 1).half()
    w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * K ** -0.5).half()
    b = torch.randn(N, device=dev) * 0.1
    ref = torch.addmm(b, x.float(), w.float().t())
    outs = {"prod": torch.empty(m, N, device=dev, dtype=torch.float16)}
    fns = {"prod": lambda: ops.gemm(x, w, bias=b, out=outs["prod"])}
    st = torch.cuda.current_stream().cuda_stream
    for v in variants:
        y = torch.empty(m, N, device=dev, dtype=torch.float16)
        outs[f"v{v}"] = y
        fns[f"v{v}"] = (lambda v=v, y=y: lab.lab_gemm(v, x.data_ptr(), w.data_ptr(), y.data_ptr(), b.data_ptr(), m, N, K, 0,
                                                      st))
    for k, f in fns.items():
        rc = f()
        if isinstance(rc, int) and rc != 0:
            raise SystemExit(f"{k}: lab_gemm rc {rc}")
    torch.cuda.synchronize()
    errs = {k: ((o.float() - ref).abs().sum() / ref.abs().sum()).item() for k, o in outs.items()}
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            times[k].append(timeit(f))
    flop = 2.0 * m * N * K
    line = [f"{name:5s} M={m} N={N} K={K}:"]
    for k in fns:
        med = statistics.median(times[k])
        line.append(f"{k} {med:7.1f}us {flop / med / 1e6:6.0f}TF err {errs[k]:.1e}")
    print(" | ".join(line), flush=True)

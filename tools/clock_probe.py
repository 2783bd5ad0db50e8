"""In-kernel shader clock of the encoder fc1 GEMM, the spatial attention and two probe kernels
(tuning tool, not product code; MI355X_MICROARCH.md 'DVFS give-back' item 6).

usage: bash tools/build_ts.sh && hipcc ... tools/clock_probe.hip (see tools/clock_probe.sh)
       python tools/clock_probe.py build/ts/libvda.so build/probe/libclockprobe.so [seconds]

Each kernel runs back to back on random data for `seconds` (default 2.5) so the chip reaches its
steady clock under that load; the LAST launch's per-block stamps (s_memtime = shader cycles,
s_memrealtime = 100 MHz ticks, at block start and end) give the clock every block held:
d(memtime) / d(realtime) x 100 MHz.  Printed: median / p10 / p90 over blocks, the launch time, and
for the GEMM the TF/s at that clock against the 2.5 PF peak rated at 2.4 GHz.
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from vda_amd import _lib

L = ctypes.CDLL(os.path.abspath(sys.argv[1]))
_lib._declare(L)
P = ctypes.CDLL(os.path.abspath(sys.argv[2]))
secs = float(sys.argv[3]) if len(sys.argv) > 3 else 2.5
out_json = sys.argv[4] if len(sys.argv) > 4 else None  # optional: the medians as JSON (profiles/<round>_clock_probe.json)
summary = {"method": "median over blocks of d(s_memtime) / d(s_memrealtime) x 100 MHz, last launch after back-to-back "
                     "launches on random data (tools/clock_probe.py, -DVDA_TS build)"}
for f in (L.vda_debug_clock_stamps, L.vda_debug_attn_clock_stamps):
    f.argtypes = [ctypes.c_void_p]
P.probe_mfma_only.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
P.probe_dma_only.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
dev = "cuda"
st = torch.cuda.current_stream().cuda_stream
cus = torch.cuda.get_device_properties(0).multi_processor_count


def run(name, launch, read, nblocks, flop=None, key=None):
    """launch() back to back for `secs`, then read the last launch's stamps."""
    launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n, t0 = 0, time.perf_counter()
    e0.record()
    while time.perf_counter() - t0 < secs:
        for _ in range(8):
            launch()
        n += 8
        torch.cuda.synchronize()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    ts = read()[:nblocks].astype(np.float64)
    dc, dr = ts[:, 2] - ts[:, 0], ts[:, 3] - ts[:, 1]
    ok = dr > 0
    ghz = dc[ok] / dr[ok] * 0.1  # 100 MHz ticks -> GHz
    span_us = (ts[:, 3].max() - ts[:, 1].min()) / 100.0
    line = (f"{name}: {n} launches, {us:8.1f} us each (events), last launch span {span_us:8.1f} us; in-kernel clock "
            f"median {np.median(ghz):.3f} GHz (p10 {np.percentile(ghz, 10):.3f}, p90 {np.percentile(ghz, 90):.3f}, "
            f"{ok.sum()} blocks)")
    if flop:
        tf = flop / us / 1e6
        line += (f"; {tf:7.1f} TF/s = {tf / 2500:.3f} of 2.5 PF, {tf / (2500 * np.median(ghz) / 2.4):.3f} of the "
                 f"peak at that clock")
    print(line, flush=True)
    if key:
        summary[key + "_clock_ghz"] = round(float(np.median(ghz)), 3)
        summary[key + "_us"] = round(us, 1)


torch.manual_seed(0)
# fc1 as the forward runs it: LN fold (statistics of the producer), GELU, M = 43,840 (ViT-L 32 x 518^2)
M, C = 43840, 1024
N, K = 4 * C, C
x = (torch.randn(M, K, device=dev) * 2).half()
w = (torch.randn(N, K, device=dev) * K ** -0.5).half()
b = torch.randn(N, device=dev) * 0.1
xf = x.float().view(M, -1, 256)
stats = torch.stack([xf.sum(-1), (xf * xf).sum(-1)], -1).contiguous()
cs = w.float().sum(1).contiguous()
y = torch.empty(M, N, device=dev, dtype=torch.float16)
e = _lib.Epilogue()
e.bias = b.data_ptr(); e.rdiv = 1; e.rmod = 1
e.ln_stats = stats.data_ptr(); e.ln_colsum = cs.data_ptr(); e.ln_parts = 4; e.ln_eps = 1e-6
e.act = _lib.ACT_GELU


def gemm():
    assert L.vda_gemm(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), N, M, N, K, ctypes.byref(e), st) == 0


def read_gemm():
    buf = np.zeros((1024, 4), dtype=np.uint64)
    assert L.vda_debug_clock_stamps(ctypes.c_void_p(buf.ctypes.data)) == 0
    return buf


run("fc1 GEMM (LN fold + GELU) 43840x4096x1024", gemm, read_gemm, cus, 2.0 * M * N * K, key="fc1")

B, Nt, H, D = 32, 1370, 16, 64
qkv = (torch.randn(B * Nt, 3 * H * D, device=dev) * 1.5).half()
ao = torch.empty(B * Nt, H * D, device=dev, dtype=torch.float16)


def attn():
    assert L.vda_spatial_attention(qkv.data_ptr(), ao.data_ptr(), B, Nt, H, D, D ** -0.5, st) == 0


def read_attn():
    buf = np.zeros((8192, 4), dtype=np.uint64)
    assert L.vda_debug_attn_clock_stamps(ctypes.c_void_p(buf.ctypes.data)) == 0
    return buf


nqb = (Nt + 127) // 128
run("spatial attention 32x1370x16x64", attn, read_attn, min(8192, B * H * nqb), 4.0 * B * H * Nt * Nt * D,
    key="spatial_attention")

ts = torch.zeros(cus * 4, dtype=torch.int64, device=dev)
src = (torch.randn(64 << 20, device=dev)).half()  # 128 MiB of random fp16
sink = torch.empty(cus * 512, device=dev)
iters = 4096


def mfma():
    assert P.probe_mfma_only(src.data_ptr(), sink.data_ptr(), ts.data_ptr(), cus, iters, st) == 0


def read_probe():
    return ts.view(cus, 4).cpu().numpy().astype(np.uint64)


# 8 waves x 8 MFMAs (16x16x32, 16 cycles each on one SIMD) per iteration
run("probe: MFMA only (8 waves/CU, operands in registers)", mfma, read_probe, cus, 2.0 * 16 * 16 * 32 * 8 * 8 * iters * cus,
    key="mfma_only_probe")
steps = 2048
src_bytes = 64 << 20


def dma():
    assert P.probe_dma_only(src.data_ptr(), src_bytes, ts.data_ptr(), cus, steps, st) == 0


run("probe: LDS-DMA staging only (64 KiB per step, 2-slot ring)", dma, read_probe, cus, key="dma_only_probe")
print(f"(dma probe: {steps} steps x 64 KiB per CU per launch)", flush=True)
if out_json:
    import json
    json.dump(summary, open(out_json, "w"), indent=1)

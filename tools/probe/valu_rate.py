"""Drive tools/probe/valu_rate.hip: shader cycles per wave64 instruction per SIMD for v_exp_f32 / v_add_f32 /
v_fma_f32 / v_cvt_pk_f16_f32 at 1, 2, 4 and 8 waves per SIMD (one block per CU).  Tuning tool.
usage: python tools/probe/valu_rate.py build/probe/libvalurate.so"""
import ctypes
import sys

import torch

P = ctypes.CDLL(sys.argv[1])
P.probe_rate.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 3
cus = torch.cuda.get_device_properties(0).multi_processor_count
iters = 256
names = ["v_exp_f32", "v_add_f32", "v_fma_f32", "v_cvt_pk_f16_f32"]
for op, name in enumerate(names):
    for wps in (1, 2, 4):
        threads = 64 * 4 * wps  # 4 SIMDs per CU
        if threads > 1024:
            threads = 1024
        out = torch.empty(cus * threads, device="cuda")
        cyc = torch.zeros(cus, dtype=torch.int64, device="cuda")
        for _ in range(2):
            assert P.probe_rate(op, cus, threads, iters, out.data_ptr(), cyc.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        c = float(cyc.float().median())
        n_per_simd = iters * 16 * 8 * (threads // 64) / 4  # wave-instructions per SIMD
        print(f"{name:18s} {threads // 256} waves/SIMD: {c / n_per_simd:6.2f} cycles per wave instruction per SIMD", flush=True)

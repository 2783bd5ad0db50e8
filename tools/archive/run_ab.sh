#!/bin/bash
# GEMM register epilogues: op tests, A/B vs round-2 kernel, full-size parity, bench
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/ab_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_gemm.py build/base/libvda.so video-depth-anything_amd/libvda.so --rounds 7 > gpurun_out/ab_gemm.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/ab_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_model.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/ab_full.log 2>&1; rc=$?; grep -E "rel|passed|failed" gpurun_out/ab_full.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/ab_bench.log 2>&1 && tail -1 gpurun_out/ab_bench.log | cut -c1-250

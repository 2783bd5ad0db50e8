#!/bin/bash
# validation of the current tree: -m gpu suite, smoke, bench line, GEMM A/B vs the round-2 library
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/v3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/v3_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/v3_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/v3_bench.log 2>&1 || exit 1
tail -1 gpurun_out/v3_bench.log | cut -c1-300
timeout -k 10 300 python tools/ab_gemm.py build/base/libvda.so video-depth-anything_amd/libvda.so --rounds 5 > gpurun_out/v3_gemm.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/v3_gemm.log

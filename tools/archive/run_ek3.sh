#!/bin/bash
# motion-module LN fold: op tests, full-size + model parity, bench
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -s --timeout 120 --timeout-method thread -k "rowbias or layernorm_fold or row_stats" > gpurun_out/ek3.log 2>&1; rc=$?; grep -E "rel-L1|passed|failed|Error" gpurun_out/ek3.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_model.py tests/test_stream.py tests/test_video.py -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/ek3_full.log 2>&1; rc=$?; grep -E "rel|passed|failed" gpurun_out/ek3_full.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/ek3_bench.log 2>&1 && tail -1 gpurun_out/ek3_bench.log | cut -c1-200

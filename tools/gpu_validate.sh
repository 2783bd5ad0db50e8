#!/bin/bash
# Round-end validation on the GPU box: the whole -m gpu suite, the default bench line, the video bench
# and smoke(), each step under its own time limit (results under gpurun_out/val_*).
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/val_tests.log 2>&1; rc=$?; tail -3 gpurun_out/val_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/val_bench.log 2>&1 && tail -1 gpurun_out/val_bench.log | cut -c1-400 &&
timeout -k 10 300 python bench.py --video --steps 3 --warmup 1 > gpurun_out/val_video.log 2>&1 && tail -1 gpurun_out/val_video.log | cut -c1-250 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"

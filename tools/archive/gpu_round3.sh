#!/bin/bash
# Round-3 validation + evidence on the GPU box: the -m gpu suite, smoke(), then tools/refresh_profiles.sh
# (bench line, rocprof kernel stats, forward trace, PMC passes) and the video bench.
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/val_tests.log 2>&1; rc=$?; tail -3 gpurun_out/val_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/val_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/val_smoke.log
bash tools/refresh_profiles.sh || exit 1
timeout -k 10 300 python bench.py --video --steps 3 --warmup 1 > gpurun_out/val_video.log 2>&1 && tail -1 gpurun_out/val_video.log | cut -c1-250

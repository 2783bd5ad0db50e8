#!/bin/bash
# Per-kernel timeline of one forward (quick A/B evidence):  bash tools/prof_quick.sh <tag> [bench args]
set -o pipefail
tag=${1:-q}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run \
  -- python3 bench.py --steps 4 --warmup 2 --cpu-baseline-frames 0 --no-probe "$@" > gpurun_out/prof_${tag}_bench.log 2>&1 || exit 1
python3 tools/trace_forward.py gpurun_out/prof_$tag/run_kernel_trace.csv > gpurun_out/prof_${tag}_fwd.txt || exit 1
grep -A40 "forward wall" gpurun_out/prof_${tag}_fwd.txt

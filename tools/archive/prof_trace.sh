#!/bin/bash
# rocprofv3 kernel trace of one-clip-in-flight forwards + per-dispatch timeline (gpurun_out/pt_*)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pt_stats -o run \
  -- python3 bench.py --streams 1 --steps 6 --warmup 2 --cpu-baseline-frames 0 > gpurun_out/pt_bench.log 2>&1 || exit 1
python3 tools/trace_forward.py gpurun_out/pt_stats/run_kernel_trace.csv > gpurun_out/pt_fwd.txt || exit 1
sed -n '/forward wall/,$p' gpurun_out/pt_fwd.txt | head -16

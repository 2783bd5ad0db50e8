#!/bin/bash
# Config 5 (ViT-L 32 x 518 x 924) evidence: bench line, rocprof kernel stats + forward trace (one clip
# in flight), MFMA-busy PMC per kernel class.  Outputs gpurun_out/c5_*.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python3 bench.py --size 518 924 --steps 20 --warmup 4 --cpu-baseline-frames 0 > gpurun_out/c5_bench.log 2>&1 || exit 1
tail -1 gpurun_out/c5_bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_stats -o run \
  -- python3 bench.py --size 518 924 --streams 1 --steps 6 --warmup 2 --cpu-baseline-frames 0 > gpurun_out/c5_rocprof_bench.log 2>&1 || exit 1
python3 tools/trace_forward.py gpurun_out/c5_stats/run_kernel_trace.csv > gpurun_out/c5_fwd.txt || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/c5_pmc \
  -o run -- python3 tools/pmc_forward.py 2 518 924 > gpurun_out/c5_pmc.log 2>&1 || exit 1
python3 tools/pmc_mfma_summary.py gpurun_out/c5_pmc/run_counter_collection.csv gpurun_out/c5_pmc_mfma.json | tail -3

#!/bin/bash
# Round-end evidence (run on the GPU box from the repo root):
#   gpurun_out/prof_bench.log        bench.py default JSON line (roofline + cpu_baseline)
#   gpurun_out/prof_stats/           rocprofv3 --kernel-trace --stats of the bench with one clip in flight
#                                    (--streams 1: per-launch kernel durations without the second clip's
#                                    kernels sharing the CUs, as the default line's single-stream probe pass)
#   gpurun_out/prof_fwd.txt          per-dispatch timeline of one forward (tools/trace_forward.py)
#   gpurun_out/pmc_fetch, pmc_write  FETCH_SIZE / WRITE_SIZE passes on the fc1 GEMM (separate runs)
#   gpurun_out/pmc_fc1.json          gfx950-corrected HBM bytes per fc1 launch (tools/pmc_summary.py)
#   gpurun_out/pmc_conv.json         the same for the 148^2 refinenet 3x3 conv (hconv) + its L2 hit rate
#   gpurun_out/pmc_mfma.json         MFMA-busy fraction + clock per kernel class over two forwards
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/prof_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run \
  -- python3 bench.py --streams 1 --steps 10 --warmup 3 --cpu-baseline-frames 0 > gpurun_out/prof_rocprof_bench.log 2>&1 || exit 1
python3 tools/trace_forward.py gpurun_out/prof_stats/run_kernel_trace.csv > gpurun_out/prof_fwd.txt || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run \
  -- python3 tools/pmc_fc1.py 5 > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run \
  -- python3 tools/pmc_fc1.py 5 > gpurun_out/pmc_write.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_fetch/run_counter_collection.csv \
  gpurun_out/pmc_write/run_counter_collection.csv "gemm256" gpurun_out/pmc_fc1.json || exit 1
bash tools/pmc_conv.sh || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma \
  -o run -- python3 tools/pmc_forward.py 2 > gpurun_out/pmc_mfma.log 2>&1 || exit 1
python3 tools/pmc_mfma_summary.py gpurun_out/pmc_mfma/run_counter_collection.csv gpurun_out/pmc_mfma.json || exit 1
tail -1 gpurun_out/prof_bench.log

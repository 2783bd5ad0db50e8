#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes (separate runs) on the 148^2 refinenet 3x3 conv
# (tools/pmc_conv.py) -> gpurun_out/pmc_conv.json.  Run on the GPU box from the repo root.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:hit"; do
  ctr=${pass%%:*}; d=${pass##*:}
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmcc_$d -o run \
    -- python3 tools/pmc_conv.py 5 > gpurun_out/pmcc_$d.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmcc_fetch/run_counter_collection.csv gpurun_out/pmcc_write/run_counter_collection.csv \
  "hconv" gpurun_out/pmc_conv.json $(( (3 * 32 * 148 * 148 * 256 + 9 * 256 * 256) * 2 )) gpurun_out/pmcc_hit/run_counter_collection.csv

#!/bin/bash
# Same-box A/B of the whole forward: bench.py of the round-2 tree (build/r02tree, a git worktree of the
# round-2 commit built in place) against the current tree, alternating, two rounds each.
set -o pipefail
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  (cd $R/build/r02tree && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-frames 0 > $R/gpurun_out/abf_r02_$i.log 2>&1) || exit 1
  tail -1 $R/gpurun_out/abf_r02_$i.log | cut -c1-200
  (cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-frames 0 > $R/gpurun_out/abf_r03_$i.log 2>&1) || exit 1
  tail -1 $R/gpurun_out/abf_r03_$i.log | cut -c1-200
done

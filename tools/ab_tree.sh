#!/bin/bash
# Same-box A/B of the whole forward: bench.py of a base tree (a git worktree built in place, path given
# relative to the repo root) against the current tree, alternating, two rounds each.
# usage: tools/ab_tree.sh build/basetree
set -o pipefail
R=$GRAFT_REPO_ROOT
B=$R/$1
for i in 1 2; do
  (cd $B && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-frames 0 > $R/gpurun_out/abt_base_$i.log 2>&1) || exit 1
  echo "base: $(tail -1 $R/gpurun_out/abt_base_$i.log | cut -c1-120)"
  (cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-frames 0 > $R/gpurun_out/abt_cur_$i.log 2>&1) || exit 1
  echo "cur:  $(tail -1 $R/gpurun_out/abt_cur_$i.log | cut -c1-120)"
done

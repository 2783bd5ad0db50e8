#!/bin/bash
# In-situ A/B of two libvda builds: rocprofv3 kernel stats of the ViT-L bench forward, ROUNDS
# alternations, per-kernel totals side by side (tools/ab_summary.py).  "old" = LIB_A, "new" = LIB_B.
# usage: tools/ab_libs.sh ROUNDS LIB_A LIB_B [bench args]
R=$1; A=$2; B=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for i in $(seq 1 $R); do
  for tag in old new; do
    L=$A; [ $tag = new ] && L=$B
    VDA_LIB_OVERRIDE=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_${tag}_$i -o run --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --no-probe --cpu-baseline-frames 0 "$@" > gpurun_out/ab_${tag}_$i.log 2>&1 || exit 1
  done
done
python3 tools/ab_summary.py $R

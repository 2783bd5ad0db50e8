#!/bin/bash
# In-situ A/B of tuning env settings on the in-tree lib: rocprof kernel stats of the bench forward
# under env A ("old") and env B ("new").  usage: tools/ab_env.sh ROUNDS "ENV_A" "ENV_B"
R=$1; A=$2; B=$3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for i in $(seq 1 $R); do
  for tag in old new; do
    E=$A; [ $tag = new ] && E=$B
    env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_${tag}_$i -o run --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --no-probe --cpu-baseline-frames 0 > gpurun_out/ab_${tag}_$i.log 2>&1 || exit 1
  done
done
python3 tools/ab_summary.py $R

#!/bin/bash
# In-situ A/B: rocprofv3 kernel stats of the ViT-L bench forward with build/old/libvda.so vs the
# in-tree lib, ROUNDS alternations; prints per-kernel average durations side by side.
# usage: tools/ab_prof.sh ROUNDS [bench args]
R=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for i in $(seq 1 $R); do
  for tag in old new; do
    L=build/old/libvda.so; [ $tag = new ] && L=video-depth-anything_amd/libvda.so
    VDA_LIB_OVERRIDE=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_${tag}_$i -o run --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --no-probe --cpu-baseline-frames 0 "$@" > gpurun_out/ab_${tag}_$i.log 2>&1 || exit 1
  done
done
python3 tools/ab_summary.py $R

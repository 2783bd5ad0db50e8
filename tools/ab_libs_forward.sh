#!/bin/bash
# Same-box A/B of the whole forward (bench.py, two clips in flight) across libvda builds: each argument is a
# directory holding a libvda.so (e.g. build/var/<name> from build_variants.sh, or video-depth-anything_amd for
# the product); a libvda_torch.so linked against it is created next to it when missing (build it on the CPU
# side beforehand: tools/ab_libs_forward.sh --link DIR ...).  Alternates the builds, two rounds each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$1" == "--link" ]; then
  shift
  TD=$(python3 -c "import os, torch; print(os.path.dirname(torch.__file__))")
  for d in "$@"; do
    [ -f $d/libvda_torch.so ] || g++ build/vda_torch.o -o $d/libvda_torch.so -shared -L $TD/lib -lc10 -lc10_hip \
      -ltorch_cpu -ltorch_hip -ltorch -L $d -lvda -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$TD/lib
  done
  exit 0
fi
for i in 1 2; do
  for d in "$@"; do
    n=$(basename $d)
    (cd $R && VDA_LIB_OVERRIDE=$R/$d/libvda.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 \
      --cpu-baseline-frames 0 > $R/gpurun_out/abl_${n}_$i.log 2>&1) || exit 1
    echo "$n: $(tail -1 $R/gpurun_out/abl_${n}_$i.log | cut -c1-110)"
  done
done

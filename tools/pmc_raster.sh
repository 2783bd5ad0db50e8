#!/bin/bash
# fc1's HBM read traffic by XCD tile raster (verdict r5 item 4): FETCH_SIZE and the L2 hit rate of the
# LN-folded fc1 GEMM (tools/pmc_fc1.py) for the product library (GROUP_M 8) and the GROUP_M variants
# built by tools/build_variants.sh (build/var/gm*/), each pass its own rocprofv3 run; then the in-process
# timing A/B of the same libraries (tools/ab_gemm.py, fc1 shape, bit-identity checked).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
libs="prod:video-depth-anything_amd/libvda.so"
for v in "$@"; do libs="$libs $v:build/var/$v/libvda.so"; done
for spec in $libs; do
  name=${spec%%:*}; lib=${spec#*:}
  if [ "$name" = prod ]; then unset VDA_LIB_OVERRIDE; else export VDA_LIB_OVERRIDE=$PWD/$lib; fi
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/raster_$name/fetch -o run \
    -- python3 tools/pmc_fc1.py 5 > gpurun_out/raster_$name.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/raster_$name/hit -o run \
    -- python3 tools/pmc_fc1.py 5 >> gpurun_out/raster_$name.log 2>&1 || exit 1
done
unset VDA_LIB_OVERRIDE
python3 - "$@" <<'PY'
import csv, re, statistics, sys
def per(path, counter):
    v = {}
    for r in csv.DictReader(open(path)):
        if re.search("gemm256", r.get("Kernel_Name", "")) and r.get("Counter_Name") == counter:
            v[r["Dispatch_Id"]] = v.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return statistics.median(v.values())
for name in ["prod"] + sys.argv[1:]:
    d = f"gpurun_out/raster_{name}"
    f = per(f"{d}/fetch/run_counter_collection.csv", "FETCH_SIZE")
    h, m = per(f"{d}/hit/run_counter_collection.csv", "TCC_HIT_sum"), per(f"{d}/hit/run_counter_collection.csv", "TCC_MISS_sum")
    print(f"{name}: FETCH {2 * f / 1024:.1f} MB per fc1 launch (x2 gfx950 correction; X + W = 98.0 MB), "
          f"L2 hit rate {h / (h + m):.3f}")
PY
args=""
for v in "$@"; do args="$args build/var/$v/libvda.so"; done
timeout -k 10 200 python3 tools/ab_gemm.py video-depth-anything_amd/libvda.so $args --shapes fc1,qkv --rounds 5

#!/bin/bash
# L2 hit rate / fabric reads of one GEMM shape: rocprofv3 --pmc passes (counters only, no traces).
# usage: tools/pmc_l2.sh TAG M N K [act]
TAG=$1; shift
i=0
for C in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum" "TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C -d gpurun_out/l2_${TAG}_$i -o run --output-format csv -- python3 tools/pmc_gemm.py "$@" > gpurun_out/l2_${TAG}_$i.log 2>&1 || exit 1
done
python3 - "$TAG" <<'PY'
import csv, glob, sys, statistics, re
tag = sys.argv[1]
tot = {}
for f in glob.glob(f"gpurun_out/l2_{tag}_*/run_counter_collection.csv"):
    per = {}
    for r in csv.DictReader(open(f)):
        if "gemm" not in r["Kernel_Name"]: continue
        per.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, v in per.items(): tot[k] = statistics.median(v.values())
print(tag, {k: f"{v:.4g}" for k, v in sorted(tot.items())})
h, m = tot.get("TCC_HIT_sum", 0), tot.get("TCC_MISS_sum", 1)
print(f"{tag}: L2 hit rate {h/(h+m):.3f}; EA rdreq {tot.get('TCC_EA0_RDREQ_sum',0)*128/1e6:.1f} MB (x128B); TCP->TCC reqs {tot.get('TCP_TCC_READ_REQ_sum',0):.4g}")
PY

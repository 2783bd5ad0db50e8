"""Median per-dispatch PMC values of the kernels whose name contains a pattern (tuning tool).
usage: python tools/pmc_kernel_summary.py <counter_collection.csv> <name-substring>"""
import csv
import statistics
import sys

per = {}
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] not in r.get("Kernel_Name", ""):
        continue
    d = per.setdefault(r["Dispatch_Id"], {})
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
keys = sorted(set().union(*per.values())) if per else []
med = {k: statistics.median(d.get(k, 0.0) for d in per.values()) for k in keys}
print(f"{len(per)} dispatches of *{sys.argv[2]}*")
for k in keys:
    print(f"  {k:32s} {med[k]:16.0f}")
wc = med.get("SQ_WAVE_CYCLES")
if wc:
    for k in keys:
        if k.startswith("SQ_WAIT") or k.startswith("SQ_ACTIVE") or k == "SQ_LDS_BANK_CONFLICT":
            print(f"  {k} / SQ_WAVE_CYCLES = {med[k] / wc:.3f}")

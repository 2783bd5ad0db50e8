"""Summarise rocprofv3 --pmc CSVs for one kernel into profiles/<round>_pmc_<kernel>.json.
usage: pmc_summary.py fetch.csv write.csv kernel_regex out.json [algorithmic_bytes [hit_miss.csv]]
(default algorithmic bytes: the ViT-L fc1 launch, X + W + Y)."""
import csv, json, sys, glob, statistics
fetch_csv, write_csv, name_re, out = sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4]
import re
def per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if re.search(name_re, r.get("Kernel_Name", "")) and r.get("Counter_Name") == counter:
            vals.setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())
f = per_dispatch(fetch_csv, "FETCH_SIZE")
w = per_dispatch(write_csv, "WRITE_SIZE")
fk, wk = statistics.median(f), statistics.median(w)
res = {"kernel_regex": name_re, "dispatches": [len(f), len(w)], "FETCH_SIZE_kB_median": fk, "WRITE_SIZE_kB_median": wk,
       "correction": "gfx950: FETCH_SIZE counts half the bytes of 16-B/lane streaming reads -> x2 (MI355X_MICROARCH.md §HBM)",
       "hbm_bytes_per_launch": int((2 * fk + wk) * 1024),
       "algorithmic_bytes_per_launch": int(sys.argv[5]) if len(sys.argv) > 5 else (43840 * 1024 + 4096 * 1024 + 43840 * 4096) * 2}
res["hbm_over_algorithmic"] = round(res["hbm_bytes_per_launch"] / res["algorithmic_bytes_per_launch"], 3)
if len(sys.argv) > 6:  # L2 (TCC) hit rate of the same kernel, from a TCC_HIT / TCC_MISS pass
    hit, miss = statistics.median(per_dispatch(sys.argv[6], "TCC_HIT_sum")), statistics.median(per_dispatch(sys.argv[6], "TCC_MISS_sum"))
    res.update({"TCC_HIT_median": hit, "TCC_MISS_median": miss, "l2_hit_rate": round(hit / max(hit + miss, 1.0), 4)})
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))

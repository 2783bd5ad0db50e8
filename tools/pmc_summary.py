"""Summarise rocprofv3 --pmc CSVs for one kernel into profiles/<round>_pmc_fc1.json."""
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
       "algorithmic_bytes_per_launch": (43840 * 1024 + 4096 * 1024 + 43840 * 4096) * 2}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))

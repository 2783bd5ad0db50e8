"""Per-dispatch timeline of ONE clip forward from a rocprofv3 --kernel-trace CSV (diagnostic).

usage: python tools/trace_forward.py <kernel_trace.csv> [n_forwards_in_trace]
Prints each dispatch of the last forward (name, grid, duration) and per-kernel-class totals."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nfw = int(sys.argv[2]) if len(sys.argv) > 2 else 1
# forwards are delimited by the patch-embed im2col dispatch
starts = [i for i, r in enumerate(rows) if "im2col" in r["Kernel_Name"] and "conv_im2col" not in r["Kernel_Name"]]
s0 = starts[-1]
s1 = len(rows)
tot = defaultdict(float)
t_first = int(rows[s0]["Start_Timestamp"])
t_last = int(rows[s1 - 1]["End_Timestamp"])
for r in rows[s0:s1]:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\(.*", "", name)[:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[name] += d
    g = f'{r.get("Grid_Size_X", r.get("Grid_Size", "?"))}'
    print(f"{d:9.1f} us  grid {g:>9}  {name}")
print(f"\nforward wall {(t_last - t_first) / 1e3:.1f} us, kernel sum {sum(tot.values()):.1f} us")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{v:9.1f} us  {k}")

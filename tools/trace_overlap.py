"""Concurrency of a two-clips-in-flight bench from a rocprofv3 --kernel-trace CSV (diagnostic).

usage: python tools/trace_overlap.py <kernel_trace.csv> [skip_first_ms]
Over the trace after the first skip_first_ms (warm-up): the wall time, the sum of kernel durations,
the time with 0 / 1 / 2+ kernels running, and per kernel class the average duration when it ran
alone vs beside another kernel (how much the second clip stretches each class)."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
iv = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    iv.append((s, e, re.sub(r"\(.*", "", name)[:60]))
iv.sort()
t0 = iv[0][0] + skip * 1e6
iv = [x for x in iv if x[0] >= t0]
t_end = max(e for _, e, _ in iv)
ev = sorted([(s, 1) for s, _, _ in iv] + [(e, -1) for _, e, _ in iv])
level, last, busy = 0, iv[0][0], defaultdict(float)
for t, d in ev:
    busy[min(level, 2)] += t - last
    level += d
    last = t
wall = t_end - iv[0][0]
ksum = sum(e - s for s, e, _ in iv)
print(f"wall {wall / 1e6:.2f} ms, kernel sum {ksum / 1e6:.2f} ms, idle {busy[0] / 1e6:.2f} ms, "
      f"one kernel {busy[1] / 1e6:.2f} ms, two or more {busy[2] / 1e6:.2f} ms")
# per class: duration alone vs overlapped (overlap = another kernel active during > 50 % of it)
starts = [s for s, _, _ in iv]
alone, shared = defaultdict(list), defaultdict(list)
for i, (s, e, n) in enumerate(iv):
    ov = 0
    for j in range(max(0, i - 40), min(len(iv), i + 40)):
        if j == i:
            continue
        s2, e2, _ = iv[j]
        ov += max(0, min(e, e2) - max(s, s2))
    (shared if ov > 0.5 * (e - s) else alone)[n].append((e - s) / 1e3)
tot = defaultdict(float)
for s, e, n in iv:
    tot[n] += (e - s) / 1e3
for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:14]:
    a, b = alone[n], shared[n]
    fa = f"{sum(a) / len(a):8.1f} us alone (n={len(a)})" if a else " " * 22
    fb = f"{sum(b) / len(b):8.1f} us shared (n={len(b)})" if b else ""
    print(f"{t / 1e3:8.2f} ms  {fa}  {fb}  {n}")

"""Side-by-side per-kernel totals (ms per forward) from tools/ab_prof.sh runs."""
import csv, sys, re, collections
R = int(sys.argv[1])
def load(tag):
    agg = collections.defaultdict(list)
    for i in range(1, R + 1):
        tot = collections.Counter(); calls = collections.Counter()
        for r in csv.DictReader(open(f"gpurun_out/ab_{tag}_{i}/run_kernel_stats.csv")):
            n = re.sub(r"\(anonymous namespace\)::", "", r["Name"])[:70]
            tot[n] += float(r["TotalDurationNs"]); calls[n] += int(r["Calls"])
        for n in tot: agg[n].append((tot[n], calls[n]))
    return agg
old, new = load("old"), load("new")
fwd = 4  # 1 warmup + 3 steps
rows = []
for n in set(old) | set(new):
    o = min(t for t, _ in old.get(n, [(0, 0)])) / fwd / 1e6
    w = min(t for t, _ in new.get(n, [(0, 0)])) / fwd / 1e6
    rows.append((max(o, w), n, o, w))
rows.sort(reverse=True)
so = sum(r[2] for r in rows); sn = sum(r[3] for r in rows)
print(f"{'kernel':70s} {'old ms':>8s} {'new ms':>8s}")
for _, n, o, w in rows[:18]:
    print(f"{n:70s} {o:8.3f} {w:8.3f}")
print(f"{'TOTAL':70s} {so:8.3f} {sn:8.3f}")

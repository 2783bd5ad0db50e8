"""Same-process A/B of the clips-in-flight stream setup on the bench workload (tuning tool, not product code):
two streams at the default priority vs one high-priority + one normal stream, and 2 vs 3 streams with mixed
priorities.  usage: python tools/ab_stream_prio.py [--rounds R] [--steps K]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd

args = sys.argv[1:]
rounds = int(args[args.index("--rounds") + 1]) if "--rounds" in args else 4
steps = int(args[args.index("--steps") + 1]) if "--steps" in args else 20
dev = torch.device("cuda", 0)
m = vda_amd.build_model("vitl", device=dev)
x = torch.randn(1, 32, 3, 518, 518, generator=torch.Generator().manual_seed(1000)).to(dev)
m.prepare(dev, (518, 518))
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
setups = {
    "2 streams, default priority": [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)],
    "2 streams, one high priority": [torch.cuda.Stream(device=dev, priority=hi), torch.cuda.Stream(device=dev)],
}
print(f"stream priority range (low, high) = ({lo}, {hi})", flush=True)
res = {k: [] for k in setups}
for r in range(rounds):
    for name, strs in setups.items():
        for st in strs:
            st.wait_stream(torch.cuda.current_stream(dev))
        for i in range(3):
            with torch.cuda.stream(strs[i % len(strs)]):
                m(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            with torch.cuda.stream(strs[i % len(strs)]):
                m(x)
        torch.cuda.synchronize()
        fps = steps * 32 / (time.perf_counter() - t0)
        res[name].append(fps)
        print(f"round {r} {name}: {fps:.2f} frames/s", flush=True)
for name in setups:
    print(f"{name}: median {statistics.median(res[name]):.2f} frames/s", flush=True)

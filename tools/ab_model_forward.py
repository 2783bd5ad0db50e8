"""Same-process A/B of a model schedule switch on the whole forward (tuning tool, not product code).

usage: python tools/ab_model_forward.py ATTR [--rounds R] [--steps K]
Builds the ViT-L model once (synthetic weights) and times bench.py's workload (1x32x3x518x518, two
clips in flight on two HIP streams, K steps after 3 warm-up steps) with ``model.ATTR`` False and True,
alternating R rounds; prints frames/s per round and the medians, and checks the depths agree.
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd

attr = sys.argv[1]
args = sys.argv[2:]
rounds = int(args[args.index("--rounds") + 1]) if "--rounds" in args else 4
steps = int(args[args.index("--steps") + 1]) if "--steps" in args else 20
dev = torch.device("cuda", 0)
m = vda_amd.build_model("vitl", device=dev)
x = torch.randn(1, 32, 3, 518, 518, generator=torch.Generator().manual_seed(1000)).to(dev)
m.prepare(dev, (518, 518))
strs = [torch.cuda.Stream(device=dev) for _ in range(2)]
res = {False: [], True: []}
outs = {}
for r in range(rounds):
    for val in (False, True):
        setattr(m, attr, val)
        for st in strs:
            st.wait_stream(torch.cuda.current_stream(dev))
        for i in range(3):
            with torch.cuda.stream(strs[i % 2]):
                m(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            with torch.cuda.stream(strs[i % 2]):
                d = m(x)
        torch.cuda.synchronize()
        fps = steps * 32 / (time.perf_counter() - t0)
        res[val].append(fps)
        outs[val] = d.float()
        print(f"round {r} {attr}={val}: {fps:.2f} frames/s", flush=True)
rel = float((outs[True] - outs[False]).abs().sum() / outs[False].abs().sum())
print(f"{attr}: False median {statistics.median(res[False]):.2f}, True median {statistics.median(res[True]):.2f} frames/s; "
      f"depth rel-L1 between the two {rel:.2e}", flush=True)

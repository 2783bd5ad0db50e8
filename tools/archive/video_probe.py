"""Where the time of bench.py --video goes on one GPU: the whole infer_video_depth job vs its
forwards alone, the host stitch, and the per-window host<->device plumbing (wall clock, synced).
STREAMS=k sets infer_video_depth(streams=k)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import vda_amd
from vda_amd import video as V
dev = torch.device("cuda")
model = vda_amd.build_model("vitl", device=dev)
n = 176
frames = np.random.default_rng(0).integers(0, 256, (n, 518, 518, 3), dtype=np.uint8)
x = torch.randn(1, 32, 3, 518, 518, device=dev)
with torch.no_grad():
    for _ in range(3):
        model(x)
torch.cuda.synchronize()

def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(); t = time.perf_counter(); r = fn(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    return min(ts) * 1e3, r

kw = dict(input_size=518, device=dev)
if os.environ.get("STREAMS"):
    kw["streams"] = int(os.environ["STREAMS"])
V.infer_video_depth(model, frames, 30, **kw)
t_job, (depth, _) = timed(lambda: V.infer_video_depth(model, frames, 30, **kw))
with torch.no_grad():
    t_fwd, _ = timed(lambda: [model(x) for _ in range(8)])
orig = V.stitch
st = []
def stitch_t(dl, nn):
    t = time.perf_counter(); r = orig(dl, nn); st.append(time.perf_counter() - t); return r
V.stitch = stitch_t
V.infer_video_depth(model, frames, 30, **kw)
V.stitch = orig
t_h2d, _ = timed(lambda: torch.from_numpy(frames[:32]).to(dev))
pre = V.DeviceIO.preprocess(torch.from_numpy(frames[:32]).to(dev), (518, 518))
t_pre, _ = timed(lambda: V.DeviceIO.preprocess(torch.from_numpy(frames[:32]).to(dev), (518, 518)))
d = torch.randn(32, 518, 518, device=dev)
t_rs, _ = timed(lambda: V.DeviceIO.resize_depth(d, (518, 518)))
print(f"job {t_job:.1f} ms = {n / t_job * 1e3:.1f} video fps; 8 forwards {t_fwd:.1f} ms; stitch {(st[0] * 1e3 if st else float('nan')):.1f} ms (nan: incremental); "
      f"per window: H2D of 32 frames {t_h2d:.2f} ms, H2D+preprocess {t_pre:.2f} ms, depth resize {t_rs:.2f} ms")

"""Where the video job's time beyond its forwards goes (tuning tool): the 176-frame ViT-L job vs the
same 8 forwards on two streams back to back, the host stitch per window, and the tail after the
last forward is enqueued."""
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
strs = [torch.cuda.Stream(device=dev) for _ in range(2)]
with torch.no_grad():
    for _ in range(3):
        model(x)
torch.cuda.synchronize()
for st in strs:
    st.wait_stream(torch.cuda.current_stream())


def fwd8():
    with torch.no_grad():
        for i in range(8):
            with torch.cuda.stream(strs[i % 2]):
                model(x)
    for st in strs:
        torch.cuda.current_stream().wait_stream(st)


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(); t = time.perf_counter(); fn(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t)
    return min(ts) * 1e3


adds, puts, res = [], [], []
oadd, oput, ores = V.Stitcher.add, V._HostSink.put, V._HostSink.result
def add(self, win):
    t = time.perf_counter(); oadd(self, win); adds.append(time.perf_counter() - t)
def put(self, k, d):
    t = time.perf_counter(); oput(self, k, d); puts.append(time.perf_counter() - t)
def result(self):
    t = time.perf_counter(); r = ores(self); res.append(time.perf_counter() - t); return r
V.infer_video_depth(model, frames, 30, input_size=518, device=dev)
t_job = timed(lambda: V.infer_video_depth(model, frames, 30, input_size=518, device=dev))
t_f8 = timed(fwd8)
V.Stitcher.add, V._HostSink.put, V._HostSink.result = add, put, result
torch.cuda.synchronize(); t0 = time.perf_counter()
V.infer_video_depth(model, frames, 30, input_size=518, device=dev)
torch.cuda.synchronize(); t_inst = (time.perf_counter() - t0) * 1e3
print(f"job {t_job:.1f} ms ({n / t_job * 1e3:.1f} video fps); 8 forwards on 2 streams {t_f8:.1f} ms; "
      f"instrumented job {t_inst:.1f} ms: Stitcher.add {' '.join(f'{a * 1e3:.1f}' for a in adds)} ms, "
      f"put {' '.join(f'{p * 1e3:.1f}' for p in puts)} ms, result() {res[0] * 1e3:.1f} ms", flush=True)

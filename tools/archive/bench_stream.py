"""Streaming-mode throughput (video_depth.py:91-327 infere_single_image): per-frame cost of one
forward_single_image step on ViT-L at 518x518 with a 31-frame context and alignment rows, and the
whole driver on a synthetic uint8 video (preprocess + store + alignment included).  Diagnostic."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import vda_amd

enc = sys.argv[1] if len(sys.argv) > 1 else "vitl"
m = vda_amd.build_model(enc, device="cuda")
g = torch.Generator().manual_seed(0)
T = 32
ctx = m.get_motion_features(torch.randn(T - 1, 3, 518, 518, generator=g).cuda())
x = torch.randn(1, 1, 3, 518, 518, generator=g).cuda()
for pred in (None, [0, 30, 20]):
    for _ in range(3):
        m.forward_single_image(x, ctx, pred, T)
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        d, _ = m.forward_single_image(x, ctx, None if pred is None else list(pred), T)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"{enc} forward_single_image 518x518, context {T - 1}, pred_idx {pred}: {dt * 1e3:.2f} ms/frame "
          f"({1 / dt:.1f} frames/s)", flush=True)
# whole driver: 80-frame 480x640 video, keyframes [2, 12] with alignment
fr = (np.random.default_rng(0).random((80, 480, 640, 3)) * 255).astype(np.uint8)
m.infere_single_image(fr[:40], 24, keyframe_list=[2, 12])
torch.cuda.synchronize()
t0 = time.perf_counter()
d, _ = m.infere_single_image(fr, 24, keyframe_list=[2, 12])
dt = time.perf_counter() - t0
print(f"{enc} infere_single_image 80 frames 480x640 (net 518x686): {dt:.2f} s, {len(d)} depth frames, "
      f"{len(fr) / dt:.1f} input frames/s", flush=True)

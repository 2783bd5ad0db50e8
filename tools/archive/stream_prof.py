import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, vda_amd
m = vda_amd.build_model("vitl", device="cuda")
g = torch.Generator().manual_seed(0)
ctx = m.get_motion_features(torch.randn(31, 3, 518, 518, generator=g).cuda())
x = torch.randn(1, 1, 3, 518, 518, generator=g).cuda()
for _ in range(3): m.forward_single_image(x, ctx, None, 32)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10): m.forward_single_image(x, ctx, None, 32)
torch.cuda.synchronize()
print("ms/frame", (time.perf_counter() - t0) / 10 * 1e3)

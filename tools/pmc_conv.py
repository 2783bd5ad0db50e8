"""Run the refinenet residual conv unit's 3x3 conv of ViT-L 32x518x518 as the forward runs it
(32 x 148 x 148 x 256 -> 256, pre-ReLU, bias, + residual; the hconv kernel) a few times: the PMC
subject for the conv traffic summary (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT,TCC_MISS in
separate passes, tools/refresh_profiles.sh -> profiles/<round>_pmc_conv.json)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops
BT, H, W, C = 32, 148, 148, 256
x = torch.randn(BT, H, W, C, device="cuda", dtype=torch.float16)
w = (torch.randn(C, 3, 3, C, device="cuda") * (9 * C) ** -0.5).half()
b = torch.randn(C, device="cuda") * 0.1
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    y = ops.conv2d(x, w, bias=b, pre_relu=True, res=x)
torch.cuda.synchronize()
print("alg bytes per launch", (3 * BT * H * W * C + 9 * C * C) * 2)

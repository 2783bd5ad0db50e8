"""Debug: which statistics each output element of groupnorm_linear used (identity W) (tuning tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import ops
dev = "cuda"
torch.manual_seed(0)
Fr, S, C = 3, 12, 256
f = torch.arange(Fr, device=dev).view(Fr, 1, 1).float()
c = torch.arange(C, device=dev).view(1, 1, C).float()
x = (10 * f + 0.25 * (c // 8) + 0.01 * torch.randn(Fr, S, C, device=dev)).reshape(-1, C).half()
g = torch.ones(C, device=dev)
b = torch.zeros(C, device=dev)
w = torch.eye(C, device=dev).half()
yf = ops.groupnorm_linear(x, g, b, Fr, 32, 1e-6, w).float()
yc = ops.groupnorm(x, g, b, Fr, 32, 1e-6).float()
torch.set_printoptions(precision=1, linewidth=250, sci_mode=False)
d = (yf - yc).view(-1, 32, 8).mean(-1)  # per row, per group
print("rows x groups: mean abs diff of the group's 8 channels (fused - reference)")
for r in range(Fr * S):
    print(r, d[r].abs().max().item(), (d[r].abs() > 0.5).nonzero().flatten().tolist()[:12])

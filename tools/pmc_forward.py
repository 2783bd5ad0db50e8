"""PMC subject: two ViT-L 1x32x3xHxW clip forwards (bench.py's workload, synthetic weights).
usage: python tools/pmc_forward.py [n_forwards] [H W]   (default 2, 518 518; config 5 = 518 924)

Run under `rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE` and summarise with
tools/pmc_mfma_summary.py (MFMA-busy fraction and in-kernel clock per kernel class)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import vda_amd
dev = torch.device("cuda", 0)
m = vda_amd.build_model("vitl", device=dev)
H, W = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (518, 518)
x = torch.randn(1, 32, 3, H, W, generator=torch.Generator().manual_seed(1000)).to(dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    d = m(x)
torch.cuda.synchronize()
print("depth", tuple(d.shape), float(d.float().mean()))

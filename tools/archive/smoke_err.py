import os, sys
REPO = os.environ.get("TREE", os.getcwd())
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "oracle"))
import torch, vda_amd, vda_oracle
from vda_amd import _lib
L = _lib.lib()
dev = torch.device("cuda", 0)
m = vda_amd.build_model("vits", device=dev)
g = torch.Generator().manual_seed(0)
x = torch.randn(1, 4, 3, 70, 98, generator=g)
sd = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
ref = vda_oracle.forward(sd, "vits", x)
def run(tag):
    d = m(x.to(dev)).float().cpu()
    print(f"{tag}: rel-L1 {vda_oracle.rel_l1(d, ref):.3e}", flush=True)
run("default")
if hasattr(L, "vda_debug_strip_split"):
    L.vda_debug_strip_split(1); run("strip split 1"); L.vda_debug_strip_split(0)
L.vda_debug_force_tile(-2); run("no strip"); L.vda_debug_force_tile(-1)
# fp32 x through an fp16 autocast-like CPU run of the oracle is not available; report the fp32 forward too
d32 = m(x.to(dev), fp32=True).float().cpu()
print(f"fp32 mode: rel-L1 {vda_oracle.rel_l1(d32, ref):.3e}")

"""Strip-conv split count A/B through the tuning build (tuning tool, not product code).

usage: python tools/ab_strip_split.py [--rounds R]
The 37^2 / 19^2 (and 518x924: 37x66 / 19x33) 3x3 convs with 256 outputs (layer3_rn, layer4_rn: Cin 1024;
RCU at 19^2: Cin 256) of a 32-frame clip, timed with every split count the kernel accepts (vda_debug_strip_split) against the
automatic choice; outputs compared with the unsplit result (the split sums fp32 partials in another
order: close, not bit-identical).
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from tunelib import tune_lib

rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
T = tune_lib()
torch.manual_seed(0)
for name, BT, H, W, Cin in [("layer3_rn", 32, 37, 37, 1024), ("layer4_rn", 32, 19, 19, 1024), ("rcu19", 32, 19, 19, 256),
                            ("layer3_rn_924", 32, 37, 66, 1024), ("layer4_rn_924", 32, 19, 33, 1024),
                            ("rcu19_924", 32, 19, 33, 256)]:
    x = (torch.randn(BT, H, W, Cin, device="cuda") * 0.5).half()
    w = (torch.randn(256, 3, 3, Cin, device="cuda") * (9 * Cin) ** -0.5).half()
    res = {}
    for s in (0, 1, 2, 4, 8):
        with T.route(force_tile=-3, strip_split=s):
            try:
                y = T.conv2d(x, w)
            except RuntimeError as e:
                print(f"{name} split {s}: {e}")
                continue
            times = []
            for _ in range(rounds):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    T.conv2d(x, w)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / 10 * 1e3)
        res[s] = (statistics.median(times), y)
    y1 = res[1][1].float()
    for s, (t, y) in res.items():
        err = float((y.float() - y1).abs().sum() / y1.abs().sum())
        print(f"{name}: split {'auto' if s == 0 else s}: {t:7.1f} us  rel vs unsplit {err:.2e}", flush=True)

"""Generate golden fixtures from the REFERENCE implementation (build container only).

Runs FriedFeid/Video-Depth-Anything's own ``VideoDepthAnything.forward`` (read-only at
/root/reference, imported with three tiny sys.modules shims for easydict / cv2 / torchvision that
the model path only touches at import time) on the synthetic weight recipe of
``vda_amd.weights`` and seeded inputs, fp32 on CPU, and writes small ``.npz`` fixtures:

    x        input clip [B, T, 3, H, W] (fp16-representable values, stored as float16)
    depth    reference depth [B, T, H, W] float32
    tap_stats  per encoder tap: (mean, std, abs-mean) of the normalised patch tokens

plus ``state_dict_keys_<enc>.json`` (every reference key with its shape).  Nothing from the
reference is copied into the repo: only these input/output vectors.  The GPU box never runs this.

    python tests/golden/make_golden.py
"""
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

CASES = [
    # name, encoder, B, T, H, W, skip_tmp_block
    ("vits_t8_126", "vits", 1, 8, 126, 126, False),
    ("vits_t8_126_skip", "vits", 1, 8, 126, 126, True),
    ("vits_t4_70x126", "vits", 1, 4, 70, 126, False),
    ("vits_t1_518", "vits", 1, 1, 518, 518, False),
    ("vitl_t4_70", "vitl", 1, 4, 70, 70, False),
    ("vitl_t3_84x56_b2", "vitl", 2, 3, 84, 56, False),
]
CONFIGS = {  # run.py:74-77
    "vits": dict(encoder="vits", features=64, out_channels=[48, 96, 192, 384]),
    "vitl": dict(encoder="vitl", features=256, out_channels=[256, 512, 1024, 1024]),
}


def import_reference():
    sys.path.insert(0, REF)
    ed = types.ModuleType("easydict"); ed.EasyDict = dict; sys.modules["easydict"] = ed
    cv2 = types.ModuleType("cv2"); cv2.INTER_CUBIC, cv2.INTER_AREA, cv2.INTER_NEAREST = 2, 3, 0
    sys.modules["cv2"] = cv2
    tv = types.ModuleType("torchvision"); tvt = types.ModuleType("torchvision.transforms")

    class Compose:
        def __init__(self, t): self.t = t
        def __call__(self, x):
            for f in self.t: x = f(x)
            return x
    tvt.Compose = Compose; tv.transforms = tvt
    sys.modules["torchvision"] = tv; sys.modules["torchvision.transforms"] = tvt
    from video_depth_anything.video_depth import VideoDepthAnything
    return VideoDepthAnything


def main():
    sys.path.insert(0, REPO)
    import vda_amd.weights as W
    VDA = import_reference()
    torch.set_num_threads(8)
    models = {}
    for enc in ("vits", "vitl"):
        torch.manual_seed(0)
        m = VDA(**CONFIGS[enc]).eval()
        keys = [(k, list(v.shape)) for k, v in m.state_dict().items()]
        with open(os.path.join(HERE, f"state_dict_keys_{enc}.json"), "w") as f:
            json.dump(keys, f)
        sd = W.synthetic_state_dict((k, tuple(s)) for k, s in keys)
        m.load_state_dict(sd, strict=True)
        models[enc] = m
    for name, enc, B, T, H, Wd, skip in CASES:
        m = models[enc]
        g = torch.Generator().manual_seed(1234 + T * 7 + H)
        x = torch.randn(B, T, 3, H, Wd, generator=g).half().float()  # fp16-exact, stored as fp16
        taps = []
        with torch.no_grad():
            feats = m.pretrained.get_intermediate_layers(x.flatten(0, 1), m.intermediate_layer_idx[enc],
                                                         return_class_token=True)
            for f, _cls in feats:
                taps.append([float(f.mean()), float(f.std()), float(f.abs().mean())])
            d = m(x, skip_tmp_block=skip)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), x=x.half().numpy(), depth=d.numpy().astype(np.float32),
                            tap_stats=np.array(taps, dtype=np.float64),
                            meta=np.array(json.dumps(dict(encoder=enc, B=B, T=T, H=H, W=Wd, skip_tmp_block=skip))))
        print(name, tuple(d.shape), float(d.mean()), float(d.min()), float(d.max()), flush=True)


if __name__ == "__main__":
    main()

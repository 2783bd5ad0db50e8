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

    def resize(img, dsize, interpolation=None):
        # stand-in for cv2.resize(INTER_CUBIC) used only by the video case: torch bicubic
        # (a = -0.75, the same kernel); the windowing/stitching logic is what that case pins.
        w, h = dsize
        t = torch.from_numpy(np.ascontiguousarray(img, dtype=np.float32)).permute(2, 0, 1)[None]
        t = torch.nn.functional.interpolate(t, size=(h, w), mode="bicubic", align_corners=False)
        return t[0].permute(1, 2, 0).numpy()
    cv2.resize = resize
    sys.modules["cv2"] = cv2
    tq = types.ModuleType("tqdm"); tq.tqdm = lambda it, *a, **k: it; sys.modules.setdefault("tqdm", tq)
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
    # long-video windowing + stitching (video_depth.py:329-417): 57 frames -> 3 windows
    g = torch.Generator().manual_seed(99)
    base = torch.rand(1, 3, 8, 10, generator=g)
    frames = []
    for t in range(57):  # a smoothly drifting synthetic scene, uint8 RGB 48x64
        f = torch.nn.functional.interpolate(torch.roll(base, shifts=t // 6, dims=3), size=(48, 64), mode="bilinear",
                                            align_corners=False)
        frames.append((f[0].permute(1, 2, 0) * 255).clamp(0, 255).to(torch.uint8).numpy())
    frames = np.stack(frames)
    with torch.no_grad():
        depth, fps = models["vits"].infer_video_depth(frames, 24, input_size=56, device="cpu", fp32=True)
    np.savez_compressed(os.path.join(HERE, "video_vits_57f.npz"), frames=frames, depth=depth.astype(np.float32),
                        meta=np.array(json.dumps(dict(encoder="vits", input_size=56, fps=fps))))
    print("video_vits_57f", depth.shape, float(depth.mean()), flush=True)


if __name__ == "__main__":
    main()

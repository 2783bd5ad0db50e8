"""Golden fixture for the pe='rope' motion-module variant, generated from the REFERENCE (container only).

``VideoDepthAnything(..., pe='rope')`` (video_depth.py:36-45 -> dpt_temporal.py:30-40 ->
motion_module.py:238-242, 290-293; attention.py:403-429) on the synthetic vits weights of
``vda_amd.weights`` over its own key list (the rope tree has no ``pos_encoder.pe`` buffers), fp32 on
CPU, with the import shims of ``make_golden.py``.  Writes ``vits_t8_126_rope.npz`` (x, depth, meta) and
``state_dict_keys_vits_rope.json``.

    python tests/golden/make_rope_golden.py
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)


def main():
    import make_golden as MG
    import vda_amd.weights as W
    VDA = MG.import_reference()
    torch.set_num_threads(8)
    torch.manual_seed(0)
    m = VDA(**MG.CONFIGS["vits"], pe="rope").eval()
    keys = [(k, list(v.shape)) for k, v in m.state_dict().items()]
    with open(os.path.join(HERE, "state_dict_keys_vits_rope.json"), "w") as f:
        json.dump(keys, f)
    m.load_state_dict(W.synthetic_state_dict((k, tuple(s)) for k, s in keys), strict=True)
    g = torch.Generator().manual_seed(4321)
    x = torch.randn(1, 8, 3, 126, 126, generator=g).half().float()
    with torch.no_grad():
        d = m(x)
    np.savez_compressed(os.path.join(HERE, "vits_t8_126_rope.npz"), x=x.half().numpy(), depth=d.numpy().astype(np.float32),
                        tap_stats=np.zeros((4, 3)),
                        meta=np.array(json.dumps(dict(encoder="vits", B=1, T=8, H=126, W=126, skip_tmp_block=False,
                                                      pe="rope"))))
    print("vits_t8_126_rope", tuple(d.shape), float(d.mean()))


if __name__ == "__main__":
    main()

"""Golden fixture for the non-default head options, generated from the REFERENCE (container only).

``VideoDepthAnything(**vits, use_bn=True, use_clstoken=True)``: BatchNorm after each ResidualConvUnit
conv (util/blocks.py:60-62, :79-85, eval mode) and the cls-token readout projections (dpt.py:92-98,
:129-132), on the synthetic weights of ``vda_amd.weights`` over the tree's own keys, fp32 CPU, with the
import shims of ``make_golden.py``.  Writes ``vits_t4_70x98_bn_cls.npz`` and
``state_dict_keys_vits_bn_cls.json``.

    python tests/golden/make_variant_golden.py
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
    m = VDA(**MG.CONFIGS["vits"], use_bn=True, use_clstoken=True).eval()
    keys = [(k, list(v.shape)) for k, v in m.state_dict().items()]
    with open(os.path.join(HERE, "state_dict_keys_vits_bn_cls.json"), "w") as f:
        json.dump(keys, f)
    m.load_state_dict(W.synthetic_state_dict((k, tuple(s)) for k, s in keys), strict=True)
    g = torch.Generator().manual_seed(777)
    x = torch.randn(1, 4, 3, 70, 98, generator=g).half().float()
    with torch.no_grad():
        d = m(x)
    np.savez_compressed(os.path.join(HERE, "vits_t4_70x98_bn_cls.npz"), x=x.half().numpy(),
                        depth=d.numpy().astype(np.float32), tap_stats=np.zeros((4, 3)),
                        meta=np.array(json.dumps(dict(encoder="vits", B=1, T=4, H=70, W=98, skip_tmp_block=False,
                                                      use_bn=True, use_clstoken=True))))
    print("vits_t4_70x98_bn_cls", tuple(d.shape), float(d.mean()))


if __name__ == "__main__":
    main()

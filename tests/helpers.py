"""Shared test helpers: golden loading, the synthetic-recipe state_dict, the oracle import."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
if REPO not in sys.path:
    sys.path.insert(0, REPO)
ORACLE_DIR = os.path.join(REPO, "oracle")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)

import vda_oracle  # noqa: E402  (test infrastructure only)
import vda_amd  # noqa: E402
from vda_amd.weights import synthetic_state_dict  # noqa: E402

GOLDEN_CASES = ["vits_t8_126", "vits_t8_126_skip", "vits_t4_70x126", "vits_t1_518", "vitl_t4_70",
                "vitl_t3_84x56_b2"]


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return torch.from_numpy(z["x"].astype(np.float32)), torch.from_numpy(z["depth"]), z["tap_stats"], meta


_SD = {}


def recipe_state_dict(enc):
    if enc not in _SD:
        m = vda_amd.VideoDepthAnything.from_config(enc, device="meta")
        _SD[enc] = synthetic_state_dict((k, tuple(v.shape)) for k, v in m.state_dict().items())
    return _SD[enc]


def rel_l1(a, b):
    return vda_oracle.rel_l1(a, b)

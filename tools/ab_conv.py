"""In-process A/B of the decoder's big convs across libvda builds (tuning tool, not product code).

usage: python tools/ab_conv.py LIB_A.so[@knob=v] [LIB_B.so ...] [--rounds R] [--shapes oc1,depth,rcu148]
oc1:    output_conv1, 3x3 256 -> 128 on the x2 bilinear resize of a [32, 148, 148, 256] map (fused)
oc1u:   the same through the materialised resize + the plain halo conv (compare with oc1: same output)
depth:  the depth tail on the [32, 296, 296, 128] output_conv1 map, resized to 518 x 518 (fused)
rcu148: refinenet1 RCU conv, 3x3 256 -> 256 at 148^2 with pre-ReLU + ReLU
rcu148r: the RCU's second conv (pre-ReLU, bias, + residual)
rcu74 / l2rn: refinenet2's RCU conv1 / layer2_rn (512 -> 256) at 74^2
l3rn / l4rn: layer3_rn / layer4_rn, 3x3 1024 -> 256 (no bias) at 37^2 / 19^2 (the strip conv; 19^2 splits)
Outputs compared bit-for-bit against the first library's.
"""
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib

args = sys.argv[1:]
rounds, shapes, libs = 5, ["oc1", "depth"], []
i = 0
while i < len(args):
    if args[i] == "--rounds":
        rounds = int(args[i + 1]); i += 2
    elif args[i] == "--shapes":
        shapes = args[i + 1].split(","); i += 2
    else:
        libs.append(args[i]); i += 1
L = []
for p in libs:
    # LIB.so@name=v: a tuning-build library with vda_debug_<name>(v) set first (a copy per setting)
    path, _, knob = p.partition("@")
    l = ctypes.CDLL(os.path.abspath(path)); _lib._declare(l)
    if knob:
        fn, _, v = knob.partition("=")
        assert getattr(l, "vda_debug_" + fn)(int(v)) == 0
    L.append(l)
dev = "cuda"
torch.manual_seed(0)
st = torch.cuda.current_stream().cuda_stream


def case(name):
    if name == "oc1":
        x = (torch.randn(32, 148, 148, 256, device=dev) * 0.5).half()
        w = (torch.randn(128, 3, 3, 256, device=dev) * (9 * 256) ** -0.5).half()
        b = torch.randn(128, device=dev) * 0.1
        y = torch.empty(32, 296, 296, 128, device=dev, dtype=torch.float16)
        e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr())
        fl = 2.0 * 32 * 296 * 296 * 128 * 2304

        def run(l):
            return l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 148, 148, 256, 128, 3, 1, 1, 0, 296, 296,
                                ctypes.byref(e), None, 0, st)
        return run, y, fl, [x, w, b, e]
    if name == "oc1u":  # the unfused route: the x2 resize materialised, then the plain halo conv at 296^2
        x = (torch.randn(32, 148, 148, 256, device=dev) * 0.5).half()
        u = torch.empty(32, 296, 296, 256, device=dev, dtype=torch.float16)
        w = (torch.randn(128, 3, 3, 256, device=dev) * (9 * 256) ** -0.5).half()
        b = torch.randn(128, device=dev) * 0.1
        y = torch.empty(32, 296, 296, 128, device=dev, dtype=torch.float16)
        e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr())
        fl = 2.0 * 32 * 296 * 296 * 128 * 2304

        def run(l):
            rc = l.vda_upsample_bilinear(x.data_ptr(), u.data_ptr(), 32, 148, 148, 256, 296, 296, st)
            return rc or l.vda_conv2d(u.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 296, 296, 256, 128, 3, 1, 1, 0, 0, 0,
                                      ctypes.byref(e), None, 0, st)
        return run, y, fl, [x, u, w, b, e]
    if name == "rcu148r":  # the RCU's second conv: pre-ReLU, bias, + the block input as residual
        x = (torch.randn(32, 148, 148, 256, device=dev) * 0.5).half()
        w = (torch.randn(256, 3, 3, 256, device=dev) * (9 * 256) ** -0.5).half()
        b = torch.randn(256, device=dev) * 0.1
        r = torch.randn(32, 148, 148, 256, device=dev).half()
        y = torch.empty(32, 148, 148, 256, device=dev, dtype=torch.float16)
        e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr())
        e.res = r.data_ptr(); e.ldres = 256
        fl = 2.0 * 32 * 148 * 148 * 256 * 2304

        def run(l):
            return l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 148, 148, 256, 256, 3, 1, 1, 1, 0, 0,
                                ctypes.byref(e), None, 0, st)
        return run, y, fl, [x, w, b, r, e]
    if name in ("rcu74", "l2rn"):  # refinenet2's RCU conv1 (pre-ReLU, bias, ReLU) / layer2_rn (512 -> 256) at 74^2
        ci = 256 if name == "rcu74" else 512
        x = (torch.randn(32, 74, 74, ci, device=dev) * 0.5).half()
        w = (torch.randn(256, 3, 3, ci, device=dev) * (9 * ci) ** -0.5).half()
        b = torch.randn(256, device=dev) * 0.1
        y = torch.empty(32, 74, 74, 256, device=dev, dtype=torch.float16)
        e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr(), act=_lib.ACT_RELU if ci == 256 else 0)
        fl = 2.0 * 32 * 74 * 74 * 256 * 9 * ci

        def run(l):
            return l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 74, 74, ci, 256, 3, 1, 1, int(ci == 256), 0,
                                0, ctypes.byref(e), None, 0, st)
        return run, y, fl, [x, w, b, e]
    if name == "rcu148":
        x = (torch.randn(32, 148, 148, 256, device=dev) * 0.5).half()
        w = (torch.randn(256, 3, 3, 256, device=dev) * (9 * 256) ** -0.5).half()
        b = torch.randn(256, device=dev) * 0.1
        y = torch.empty(32, 148, 148, 256, device=dev, dtype=torch.float16)
        e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr(), act=_lib.ACT_RELU)
        fl = 2.0 * 32 * 148 * 148 * 256 * 2304

        def run(l):
            return l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, 148, 148, 256, 256, 3, 1, 1, 1, 0, 0,
                                ctypes.byref(e), None, 0, st)
        return run, y, fl, [x, w, b, e]
    if name in ("l3rn", "l4rn"):
        S = 37 if name == "l3rn" else 19
        x = (torch.randn(32, S, S, 1024, device=dev) * 0.5).half()
        w = (torch.randn(256, 3, 3, 1024, device=dev) * (9 * 1024) ** -0.5).half()
        y = torch.empty(32, S, S, 256, device=dev, dtype=torch.float16)
        e = _lib.Epilogue(rdiv=1, rmod=1)
        fl = 2.0 * 32 * S * S * 256 * 9216
        nb = max(L[0].vda_conv2d_workspace(32, S, S, 1024, 256, 3, 1, 1), 16)
        ws = torch.empty(nb, device=dev, dtype=torch.uint8)

        def run(l):
            return l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), 32, S, S, 1024, 256, 3, 1, 1, 0, 0, 0,
                                ctypes.byref(e), ws.data_ptr(), nb, st)
        return run, y, fl, [x, w, e, ws]
    x = (torch.randn(32, 296, 296, 128, device=dev) * 0.5).half()
    w32 = torch.randn(32, 3, 3, 128, device=dev) * (9 * 128) ** -0.5
    w1 = torch.cat([w32.half(), (w32 - w32.half().float()).half()], 0).contiguous()
    b1, w2, b2 = torch.randn(32, device=dev) * 0.1, torch.rand(32, device=dev) * 0.2, torch.tensor([0.05], device=dev)
    d = torch.empty(32, 518, 518, device=dev)
    fl = 2.0 * 32 * 518 * 518 * 64 * 1152

    def run(l):
        ws = l.vda_depth_head_workspace(32, 296, 296, 128, 518, 518)
        assert ws == 0, ws
        return l.vda_depth_head(x.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr(), d.data_ptr(),
                                None, 32, 296, 296, 128, 518, 518, st)
    return run, d, fl, [x, w1, b1, w2, b2]


for name in shapes:
    run, y, fl, keep = case(name)
    outs = []
    for l in L:
        assert run(l) == 0, l.vda_last_error()
        torch.cuda.synchronize()
        outs.append(y.clone())
    same = [bool(torch.equal(outs[0], o)) or f"rel {float((o.float() - outs[0].float()).abs().sum() / outs[0].float().abs().sum()):.1e}"
            for o in outs[1:]]
    times = [[] for _ in L]
    for r in range(rounds):
        for li, l in enumerate(L):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                run(l)
            e1.record()
            torch.cuda.synchronize()
            times[li].append(e0.elapsed_time(e1) / 3 * 1e3)
    line = f"{name:6s}: " + " | ".join(f"{os.path.basename(os.path.dirname(p))}: med {statistics.median(t):7.1f}us min {min(t):7.1f}us "
                                      f"{fl / statistics.median(t) / 1e6:6.1f}TF" for p, t in zip(libs, times))
    print(line + f" | bit-identical {same}", flush=True)

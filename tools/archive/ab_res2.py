"""In-process A/B of refinenet1's RCU conv2 with the upsampled skip input (vda_epilogue.res2_h/w) across
libvda builds (tuning tool): 3x3 256 -> 256 at 148^2, res = x1, res2 = a 74^2 map read through the
bilinear upsample; outputs compared bit-for-bit with the first library's and with the materialised
upsample + conv of the first library.  usage: python tools/ab_res2.py LIB_A.so [LIB_B.so ...]"""
import ctypes, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vda_amd import _lib

libs = [a for a in sys.argv[1:] if a.endswith(".so")]
L = []
for p in libs:
    l = ctypes.CDLL(os.path.abspath(p)); _lib._declare(l); L.append(l)
BT, H, W, C, Hs, Ws = 32, 148, 148, 256, 74, 74
torch.manual_seed(0)
x = (torch.randn(BT, H, W, C, device="cuda") * 0.5).half()
w = (torch.randn(C, 3, 3, C, device="cuda") * (9 * C) ** -0.5).half()
b = torch.randn(C, device="cuda") * 0.1
r1 = torch.randn(BT, H, W, C, device="cuda").half()
r2 = torch.randn(BT, Hs, Ws, C, device="cuda").half()
st = torch.cuda.current_stream().cuda_stream


def conv(l, y, res2, up):
    e = _lib.Epilogue(rdiv=1, rmod=1, bias=b.data_ptr(), res=r1.data_ptr(), ldres=C, res2=res2.data_ptr(), ldres2=C)
    if up:
        e.res2_h, e.res2_w = Hs, Ws
    rc = l.vda_conv2d(x.data_ptr(), w.data_ptr(), y.data_ptr(), BT, H, W, C, C, 3, 1, 1, 0, 0, 0, ctypes.byref(e), None, 0, st)
    assert rc == 0, l.vda_last_error()


up = torch.empty(BT, H, W, C, device="cuda", dtype=torch.float16)
assert L[0].vda_upsample_bilinear(r2.data_ptr(), up.data_ptr(), BT, Hs, Ws, C, H, W, st) == 0
ref = torch.empty(BT, H, W, C, device="cuda", dtype=torch.float16)
conv(L[0], ref, up, False)
outs = []
for l in L:
    y = torch.empty_like(ref)
    conv(l, y, r2, True)
    outs.append(y)
torch.cuda.synchronize()
print("bit-identical to materialised upsample + conv:", [bool(torch.equal(o, ref)) for o in outs], flush=True)
times = [[] for _ in L]
for _ in range(7):
    for i, l in enumerate(L):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            conv(l, outs[i], r2, True)
        e1.record(); torch.cuda.synchronize()
        times[i].append(e0.elapsed_time(e1) / 5 * 1e3)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    conv(L[0], ref, up, False)
e1.record(); torch.cuda.synchronize()
print(f"materialised res2 (same-grid epilogue) {e0.elapsed_time(e1) / 5 * 1e3:.1f} us")
for p, t in zip(libs, times):
    print(f"{p}: upsampled res2 med {statistics.median(t):.1f} us  min {min(t):.1f} us", flush=True)

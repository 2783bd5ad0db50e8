"""Timing-only variants of the depth conv (build/var/<name>/libvda.so from tools/build_variants.sh with
SRC=vda_dconv and -DDC_EXP_* flags): which part bounds it.  Calls the C ABI directly through ctypes so
the override library is the one that runs."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.manual_seed(0)
BT, H, W, C = 32, 518, 518, 128
U = (torch.randn(BT, H, W, C, device="cuda") * 0.5).half()
w1 = (torch.randn(64, 3, 3, C, device="cuda") * 0.03).half()
b1 = torch.randn(32, device="cuda"); w2 = torch.rand(32, device="cuda"); b2 = torch.zeros(1, device="cuda")
d = torch.empty(BT, H, W, device="cuda")
P = ctypes.c_void_p
for name in sys.argv[1:]:
    lib = ctypes.CDLL(os.path.abspath(f"build/var/{name}/libvda.so"))
    # depth head on an identity-size map: resize is a copy (materialised path, then the depth conv)
    ws = torch.empty(BT * H * W * C * 2, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: lib.vda_depth_head(P(U.data_ptr()), P(w1.data_ptr()), P(b1.data_ptr()), P(w2.data_ptr()), P(b2.data_ptr()),
                                   P(d.data_ptr()), P(ws.data_ptr()), BT, H, W, C, H, W, P(st))
    assert f() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(5): f()
        e1.record(); torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 5 * 1e3)
    print(f"{name}: depth head (identity resize + conv) {best:.0f} us", flush=True)

"""Same-box A/B of vda_groupnorm (the motion modules' chunked partial -> finalize -> apply chain)
between two builds of libvda (GPU; tools only):

    python tools/ab_gn.py build/var/base/libvda.so video-depth-anything_amd/libvda.so [--rounds 9]

Shapes: the forward's four GroupNorm inputs (32 frames, 32 groups); outputs checked bit-for-bit.
"""
import argparse
import ctypes
import statistics

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    libs = [ctypes.CDLL(p) for p in args.libs]
    for lib in libs:
        lib.vda_groupnorm.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int32] * 4 + [ctypes.c_float, ctypes.c_void_p,
                                                                                     ctypes.c_void_p]
        lib.vda_groupnorm.restype = ctypes.c_int
        lib.vda_groupnorm_workspace.argtypes = [ctypes.c_int32] * 4
        lib.vda_groupnorm_workspace.restype = ctypes.c_int64
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for F, S, C in [(32, 1369, 1024), (32, 361, 1024), (32, 1369, 256), (32, 5476, 256)]:
        G = 32
        x = (torch.randn(F, S, C, device=dev) * 3 + 1).half()
        gam, bet = torch.randn(C, device=dev), torch.randn(C, device=dev)
        ws = torch.empty(int(libs[0].vda_groupnorm_workspace(F, S, C, G)), device=dev)
        outs = [torch.empty_like(x) for _ in libs]
        times = [[] for _ in libs]

        def call(i):
            rc = libs[i].vda_groupnorm(x.data_ptr(), outs[i].data_ptr(), gam.data_ptr(), bet.data_ptr(), F, S, C, G,
                                       1e-5, ws.data_ptr(), ctypes.c_void_p(st.cuda_stream))
            assert rc == 0

        for r in range(args.rounds):
            for i in range(len(libs)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.iters):
                    call(i)
                e1.record(st)
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) * 1e3 / args.iters)
        same = torch.equal(outs[0], outs[1])
        line = f"F {F} S {S} C {C}:"
        for p, t in zip(args.libs, times):
            line += f" | {p.split('/')[-2]}: med {statistics.median(t):.1f}us min {min(t):.1f}us"
        print(line + f" | bit-identical [{same}]", flush=True)


if __name__ == "__main__":
    main()

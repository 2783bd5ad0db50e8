"""Same-box A/B of vda_upsample_bilinear between two builds of libvda (GPU; tools only):

    python tools/ab_upsample.py build/var/base/libvda.so video-depth-anything_amd/libvda.so [--rounds 9]

Shapes: the forward's resizes (the motion-module / fusion x2 upsamples, the depth tail's 296 -> 518) and
odd cases (a frame boundary inside a row pair, a downscale); outputs checked bit-for-bit.
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
        lib.vda_upsample_bilinear.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int32] * 6 + [ctypes.c_void_p]
        lib.vda_upsample_bilinear.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for BT, H, W, C, Ho, Wo in [(32, 19, 19, 256, 37, 37), (32, 37, 37, 256, 74, 74), (32, 74, 74, 256, 148, 148),
                                (32, 148, 148, 256, 296, 296), (32, 296, 296, 128, 518, 518), (3, 5, 7, 64, 9, 13),
                                (2, 40, 30, 64, 17, 23)]:
        x = torch.randn(BT, H, W, C, device=dev).half()
        outs = [torch.full((BT, Ho, Wo, C), float("nan"), device=dev, dtype=torch.float16) for _ in libs]
        times = [[] for _ in libs]
        for r in range(args.rounds):
            for i, lib in enumerate(libs):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.iters):
                    rc = lib.vda_upsample_bilinear(x.data_ptr(), outs[i].data_ptr(), BT, H, W, C, Ho, Wo,
                                                   ctypes.c_void_p(st.cuda_stream))
                    assert rc == 0
                e1.record(st)
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) * 1e3 / args.iters)
        same = torch.equal(outs[0], outs[1])
        line = f"{BT}x{H}x{W}x{C} -> {Ho}x{Wo}:"
        for p, t in zip(args.libs, times):
            line += f" | {p.split('/')[-2]}: med {statistics.median(t):.1f}us min {min(t):.1f}us"
        print(line + f" | bit-identical [{same}]", flush=True)


if __name__ == "__main__":
    main()

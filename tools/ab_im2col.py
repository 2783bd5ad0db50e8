"""Same-box A/B of vda_patch_im2col between two builds of libvda (GPU; tools only).

    python tools/ab_im2col.py build/var/base/libvda.so video-depth-anything_amd/libvda.so [--rounds 9]

Times each library's patch im2col on the bench's input (32 x 3 x 518 x 518 fp32 -> [32 * 1370, 640]
fp16) and on ViT-L 32x518x924, interleaved, and checks the outputs are bit-identical.
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
        lib.vda_patch_im2col.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int32] * 4 + [ctypes.c_void_p]
        lib.vda_patch_im2col.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for BT, H, W, Kp in [(32, 518, 518, 640), (32, 518, 924, 640), (2, 70, 518, 592)]:
        img = torch.randn(BT, 3, H, W, device=dev)
        np_ = (H // 14) * (W // 14)
        outs = [torch.full((BT * (1 + np_), Kp), float("nan"), device=dev, dtype=torch.float16) for _ in libs]
        times = [[] for _ in libs]
        for r in range(args.rounds):
            for i, lib in enumerate(libs):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(args.iters):
                    rc = lib.vda_patch_im2col(img.data_ptr(), outs[i].data_ptr(), BT, H, W, Kp, ctypes.c_void_p(st.cuda_stream))
                    assert rc == 0
                e1.record(st)
                torch.cuda.synchronize()
                times[i].append(e0.elapsed_time(e1) * 1e3 / args.iters)
        same = torch.equal(outs[0], outs[1])
        gb = (img.numel() * 4 + outs[0].numel() * 2) / 1e9
        line = f"{BT}x{H}x{W} Kp {Kp}:"
        for p, t in zip(args.libs, times):
            med = statistics.median(t)
            line += f" | {p.split('/')[-2]}: med {med:.1f}us min {min(t):.1f}us {gb / med * 1e6 / 1e3:.2f} TB/s"
        print(line + f" | bit-identical [{same}]", flush=True)


if __name__ == "__main__":
    main()

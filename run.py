"""Command-line driver with the reference's flags (run.py), on the MI355X path.

    python run.py --input_video clip.y4m --output_dir out --encoder vitl [--process_single_image ...]

Mirrors FriedFeid/Video-Depth-Anything run.py:27-166: loads ``checkpoints/video_depth_anything_<enc>.pth``
(``torch.load(weights_only=True)``, strict), reads the video (vda_amd.video_io: .y4m / frame stacks /
Pillow formats; decord when installed), runs ``infer_video_depth`` (or ``infere_single_image`` with
``--process_single_image``), and writes the requested outputs (npz ``depths``, float32 TIFF stack,
source / visualisation videos as .y4m, or .gif/.png/.webp via ``--vis_format``).  ``--synthetic_weights``
uses the deterministic recipe of vda_amd.weights when no checkpoint is available (this image has none).
``--fp32`` selects the fp32 kernels (the reference's autocast-off path); the default is fp16 compute.
"""
import argparse
import os
import sys
import time
from datetime import datetime

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)


def parse(argv=None):
    p = argparse.ArgumentParser(description="Video Depth Anything (MI355X)")
    p.add_argument("--device", type=str, default="cuda:0")
    p.add_argument("--input_video", type=str, required=True)
    p.add_argument("--output_dir", type=str, default="./outputs")
    p.add_argument("--process_single_image", action="store_true")
    p.add_argument("--inference_length", type=int, default=32)
    p.add_argument("--keyframe_list", type=int, nargs="+", default=[20])
    p.add_argument("--align_each_new_frame", action="store_true")
    p.add_argument("--original", action="store_true")
    p.add_argument("--skip_tmp_block", action="store_true")
    p.add_argument("--input_size", type=int, default=518)
    p.add_argument("--max_res", type=int, default=1280)
    p.add_argument("--encoder", type=str, default="vitl", choices=["vits", "vitl"])
    p.add_argument("--max_len", type=int, default=-1)
    p.add_argument("--target_fps", type=int, default=-1)
    p.add_argument("--fp32", action="store_true")
    p.add_argument("--grayscale", action="store_true")
    p.add_argument("--save_npz", action="store_true")
    p.add_argument("--save_tiff", action="store_true")
    p.add_argument("--save_orig", action="store_true")
    p.add_argument("--save_vis", action="store_true")
    p.add_argument("--save_stats", action="store_true")
    p.add_argument("--vis_format", type=str, default="y4m", choices=["y4m", "gif", "png", "webp", "mp4"])
    p.add_argument("--checkpoint", type=str, default=None)
    p.add_argument("--synthetic_weights", action="store_true")
    p.add_argument("--windows_per_batch", type=int, default=1,
                   help="windows per forward in the long-video path (2: ~3%% more frames/s on MI355X)")
    a = p.parse_args(argv)
    assert a.inference_length > len(a.keyframe_list) + 2, "Inference length to small for the number of geiven keyframes"
    return a


def main(argv=None):
    args = parse(argv)
    import vda_amd
    from vda_amd import video_io as VIO
    if not torch.cuda.is_available():
        raise RuntimeError("the MI355X path needs a GPU (there is no CPU mode)")
    dev = args.device
    if args.synthetic_weights:
        model = vda_amd.build_model(args.encoder, device=dev)
    else:
        ck = args.checkpoint or os.path.join("checkpoints", f"video_depth_anything_{args.encoder}.pth")
        sd = torch.load(ck, map_location="cpu", weights_only=True)
        model = vda_amd.build_model(args.encoder, state_dict=sd, device=dev)
    if args.save_stats:
        torch.cuda.reset_peak_memory_stats(dev)
    frames, target_fps = VIO.read_video_frames(args.input_video, args.max_len, args.target_fps, args.max_res)
    total = len(frames)
    t0 = time.time()
    if args.process_single_image:  # checked before --original, as in the reference (run.py:93-100)
        depths, fps = model.infere_single_image(frames, target_fps, device=dev, fp32=args.fp32, input_size=args.input_size,
                                                inference_length=args.inference_length, keyframe_list=args.keyframe_list,
                                                align_each_new_frame=args.align_each_new_frame, warmup=True,
                                                skip_tmp_block=args.skip_tmp_block)
    else:
        depths, fps = model.infer_video_depth(frames, target_fps, input_size=args.input_size, device=dev, fp32=args.fp32,
                                              skip_tmp_block=args.skip_tmp_block and not args.original,
                                              windows_per_batch=max(1, args.windows_per_batch))
    dur = time.time() - t0
    os.makedirs(args.output_dir, exist_ok=True)
    stem = os.path.splitext(os.path.basename(args.input_video))[0]
    name = ("Single_" if args.process_single_image else "") + f"VideoDepthAny_{args.encoder}_{stem}"
    if args.save_stats:
        lines = [f"Run: {args.encoder} {args.inference_length} {'Single Image' if args.process_single_image else ''} "
                 f"{'Align each frame' if args.align_each_new_frame else ''} keyframes {args.keyframe_list} "
                 f"{datetime.now():%Y-%m-%d %H:%M:%S}", "", "Times", "___________________________",
                 f"Runtime: {dur}", f"Processed Frames: {len(depths)}", f"Total Frames: {total}",
                 f"FPS (Processed): {len(depths) / dur}", f"Raw FPS: {total / dur}", "", "Memory",
                 "___________________________", f"GPU Memory (mb): {torch.cuda.max_memory_reserved(dev) / 2**20}", "", ""]
        with open(os.path.join(args.output_dir, "inference_log.txt"), "a") as f:
            f.write("\n".join(lines) + "\n")
    ext = "." + args.vis_format
    if args.save_orig:
        VIO.save_video(frames, os.path.join(args.output_dir, name + "_src" + ext), fps=fps)
    if args.save_vis:
        VIO.save_video(depths, os.path.join(args.output_dir, name + "_vis" + ext), fps=fps, is_depths=True,
                       grayscale=args.grayscale, spectral=not args.grayscale)
    if args.save_npz:
        VIO.save_npz(os.path.join(args.output_dir, name + "_depths.npz"), depths)
    if args.save_tiff:
        VIO.save_tiff(os.path.join(args.output_dir, name + "_depths.tiff"), depths)
    print(f"{name}: {len(depths)} depth frames from {total} input frames in {dur:.2f} s")
    return depths


if __name__ == "__main__":
    main()

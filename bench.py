"""Benchmark: depth frames/s of the Video-Depth-Anything clip forward on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--encoder vitl] [--frames 32] [--size 518 518]

A step is one ``VideoDepthAnything.forward`` of a [1, 32, 3, 518, 518] clip (BASELINE.json
configs[2]: ViT-L fp16, full HIP path) on every rank.  Multi-GPU runs are clip-parallel (one
process per GPU via torch.distributed.run, RCCL): rank 0's weights are broadcast once over
xGMI, every rank runs its own clips (no collective inside the timed loop: clips are
independent windows), the timed region is bracketed by barrier + synchronize and the MAX over
ranks is taken; value = all ranks' frames / that time ("scaling": "weak").

Extra fields:
  roofline      dominant kernel = encoder MLP fc1 GEMM + GELU (vda gemm_kernel<..., GELU>), timed
                per launch with HIP events on its launch stream inside the timed region;
                achieved = algorithmic FLOPs per launch / mean launch time vs 2.5 PFLOP/s dense
                fp16; traffic from profiles/<round>_pmc_fc1.json (rocprofv3 PMC, gfx950-corrected),
                mfma_busy_pmc from profiles/<round>_pmc_mfma.json (SQ_VALU_MFMA_BUSY_CYCLES pass)
  cpu_baseline  the oracle's fp32 PyTorch-CPU forward (oracle/vda_oracle.py), rank 0 / N=1 only,
                on a bounded sample (a 4-frame ViT-L 518x518 clip) - a reported baseline only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_FP16_TFLOPS = 2500.0  # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
REF_A100_FPS = 71.4        # README.md:52-61 ViT-L fp16 14 ms/frame on 1x A100
GFLOP_PER_FRAME = {("vitl", 518, 518): 1404.6, ("vits", 518, 518): 121.3, ("vitl", 518, 924): 2761.5}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--encoder", default="vitl")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--size", type=int, nargs=2, default=[518, 518], metavar=("H", "W"))
    ap.add_argument("--clips-per-gpu", type=int, default=1)
    ap.add_argument("--cpu-baseline-frames", type=int, default=4,
                    help="frames of the bounded CPU-oracle sample (0 disables)")
    ap.add_argument("--no-probe", action="store_true", help="skip the per-launch event probe")
    ap.add_argument("--graph", action="store_true", help="replay the forward as a captured HIP graph")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo for rehearsal)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    ndev = torch.cuda.device_count()
    local = local % max(1, ndev)  # (rehearsal with more ranks than GPUs: ranks share a device)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as tdist
        if args.backend == "nccl":
            tdist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:
            tdist.init_process_group(args.backend)

    import vda_amd
    from vda_amd import ops

    enc = args.encoder
    T, (H, W) = args.frames, args.size
    # weights: synthetic recipe (no checkpoint offline) built on rank 0 and broadcast over RCCL
    model = vda_amd.build_model(enc, device=dev)
    if dist:
        import torch.distributed as tdist
        for t in model.state_dict().values():
            if args.backend == "nccl":
                tdist.broadcast(t, src=0)
            else:  # gloo rehearsal: host copies
                c = t.detach().cpu()
                tdist.broadcast(c, src=0)
                t.copy_(c)
        model.load_state_dict(model.state_dict(), strict=True)  # drop packs; re-pack from broadcast weights
    g = torch.Generator().manual_seed(1000 + rank)
    x = torch.randn(args.clips_per_gpu, T, 3, H, W, generator=g).to(dev)

    def step():
        return model(x)

    fn = step
    if args.graph:
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out_static = step()
        fn = lambda: (graph.replay(), out_static)[1]  # noqa: E731

    for _ in range(args.warmup):
        fn()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    probe = not args.no_probe and not args.graph
    if probe:
        ops.enable_probe(["enc_fc1"])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        depth = fn()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    launches = ops.take_probe() if probe else {}
    if dist:
        cdev = dev if args.backend == "nccl" else torch.device("cpu")
        tt = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # one-off (untimed) gather of the last clip's depth to rank 0: the clip-parallel output path
        dd = depth.contiguous().to(cdev)
        lst = [torch.empty_like(dd) for _ in range(world)] if rank == 0 else None
        tdist.gather(dd, lst, dst=0)
    frames = world * args.steps * args.clips_per_gpu * T
    value = frames / elapsed
    if not bool(torch.isfinite(depth).all()):
        raise RuntimeError("non-finite depth")

    roof = None
    if launches.get("enc_fc1"):
        C = model.pretrained.embed_dim
        rec = launches["enc_fc1"]
        flop = sum(f for _, f in rec) / len(rec)          # algorithmic 2*M*N*K per launch
        ms = sum(t for t, _ in rec) / len(rec)
        M = int(round(flop / (2.0 * 4 * C * C)))
        achieved = flop / (ms * 1e-3) / 1e12
        traffic = None
        pmc = os.path.join(REPO, "profiles", "r01_pmc_fc1.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        # MFMA-busy fraction of the same kernel class from the committed PMC pass
        # (profiles/<round>_pmc_mfma.json: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * CUs * 4))
        mfma_busy = None
        pmm = os.path.join(REPO, "profiles", "r01_pmc_mfma.json")
        if os.path.exists(pmm):
            with open(pmm) as f:
                for name, e in json.load(f).get("kernels", {}).items():
                    if "gemm256_kernel<2, 2, false, 1, false>" in name:
                        mfma_busy = e.get("mfma_busy")
        roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_FP16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP16_TFLOPS, 4), "traffic": traffic, "mfma_busy_pmc": mfma_busy,
                "kernel": f"gemm256_kernel<2,2,dense,GELU> (encoder fc1) M={M} N={4 * C} K={C}",
                "flop_per_launch": flop, "avg_launch_ms": round(ms, 4), "launches": len(launches["enc_fc1"])}

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline_frames > 0:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import vda_oracle  # test infrastructure: the reported CPU baseline only
        nthr = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
        omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)  # the box's CPU share (16 per GPU)
        nthr = max(1, min(nthr, omp) if omp > 0 else min(nthr, 16))
        torch.set_num_threads(nthr)
        sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
        xs = x[:1, : args.cpu_baseline_frames].float().cpu()
        vda_oracle.forward(sd, enc, xs[:, :1, :, :84, :84])  # warm the CPU kernels
        t1 = time.perf_counter()
        vda_oracle.forward(sd, enc, xs)
        cpu_s = time.perf_counter() - t1
        cpu = {"value": round(xs.shape[1] / cpu_s, 4), "unit": "frames/s", "cores": torch.get_num_threads(),
               "kind": "port",
               "sample": f"oracle fp32 PyTorch-CPU forward of one {enc} 1x{xs.shape[1]}x3x{H}x{W} clip "
                         f"({cpu_s:.1f} s)"}

    if rank == 0:
        gflop = GFLOP_PER_FRAME.get((enc, H, W))
        line = {
            "metric": "depth frames/sec at 32x518x518, ViT-L fp16, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / REF_A100_FPS, 3) if (enc, T, H, W) == ("vitl", 32, 518, 518) else None,
            "dtype": "fp16", "data": "synthetic (randn clip; seeded synthetic-recipe weights, no checkpoint offline)",
            "config": {"workload": f"VideoDepthAnything.forward {enc} {args.clips_per_gpu}x{T}x3x{H}x{W} per GPU",
                       "encoder": enc, "frames_per_clip": T, "H": H, "W": W,
                       "clips_per_gpu": args.clips_per_gpu, "parallelism": f"clip-parallel dp{world}",
                       "hip_graph": bool(args.graph)},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if gflop:
            line["model_tflops"] = round(value * gflop / 1e3, 1)
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Benchmark: depth frames/s of the Video-Depth-Anything clip forward on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--encoder vitl] [--frames 32] [--size 518 518]
    python bench.py --video [--gpus N] ...      # BASELINE configs[3]: a 176-frame video, 8 windows

Default mode (BASELINE.json configs[2], and configs[3]'s clip-parallel form for N > 1): a step is one
``VideoDepthAnything.forward`` of a [1, 32, 3, 518, 518] clip (ViT-L fp16, full HIP path) on every
rank, inputs resident in HBM.  Multi-GPU is clip-parallel, one process per GPU (RCCL over xGMI):
rank 0's weights are broadcast once, every rank runs its own clips, and each step's depth
[32, 518, 518] fp32 is gathered to rank 0 inside the timed region (an async RCCL gather on the
collective stream, overlapped with the next step's forward).  The timed region is bracketed by
barrier + synchronize; the MAX over ranks is taken; value = all ranks' frames / that time
("scaling": "weak").  ``--gpus N`` without torchrun's WORLD_SIZE re-launches this script under
``torch.distributed.run`` with N ranks (as a child process, before anything touches the GPU).
``--streams S`` (default 2): S clips in flight per GPU — step i runs on HIP stream i % S, so one
clip's low-occupancy kernels and partial last rounds share the CUs with the other clip's; every
step is still one whole forward, all inside the timed region.

``--video`` (BASELINE configs[3] as a video job): a synthetic 176-frame 518x518 uint8 video through
``infer_video_depth`` (GPU preprocessing, 8 overlapping 32-frame windows sharded round-robin over the
ranks, depth resize, per-round RCCL gather to rank 0, host scale/shift stitching) -- all inside the
timed region.  value = video frames / s ("scaling": "strong": the video is fixed as N grows).

Extra fields:
  roofline      dominant kernel = encoder MLP fc1 GEMM + GELU, timed per launch with HIP events on its
                launch stream (inside the timed region with one clip in flight; with several, over
                single-stream forwards right after it, see roofline.probe); achieved = algorithmic FLOPs per launch / mean
                launch time vs 2.5 PFLOP/s dense fp16; traffic from profiles/<round>_pmc_fc1.json
                (rocprofv3 PMC, gfx950-corrected), mfma_busy_pmc from profiles/<round>_pmc_mfma.json
  cpu_baseline  the oracle's fp32 PyTorch-CPU forward (oracle/vda_oracle.py) of one whole clip of the
                same workload (default all 32 frames, ~80 s on 16 threads; ``--cpu-baseline-frames F``
                times a 1xF clip instead, recorded in ``frames``), rank 0 / N=1 only - a reported
                baseline only.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

PEAK_FP16_TFLOPS = 2500.0  # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense)
REF_A100_FPS = 71.4        # README.md:52-61 ViT-L fp16 14 ms/frame on 1x A100
GFLOP_PER_FRAME = {("vitl", 518, 518): 1404.6, ("vits", 518, 518): 121.3, ("vitl", 518, 924): 2761.5}
PROFILE_ROUND = "r06"      # profiles/<round>_pmc_*.json carry the PMC figures quoted in the line


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--encoder", default="vitl")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--size", type=int, nargs=2, default=[518, 518], metavar=("H", "W"))
    ap.add_argument("--clips-per-gpu", type=int, default=1)
    ap.add_argument("--video", action="store_true", help="time infer_video_depth on a synthetic video (configs[3])")
    ap.add_argument("--video-frames", type=int, default=176, help="frames of the --video input (176 = 8 windows)")
    ap.add_argument("--cpu-baseline-frames", type=int, default=32,
                    help="frames of the CPU-oracle clip timed as the cpu_baseline (0 disables; the default is the "
                         "whole 32-frame clip of the workload, ~80 s on the box's 16 threads)")
    ap.add_argument("--no-probe", action="store_true", help="skip the per-launch event probe")
    ap.add_argument("--graph", action="store_true", help="replay the forward as a captured HIP graph")
    ap.add_argument("--streams", type=int, default=2,
                    help="clips in flight per GPU: step i runs on HIP stream i %% streams (the fc1 roofline "
                         "probe then runs in a single-stream pass after the timed region)")
    ap.add_argument("--tiles", choices=["model", "static", "dynamic"], default="model",
                    help="A/B: the encoder GEMMs' tile schedule (model = the model's default)")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip the per-step depth gather to rank 0")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL; gloo for rehearsal)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only rehearsal of the launch / gather / timing plumbing with a stand-in forward "
                         "(tests; the line it prints is not a measurement)")
    return ap.parse_args()


class _StandIn(torch.nn.Module):
    """--dry-run's clip forward: [B, T, 3, H, W] -> [B, T, H, W] on the CPU (no libvda, no GPU)."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.ones(3))

    def forward(self, x):
        return torch.relu(torch.einsum("btchw,c->bthw", x, self.w.detach()))


def relaunch(args) -> int:
    """--gpus N > 1 outside torchrun: start N ranks under torch.distributed.run as a child process
    (nothing has touched the GPU yet in this process) and return its exit status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc(name):
    path = os.path.join(REPO, "profiles", f"{PROFILE_ROUND}_{name}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if rank == 0:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    dist = world > 1
    if args.dry_run:
        args.backend = "gloo"
        dev = torch.device("cpu")
    else:
        ndev = torch.cuda.device_count()
        local = local % max(1, ndev)  # (gloo rehearsal with more ranks than GPUs: ranks share a device)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    tdist = None
    if dist:
        import torch.distributed as tdist
        if args.backend == "nccl":
            tdist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:
            tdist.init_process_group(args.backend)

    enc = args.encoder
    T, (H, W) = args.frames, args.size
    if args.dry_run:
        ops = None
        model = _StandIn()
        args.no_probe, args.cpu_baseline_frames = True, 0
    else:
        import vda_amd
        from vda_amd import ops
        # weights: the synthetic recipe (no checkpoint offline) built on rank 0 and broadcast over RCCL
        # (the recipe is deterministic, so every rank could build it; the broadcast is the deployment
        # path for a checkpoint that only rank 0 reads)
        model = vda_amd.build_model(enc, device=dev)
        if args.tiles != "model":
            model.dynamic_tiles = args.tiles == "dynamic"
    if dist:
        for t in model.state_dict().values():
            if args.backend == "nccl":
                tdist.broadcast(t, src=0)
            else:  # gloo rehearsal: host copies
                c = t.detach().cpu()
                tdist.broadcast(c, src=0)
                t.copy_(c)
        if not args.dry_run:
            model.load_state_dict(model.state_dict(), strict=True)  # drop packs; re-pack from broadcast weights
    # distinct devices in the job (gloo rehearsals may put several ranks on one GPU)
    ident = (socket.gethostname(), local)
    if dist:
        ids = [None] * world
        tdist.all_gather_object(ids, ident)
        n_dev = len(set(ids))
    else:
        n_dev = 1

    if args.video:
        run_video(args, model, dev, rank, world, n_dev, tdist)
        return

    g = torch.Generator().manual_seed(1000 + rank)
    x = torch.randn(args.clips_per_gpu, T, 3, H, W, generator=g).to(dev)

    gather = dist and not args.no_gather
    nccl = args.backend == "nccl"
    pending = []  # async gathers in flight (two steps deep)
    gbufs = ([[None] * world for _ in range(2)]) if gather else None

    if not args.dry_run:
        # the packed weights and the token bias are built lazily by the first forward; build them here,
        # on the current stream, before any side stream can read them (the video driver does the same)
        model.prepare(dev, (H, W))
    strs = []
    if args.streams > 1 and dev.type == "cuda":
        strs = [torch.cuda.Stream(device=dev) for _ in range(args.streams)]
        for st in strs:
            st.wait_stream(torch.cuda.current_stream(dev))

    def step(i):
        if strs:
            with torch.cuda.stream(strs[i % len(strs)]):
                return step1(i)
        return step1(i)

    def step1(i):
        d = model(x)
        if gather:
            # clip-parallel output path: every step's depth goes to rank 0 (RCCL gather on the
            # collective stream, overlapped with the next step's forward)
            if len(pending) >= 2:
                pending.pop(0).wait()
            slot = i % 2
            if nccl:
                if rank == 0 and gbufs[slot][0] is None:
                    gbufs[slot] = [torch.empty_like(d) for _ in range(world)]
                pending.append(tdist.gather(d, gbufs[slot] if rank == 0 else None, dst=0, async_op=True))
            else:  # gloo rehearsal: host copies, synchronous
                c = d.cpu()
                tdist.gather(c, [torch.empty_like(c) for _ in range(world)] if rank == 0 else None, dst=0)
        return d

    fn = step
    if args.graph:
        if gather:
            raise SystemExit("--graph is single-rank only (the gather runs outside the captured forward)")
        for _ in range(2):
            model(x)
        torch.cuda.synchronize()
        # one captured forward per clip-in-flight stream (each graph owns its memory pool), replayed
        # on that stream
        graphs, outs = [], []
        for st in (strs or [None]):
            g_ = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_, stream=st):
                outs.append(model(x))
            graphs.append(g_)
        torch.cuda.synchronize()

        def fn(i):
            j = i % len(graphs)
            if strs:
                with torch.cuda.stream(strs[j]):
                    graphs[j].replay()
            else:
                graphs[j].replay()
            return outs[j]

    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    for i in range(args.warmup):
        fn(i)
    while pending:
        pending.pop(0).wait()
    sync()
    if dist:
        tdist.barrier()
    probe = not args.no_probe and not args.graph
    live = probe and not strs  # concurrent clips share the CUs: per-launch durations would not be the kernel's
    if live:
        ops.enable_probe(["enc_fc1"])
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        depth = fn(i)
    while pending:
        pending.pop(0).wait()
    sync()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    launches = ops.take_probe() if live else {}
    elapsed = max_over_ranks(elapsed, dev, tdist, args.backend)
    frames = world * args.steps * args.clips_per_gpu * T
    value = frames / elapsed
    if not bool(torch.isfinite(depth).all()):
        raise RuntimeError("non-finite depth")
    if gather and rank == 0 and nccl:
        got = gbufs[(args.steps - 1) % 2]
        if not all(bool(torch.isfinite(t).all()) for t in got):
            raise RuntimeError("non-finite gathered depth")
    probe_steps = 0
    if probe and not live:  # the same forward, one clip at a time, after the timed region
        probe_steps = min(args.steps, 10)
        ops.enable_probe(["enc_fc1"])
        for _ in range(probe_steps):
            model(x)
        sync()
        launches = ops.take_probe()

    # the committed PMC summaries were collected on the default workload (ViT-L 32 x 518 x 518)
    pmc_ok = args.encoder == "vitl" and args.frames == 32 and tuple(args.size) == (518, 518)
    roof = roofline(model, launches, pmc_ok)
    if roof:
        roof["probe"] = ("HIP events on the launch stream over the timed region" if live else
                         f"HIP events on the launch stream over {probe_steps} single-stream forwards after the "
                         f"timed region ({len(strs)} clips in flight would share the CUs)")
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline_frames > 0:
        cpu = cpu_baseline(model, x, enc, args.cpu_baseline_frames, H, W)

    if rank == 0:
        gflop = GFLOP_PER_FRAME.get((enc, H, W))
        line = {
            "metric": "depth frames/sec at 32x518x518, ViT-L fp16, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": n_dev, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / REF_A100_FPS, 3) if (enc, T, H, W) == ("vitl", 32, 518, 518) else None,
            "dtype": "fp16", "data": ("DRY RUN: CPU stand-in forward, not a measurement" if args.dry_run else
                                      "synthetic (randn clip; seeded synthetic-recipe weights, no checkpoint offline)"),
            "config": {"workload": f"VideoDepthAnything.forward {enc} {args.clips_per_gpu}x{T}x3x{H}x{W} per GPU",
                       "encoder": enc, "frames_per_clip": T, "H": H, "W": W,
                       "clips_per_gpu": args.clips_per_gpu, "parallelism": f"clip-parallel dp{world}",
                       "ranks": world, "depth_gather_to_rank0": bool(gather), "hip_graph": bool(args.graph),
                       "clips_in_flight": max(1, args.streams)},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if gflop:
            line["model_tflops"] = round(value * gflop / 1e3, 1)
            if roof is not None:
                # the whole forward's algorithmic FLOPs at the measured frame rate, per GPU, against the
                # dense fp16 peak (north_star's MFMA-utilisation bar), beside the dominant kernel's frac
                roof["forward_frac"] = round(value / n_dev * gflop / 1e3 / PEAK_FP16_TFLOPS, 4)
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


def max_over_ranks(elapsed, dev, tdist, backend):
    if tdist is None:
        return elapsed
    cdev = dev if backend == "nccl" else torch.device("cpu")
    tt = torch.tensor([elapsed], device=cdev, dtype=torch.float64)
    tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
    return float(tt.item())


def roofline(model, launches, pmc_ok=True):
    if not launches.get("enc_fc1"):
        return None
    C = model.pretrained.embed_dim
    rec = launches["enc_fc1"]
    flop = sum(f for _, f in rec) / len(rec)          # algorithmic 2*M*N*K per launch
    ms = sum(t for t, _ in rec) / len(rec)
    M = int(round(flop / (2.0 * 4 * C * C)))
    achieved = flop / (ms * 1e-3) / 1e12
    f1 = (pmc("pmc_fc1") or {}) if pmc_ok else {}
    mm = (pmc("pmc_mfma") or {}) if pmc_ok else {}
    mfma_busy = next((e.get("mfma_busy") for e in mm.get("kernels", {}).values() if e.get("tag") == "enc_fc1"), None)
    src = lambda name, d: f"profiles/{PROFILE_ROUND}_{name}.json" if d else None
    # the shader clock fc1 holds under load, measured in-kernel (s_memtime / s_memrealtime stamps of a
    # -DVDA_TS build, tools/clock_probe.py): the 2.5 PF peak is rated at 2.4 GHz, so frac_at_held_clock is
    # the same launch against the peak at the clock the chip actually sustains (not measured by this run)
    ck = (pmc("clock_probe") or {}) if pmc_ok else {}
    clk = ck.get("fc1_clock_ghz")
    return {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_FP16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_FP16_TFLOPS, 4), "traffic": f1.get("hbm_bytes_per_launch"),
            "mfma_busy_pmc": mfma_busy,
            "clock_ghz_in_kernel": clk,
            "frac_at_held_clock": round(achieved / (PEAK_FP16_TFLOPS * clk / 2.4), 4) if clk else None,
            # traffic and mfma_busy_pmc are NOT measured by this run: they are read from the committed
            # rocprofv3 --pmc summaries named here (tools/pmc_fc1.py, tools/pmc_mfma_summary.py)
            "pmc_source": {"traffic": src("pmc_fc1", f1), "mfma_busy_pmc": src("pmc_mfma", mfma_busy is not None),
                           "clock_ghz_in_kernel": src("clock_probe", clk),
                           "pmc_tag": "enc_fc1",
                           "note": None if pmc_ok else "the committed PMC summaries cover the ViT-L 32x518x518 "
                                                        "workload only; traffic / mfma_busy_pmc left null"},
            "kernel": f"gemm256_kernel<2,2,dense,GELU,LN-fold> (encoder norm2 + fc1) M={M} N={4 * C} K={C}",
            "flop_per_launch": flop, "avg_launch_ms": round(ms, 4), "launches": len(rec)}


def cpu_baseline(model, x, enc, nframes, H, W):
    """The oracle's fp32 CPU forward of one clip of the same workload, on the job's CPU share."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import vda_oracle  # test infrastructure: the reported CPU baseline only
    nthr = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)  # the box's CPU share (16 per GPU)
    nthr = max(1, min(nthr, omp) if omp > 0 else min(nthr, 16))
    torch.set_num_threads(nthr)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    xs = x[:1, :nframes].float().cpu()
    vda_oracle.forward(sd, enc, xs[:, :1, :, :84, :84])  # warm the CPU kernels
    print(f"bench.py: timing the CPU oracle on one {enc} 1x{xs.shape[1]}x3x{H}x{W} clip ...", file=sys.stderr,
          flush=True)
    t1 = time.perf_counter()
    vda_oracle.forward(sd, enc, xs)
    cpu_s = time.perf_counter() - t1
    return {"value": round(xs.shape[1] / cpu_s, 4), "unit": "frames/s", "cores": torch.get_num_threads(),
            "kind": "port", "cpu": cpu_model(), "frames": int(xs.shape[1]),
            "sample": f"oracle fp32 PyTorch-CPU forward of one {enc} 1x{xs.shape[1]}x3x{H}x{W} clip "
                      f"({cpu_s:.1f} s, {torch.get_num_threads()} threads)"}


def run_video(args, model, dev, rank, world, n_dev, tdist):
    """configs[3] as a video job: infer_video_depth over a synthetic video, everything timed."""
    import numpy as np
    from vda_amd import video as V
    H, W = args.size
    n = args.video_frames
    frames = np.random.default_rng(0).integers(0, 256, (n, H, W, 3), dtype=np.uint8)
    nwin = len(V.window_starts(n))
    io = V.DeviceIO
    if args.dry_run:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import vda_oracle  # dry run only: torch-CPU stand-ins for the preprocessing kernels
        io = vda_oracle.TorchIO

    def job():
        return V.infer_video_depth(model, frames, 30, input_size=518, device=dev, rank=rank, world=world,
                                   io=io)

    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    for _ in range(args.warmup):
        job()
    sync()
    if tdist is not None:
        tdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        depth, _ = job()
    sync()
    if tdist is not None:
        tdist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev, tdist, args.backend)
    if rank == 0:
        if depth.shape != (n, H, W) or not np.isfinite(depth).all():
            raise RuntimeError(f"bad video depth {depth.shape}")
        value = args.steps * n / elapsed
        line = {
            "metric": f"video depth frames/sec, {n}-frame {H}x{W} video ({nwin} windows of 32), "
                      f"{args.encoder} fp16, 1/2/4/8 MI355X",
            "value": round(value, 2), "unit": "video frames/s", "n_gpus": n_dev, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp16",
            "data": ("DRY RUN: CPU stand-in forward, not a measurement" if args.dry_run else
                     "synthetic (random uint8 video; seeded synthetic-recipe weights)"),
            "config": {"workload": f"infer_video_depth {args.encoder} {n}x{H}x{W} uint8 video, {nwin} windows",
                       "encoder": args.encoder, "windows": nwin, "clip_frames_computed": nwin * 32,
                       "parallelism": f"window-parallel dp{world} (round-robin), per-round RCCL gather + "
                                      "host stitch on rank 0, all timed",
                       "ranks": world},
            "clip_frames_per_s": round(args.steps * nwin * 32 / elapsed, 2),
        }
        print(json.dumps(line), flush=True)
    if tdist is not None:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()

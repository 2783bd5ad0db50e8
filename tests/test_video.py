"""Long-video orchestration (video_depth.py:329-417): windows, stitching, clip-parallel sharding.

CPU tests drive ``vda_amd.video.infer_video_depth`` with the oracle as the clip forward and
compare with the reference's own ``infer_video_depth`` output (tests/golden/video_vits_57f.npz);
the world-size-2 gloo test checks that sharding windows over ranks + gather reproduces the
single-process result exactly.  The GPU test runs the same video through libvda.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import GOLDEN, recipe_state_dict, vda_oracle
from vda_amd import video as V


def load_video_golden():
    z = np.load(os.path.join(GOLDEN, "video_vits_57f.npz"), allow_pickle=False)
    return z["frames"], z["depth"], json.loads(str(z["meta"]))


def simulate_reference_windows(n):
    """Literal replay of the reference loop (video_depth.py:351-364) on frame ids."""
    step = V.INFER_LEN - V.OVERLAP
    plist = list(range(n)) + [n - 1] * ((step - n % step) % step + (V.INFER_LEN - step))
    wins, pre = [], None
    for fid in range(0, n, step):
        cur = [plist[fid + i] for i in range(V.INFER_LEN)]
        if pre is not None:
            cur[:V.OVERLAP] = [pre[j] for j in V.KEYFRAMES]
        wins.append(cur)
        pre = cur
    return wins, len(plist)


@pytest.mark.parametrize("n", [1, 5, 22, 23, 32, 44, 57, 100, 447])
def test_window_closed_form_matches_reference_loop(n):
    wins, plen = simulate_reference_windows(n)
    assert plen == V.padded_length(n)
    assert len(wins) == len(V.window_starts(n))
    for k, w in enumerate(wins):
        assert V.window_frame_indices(k, n) == w


def test_net_input_size_rules():
    assert V.net_input_size(48, 64, 56) == (56, 70)
    assert V.net_input_size(720, 1280, 518) == (518, 924)  # 16:9 < 1.78: no shrink
    assert V.net_input_size(280, 924, 518) == (280, 924)   # ratio 3.3 > 1.78: input_size shrinks to 280
    for h, w in [(480, 640), (1080, 1920), (100, 37)]:
        H, W = V.net_input_size(h, w, 518)
        assert H % 14 == 0 and W % 14 == 0


def _oracle_forward(sd):
    return lambda x: vda_oracle.forward(sd, "vits", x.cpu())


def test_video_orchestration_matches_reference_golden():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    frames, depth_ref, meta = load_video_golden()
    sd = recipe_state_dict("vits")
    depth, fps = V.infer_video_depth(_oracle_forward(sd), frames, meta["fps"], input_size=meta["input_size"],
                                     device="cpu", io=vda_oracle.TorchIO)
    assert depth.shape == depth_ref.shape
    err = float(np.abs(depth - depth_ref).sum() / np.abs(depth_ref).sum())
    assert err <= 1e-5, err


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q, wpb=1, single=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    frames, _, meta = load_video_golden()
    sd = recipe_state_dict("vits")
    depth, _ = V.infer_video_depth(_oracle_forward(sd), frames, meta["fps"], input_size=meta["input_size"],
                                   device="cpu", rank=rank, world=world, io=vda_oracle.TorchIO, streams=2,
                                   windows_per_batch=wpb)
    if rank == 0:
        if single:  # the same job in one process, same threads: the sharded result must be these bytes
            d1, _ = V.infer_video_depth(_oracle_forward(sd), frames, meta["fps"], input_size=meta["input_size"],
                                        device="cpu", io=vda_oracle.TorchIO, streams=2)
            q.put((depth, d1))
        else:
            q.put(depth)
    dist.barrier()
    dist.destroy_process_group()


def test_clip_parallel_gloo_world2_matches_single_process():
    frames, depth_ref, meta = load_video_golden()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    depth = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    err = float(np.abs(depth - depth_ref).sum() / np.abs(depth_ref).sum())
    assert err <= 1e-5, err


def test_clip_parallel_gloo_world2_async_gather_byte_identical():
    """World 2 with streams=2: each round's gather is asynchronous and rank 0 stitches a round only
    after the next round's forward and gather are enqueued; the result is byte for byte the
    single-process job's (video_depth.py:358-413; one window per forward on both sides, so every
    window's clip forward is the same computation)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q, 1, True)) for r in range(2)]
    for p in procs:
        p.start()
    depth, d1 = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert depth.shape == d1.shape and np.array_equal(depth, d1)


@pytest.mark.gpu
def test_video_on_gpu_matches_reference_golden():
    import vda_amd
    frames, depth_ref, meta = load_video_golden()
    m = vda_amd.build_model("vits", recipe_state_dict("vits"), device="cuda")
    depth, _ = V.infer_video_depth(m, frames, meta["fps"], input_size=meta["input_size"], device="cuda",
                                   windows_per_batch=2)
    err = float(np.abs(depth - depth_ref).sum() / np.abs(depth_ref).sum())
    print(f"video 57 frames: rel-L1 vs reference = {err:.3e}")
    assert err <= 1e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("src,dst", [((48, 64), (56, 70)), ((720, 1280), (518, 924)), ((37, 53), (518, 742)),
                                     ((518, 518), (518, 518)), ((5, 3), (28, 14))])
def test_preprocess_kernel_vs_torch(src, dst):
    """vda_preprocess_frames vs the oracle's torch bicubic + normalise (fp32; down, up, identity, tiny)."""
    from vda_amd import ops
    g = torch.Generator().manual_seed(src[0] * 7 + dst[1])
    fr = torch.randint(0, 256, (3, src[0], src[1], 3), generator=g, dtype=torch.uint8)
    out = ops.preprocess_frames(fr.cuda(), *dst).cpu()
    ref = vda_oracle.TorchIO.preprocess(fr.double().to(torch.uint8), dst)
    assert out.shape == ref.shape == (3, 3) + dst
    assert (out - ref).abs().max().item() <= 2e-5
    assert V.DeviceIO.preprocess(fr[:0].cuda(), dst).shape == (0, 3) + dst


@pytest.mark.gpu
@pytest.mark.parametrize("src,dst", [((56, 70), (48, 64)), ((518, 924), (720, 1280)), ((14, 14), (1, 1)),
                                     ((1, 7), (3, 9))])
def test_depth_resize_kernel_vs_torch(src, dst):
    from vda_amd import ops
    g = torch.Generator().manual_seed(src[1] + dst[0])
    d = torch.rand(2, *src, generator=g) * 50
    out = ops.depth_resize(d.cuda(), *dst).cpu()
    ref = vda_oracle.TorchIO.resize_depth(d, dst)
    # fp32 source-coordinate rounding (o * (in-1)/(out-1) near o ~ 10^3) moves the blend weight by
    # ~1e-5, i.e. ~1e-5 of the local depth step: bound it relative to the depth range
    assert (out - ref).abs().max().item() <= 1e-4 * d.abs().max().item()
    assert vda_oracle.rel_l1(out, ref) <= 2e-5  # white-noise depth: the worst case for weight rounding


def test_config1_vits_8x518_video_cpu_plumbing():
    """BASELINE configs[0]: an 8-frame 518x518 video through the long-video driver with the fp32 CPU
    oracle as the clip forward.  The reference pads the 8 frames to one 32-frame window with copies of
    the last frame (video_depth.py:351-354) and returns the first 8; the driver must reproduce exactly
    that plumbing: equal to one oracle forward of the padded clip, cut to 8 frames."""
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    g = np.random.default_rng(11)
    frames = g.integers(0, 256, (8, 518, 518, 3), dtype=np.uint8)
    sd = recipe_state_dict("vits")
    depth, fps = V.infer_video_depth(_oracle_forward(sd), frames, 30, input_size=518, device="cpu",
                                     io=vda_oracle.TorchIO)
    assert depth.shape == (8, 518, 518) and fps == 30
    idx = V.window_frame_indices(0, 8)
    assert idx == list(range(8)) + [7] * 24
    x = vda_oracle.TorchIO.preprocess(torch.from_numpy(frames[idx]), (518, 518)).unsqueeze(0)
    ref = vda_oracle.forward(sd, "vits", x)[0, :8].numpy()
    err = float(np.abs(depth - ref).sum() / np.abs(ref).sum())
    assert err <= 1e-6, err


@pytest.mark.gpu
def test_video_device_memory_flat_in_video_length():
    """Each window's depth leaves the device right after its resize: the peak device
    memory of a 4x longer video stays the same."""
    def fwd(x):
        return x[:, :, 0].contiguous()
    peaks = []
    for n in (60, 240):
        frames = np.random.default_rng(n).integers(0, 256, (n, 48, 64, 3), dtype=np.uint8)
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        d, _ = V.infer_video_depth(fwd, frames, 24, input_size=56, device="cuda")
        assert d.shape == (n, 48, 64)
        peaks.append(torch.cuda.max_memory_allocated() - base)
    assert peaks[1] <= peaks[0] * 1.1 + (1 << 20), peaks


def test_host_sink_stitches_out_of_order_windows():
    """Multi-rank rounds land windows out of order (windows_per_batch > 1): the incremental stitcher
    must buffer them and produce exactly the one-shot stitch of the ordered list."""
    g = np.random.default_rng(5)
    nwin, n = 5, 100
    wins = [g.random((V.INFER_LEN, 6, 7), dtype=np.float32) * 10 + 1 for _ in range(nwin)]
    ref = V.stitch([f for w in wins for f in w], n)
    sink = V._HostSink(torch.device("cpu"), n)
    for k in (2, 0, 4, 1, 3):
        sink.put(k, torch.from_numpy(wins[k]))
    out = sink.result()
    assert out.shape == ref.shape == (n, 6, 7)
    assert np.array_equal(out, ref)
    # a window that never arrives is an error, not a silently short video
    sink = V._HostSink(torch.device("cpu"), n)
    sink.put(1, torch.from_numpy(wins[1]))
    with pytest.raises(RuntimeError):
        sink.result()


@pytest.mark.gpu
def test_video_two_streams_identical_to_one():
    """infer_video_depth(streams=2) runs consecutive windows on two HIP streams: same bytes as one stream."""
    import vda_amd
    frames, _, meta = load_video_golden()
    m = vda_amd.build_model("vits", recipe_state_dict("vits"), device="cuda")
    d1, _ = V.infer_video_depth(m, frames, meta["fps"], input_size=meta["input_size"], device="cuda", streams=1)
    d2, _ = V.infer_video_depth(m, frames, meta["fps"], input_size=meta["input_size"], device="cuda", streams=2)
    assert np.array_equal(d1, d2)


@pytest.mark.gpu
def test_video_two_streams_fresh_model():
    """streams=2 as the FIRST call on a freshly built model: the packed weights and the
    resolution's token bias are built on the current stream before the side streams start, so the
    result equals a fresh model's one-stream run."""
    import vda_amd
    frames, _, meta = load_video_golden()
    d = []
    for streams in (2, 1):
        m = vda_amd.build_model("vits", recipe_state_dict("vits"), device="cuda")
        d.append(m.infer_video_depth(frames, meta["fps"], input_size=meta["input_size"], device="cuda",
                                     streams=streams)[0])
        del m
    assert np.array_equal(d[0], d[1])


@pytest.mark.gpu
def test_video_frames_already_on_device():
    """frames may be handed over as a device tensor (no host staging then): same result as numpy."""
    def fwd(x):
        return x[:, :, 0].contiguous()
    frames = np.random.default_rng(3).integers(0, 256, (40, 48, 64, 3), dtype=np.uint8)
    d_host, _ = V.infer_video_depth(fwd, frames, 24, input_size=56, device="cuda")
    d_dev, _ = V.infer_video_depth(fwd, torch.from_numpy(frames).cuda(), 24, input_size=56, device="cuda")
    assert np.array_equal(d_host, d_dev)


@pytest.mark.gpu
def test_multirank_receive_buffers_survive_side_stream_reuse(monkeypatch):
    """VERDICT r3 item 4 / ADVICE r3: with world > 1 each round's receive buffers come from a side
    stream, while rank 0's sink copies them to the host on the current stream.  A stand-in gather
    returns side-stream device buffers and its wait() delays the current stream, so without the
    record_stream in ``land`` the side stream's next forward (which allocates and scribbles over
    same-size blocks) overwrites them before the copies run.  streams=2 must equal streams=1."""
    class _Work:
        def wait(self):
            torch.cuda._sleep(20_000_000)  # hold the current stream so the D2H copies queue late

    def fake_gather(buf, rank, world, group):
        bufs = [(buf * (1.0 + src)).contiguous() for src in range(world)]
        return bufs, _Work(), buf

    def fwd(x):
        for _ in range(3):  # same-size scratch written on this stream: reuses freed receive blocks
            torch.full((x.shape[0], x.shape[1], x.shape[3], x.shape[4]), -7.0, device=x.device)
        return (x[:, :, 0] * 3.0 + 1.0).contiguous()

    monkeypatch.setattr(V, "_gather_round", fake_gather)
    frames = np.random.default_rng(11).integers(0, 256, (150, 48, 64, 3), dtype=np.uint8)
    out = []
    for streams in (1, 2):
        d, _ = V.infer_video_depth(fwd, frames, 24, input_size=56, device="cuda", rank=0, world=2,
                                   streams=streams)
        torch.cuda.synchronize()
        out.append(d)
    assert np.array_equal(out[0], out[1])

"""Long-video inference: 32-frame windows, clip-parallel sharding, host scale/shift stitching.

Mirrors ``VideoDepthAnything.infer_video_depth`` (video_depth.py:329-417) and its helpers
(utils/util.py:16-73, util/transform.py:5-157):

* frames are resized (lower-bound, keep aspect, multiple of 14, bicubic) and ImageNet-normalised;
* the frame list is padded with copies of the last frame to a multiple of the 22-frame stride
  plus the 10 overlap slots (:351-354);
* window k feeds frames [k*22 .. k*22+31] with slots 0..9 overwritten by the previous window's
  slots KEYFRAMES (:363-364).  That overwrite copies *input frames*, so each window has a closed
  form (``window_frame_indices``) and windows are independent: ``infer_video_depth`` may shard
  them over ranks (one process per GPU, RCCL) with no data-path collective but the final depth
  gather to rank 0;
* rank 0 stitches: least-squares scale/shift on keyframe slots {0, 12}, 8-frame linear blend,
  clip at 0 (:379-413).

Preprocessing (bicubic resize + normalise) and the final depth resize run as libvda kernels
(``DeviceIO``).  cv2 is not available here, so the bicubic resize is pinned against torch bicubic
(a=-0.75, the same kernel as cv2.INTER_CUBIC), not cv2 itself.
"""
from __future__ import annotations

import contextlib
import math
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch

INFER_LEN = 32
OVERLAP = 10
KEYFRAMES = [0, 12, 24, 25, 26, 27, 28, 29, 30, 31]
INTERP_LEN = 8
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


# ---- windowing ------------------------------------------------------------------------------
def padded_length(n_frames: int) -> int:
    """video_depth.py:350-354: pad to a multiple of the stride plus the overlap."""
    step = INFER_LEN - OVERLAP
    return n_frames + (step - (n_frames % step)) % step + (INFER_LEN - step)


def window_starts(n_frames: int) -> List[int]:
    return list(range(0, n_frames, INFER_LEN - OVERLAP))


def window_frame_indices(k: int, n_frames: int) -> List[int]:
    """Original frame index of every slot of window k (closed form of :358-364), clamped to the
    padded list (padding repeats the last frame)."""
    step = INFER_LEN - OVERLAP
    if k == 0:
        idx = list(range(INFER_LEN))
    else:
        prev = window_frame_indices(k - 1, n_frames)
        idx = [prev[j] for j in KEYFRAMES] + [k * step + i for i in range(OVERLAP, INFER_LEN)]
    return [min(i, n_frames - 1) for i in idx]


# ---- preprocessing (util/transform.py:5-157, video_depth.py:330-348) ------------------------
def _constrain(x, multiple, min_val=0, max_val=None):
    y = int(np.round(x / multiple) * multiple)
    if max_val is not None and y > max_val:
        y = int(np.floor(x / multiple) * multiple)
    if y < min_val:
        y = int(np.ceil(x / multiple) * multiple)
    return y


def net_input_size(height: int, width: int, input_size: int = 518) -> tuple:
    """(H, W) the network sees: aspect > 1.78 shrinks input_size (:330-334); Resize lower_bound,
    keep_aspect_ratio, ensure_multiple_of=14 (transform.py:57-110)."""
    ratio = max(height, width) / min(height, width)
    if ratio > 1.78:
        input_size = int(input_size * 1.777 / ratio)
        input_size = round(input_size / 14) * 14
    sh, sw = input_size / height, input_size / width
    if sw > sh:
        sh = sw
    else:
        sw = sh
    return (_constrain(sh * height, 14, min_val=input_size), _constrain(sw * width, 14, min_val=input_size))


class DeviceIO:
    """The per-frame data formats either side of the forward, on libvda kernels:
    ``preprocess`` uint8 frames [N, h, w, 3] (on the device) -> normalised input [N, 3, H, W] fp32
    (bicubic resize + ImageNet normalise, vda_preprocess_frames); ``resize_depth`` depth [N, H, W]
    -> [N, h, w] fp32 (bilinear align_corners=True, vda_depth_resize).  The drivers take any object
    with these two methods (the tests pass the oracle's torch-CPU restatement, ``TorchIO``)."""

    @staticmethod
    def preprocess(frames: torch.Tensor, size: tuple) -> torch.Tensor:
        from . import ops
        return ops.preprocess_frames(frames, int(size[0]), int(size[1]), MEAN, STD)

    @staticmethod
    def resize_depth(depth: torch.Tensor, size: tuple) -> torch.Tensor:
        from . import ops
        return ops.depth_resize(depth.float().contiguous(), int(size[0]), int(size[1]))


# ---- stitching (video_depth.py:375-413, utils/util.py:40-73) --------------------------------
def compute_scale_and_shift(prediction, target, mask):
    prediction = prediction.astype(np.float32)
    target = target.astype(np.float32)
    mask = mask.astype(np.float32)
    a_00 = np.sum(mask * prediction * prediction)
    a_01 = np.sum(mask * prediction)
    a_11 = np.sum(mask)
    b_0 = np.sum(mask * prediction * target)
    b_1 = np.sum(mask * target)
    x_0, x_1 = 1, 0
    det = a_00 * a_11 - a_01 * a_01
    if det != 0:
        x_0 = (a_11 * b_0 - a_01 * b_1) / det
        x_1 = (-a_01 * b_0 + a_00 * b_1) / det
    return x_0, x_1


def interpolate_frames(pre: Sequence[np.ndarray], post: Sequence[np.ndarray]) -> List[np.ndarray]:
    n = len(pre)
    step = 1.0 / (n - 1)
    w = [0.0] + [i * step for i in range(1, n - 1)] + [1.0]
    return [pre[i] * (1 - w[i]) + post[i] * w[i] for i in range(n)]


class Stitcher:
    """The reference's stitch loop (video_depth.py:379-413) taken one window at a time, so the host
    aligns window k while the GPU computes window k + 1.  ``add`` takes the windows in order.  Only
    the last INTERP_LEN aligned frames can still change (the next window blends into them), so every
    earlier one is written straight into the preallocated [n_frames, h, w] result as it settles."""

    def __init__(self, n_frames: int):
        self.n = int(n_frames)
        self.out: Optional[np.ndarray] = None
        self.done = 0
        self.aligned: List[np.ndarray] = []
        self.ref_align: List[np.ndarray] = []

    def _flush(self, keep: int):
        if self.out is None:
            self.out = np.empty((self.n,) + self.aligned[0].shape, dtype=self.aligned[0].dtype)
        while len(self.aligned) > keep and self.done < self.n:
            self.out[self.done] = self.aligned.pop(0)
            self.done += 1

    def add(self, win: Sequence[np.ndarray]):
        align_len = OVERLAP - INTERP_LEN
        kf_align = KEYFRAMES[:align_len]
        if not self.aligned:
            self.aligned += list(win[:INFER_LEN])
            for kf in kf_align:
                self.ref_align.append(win[kf])
            self._flush(INTERP_LEN)
            return
        cur = [win[i] for i in range(len(kf_align))]
        scale, shift = compute_scale_and_shift(np.concatenate(cur), np.concatenate(self.ref_align),
                                               np.concatenate(np.ones_like(self.ref_align) == 1))
        pre = self.aligned[-INTERP_LEN:]
        post = list(win[align_len:OVERLAP])
        for i in range(len(post)):
            post[i] = post[i] * scale + shift
            post[i][post[i] < 0] = 0
        self.aligned[-INTERP_LEN:] = interpolate_frames(pre, post)
        for i in range(OVERLAP, INFER_LEN):
            d = win[i] * scale + shift
            d[d < 0] = 0
            self.aligned.append(d)
        self.ref_align = self.ref_align[:1]
        for kf in kf_align[1:]:
            d = win[kf] * scale + shift
            d[d < 0] = 0
            self.ref_align.append(d)
        self._flush(INTERP_LEN)

    def result(self) -> np.ndarray:
        self._flush(0)
        return self.out[:self.done]


def stitch(depth_list: List[np.ndarray], n_frames: int) -> np.ndarray:
    """depth_list: per-window depth frames concatenated (32 per window) -> [n_frames, h, w]."""
    st = Stitcher(n_frames)
    for fid in range(0, len(depth_list), INFER_LEN):
        st.add(depth_list[fid:fid + INFER_LEN])
    return st.result()


# ---- driver ---------------------------------------------------------------------------------
class _HostSink:
    """Moves each window's resized depth [32, h, w] off the device as soon as it exists (as the
    reference does, video_depth.py:372-373), so device memory stays flat in the video length, and
    stitches the windows in order as they land.  On a GPU the copies go through a ring of two
    pinned staging buffers with non-blocking D2H copies: window k is copied out and stitched on the
    host while the device runs window k + 1's forward."""

    def __init__(self, device: torch.device, n_frames: int):
        self.gpu = device.type == "cuda"
        self.ring: list = []
        self.pending: list = []  # (window id, staging slot, event)
        self.ready = {}          # landed windows not yet stitched (multi-rank rounds arrive out of order)
        self.next = 0
        self.stitcher = Stitcher(n_frames)

    def _land(self, k: int, a: np.ndarray):
        self.ready[k] = a
        while self.next in self.ready:
            self.stitcher.add(list(self.ready.pop(self.next)))
            self.next += 1

    def _drain(self, keep: int):
        while len(self.pending) > keep:
            k, slot, ev = self.pending.pop(0)
            ev.synchronize()
            self._land(k, slot.numpy().copy())

    def put(self, k: int, d: torch.Tensor):
        if not self.gpu:
            self._land(k, d.detach().to("cpu", torch.float32).numpy().copy())
            return
        self._drain(1)  # slot (len(pending) % 2) is free after this
        busy = {id(s) for _, s, _ in self.pending}
        slot = next((s for s in self.ring if id(s) not in busy and s.shape == d.shape), None)
        if slot is None:
            slot = torch.empty(d.shape, dtype=torch.float32, pin_memory=True)
            self.ring.append(slot)
            self.ring = self.ring[-2:]
        slot.copy_(d, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((k, slot, ev))

    def result(self) -> np.ndarray:
        self._drain(0)
        if self.ready:
            raise RuntimeError(f"windows {sorted(self.ready)} never became stitchable (missing {self.next})")
        return self.stitcher.result()


class _HostSource:
    """Uploads a window batch's frames: gathered on the host into one of two pinned staging
    buffers, then copied with a non-blocking H2D (a pageable copy would hold the host until the
    device had drained the previous window, leaving the GPU idle while the next forward is
    launched).  A slot is reused only after its previous copy has completed."""

    def __init__(self, frames: torch.Tensor, device: torch.device):
        self.frames, self.dev = frames, device
        self.gpu = device.type == "cuda"
        self.slots: list = []  # [pinned tensor, event or None]

    def get(self, idx: List[int]) -> torch.Tensor:
        ix = torch.as_tensor(idx, dtype=torch.long)
        if not self.gpu or self.frames.device.type != "cpu":  # CPU run, or frames already on a device
            return self.frames[ix.to(self.frames.device)].to(self.dev)
        shape = (len(idx),) + tuple(self.frames.shape[1:])
        slot = next((s for s in self.slots if tuple(s[0].shape) == shape and (s[1] is None or s[1].query())), None)
        if slot is None:
            if len(self.slots) >= 2:
                slot = self.slots.pop(0)
                slot[1].synchronize()
                if tuple(slot[0].shape) != shape:
                    slot[0] = torch.empty(shape, dtype=self.frames.dtype, pin_memory=True)
            else:
                slot = [torch.empty(shape, dtype=self.frames.dtype, pin_memory=True), None]
            self.slots.append(slot)
        torch.index_select(self.frames, 0, ix, out=slot[0])
        x = slot[0].to(self.dev, non_blocking=True)
        slot[1] = torch.cuda.Event()
        slot[1].record()
        return x


def _gather_round(buf: torch.Tensor, rank: int, world: int, group):
    """Start gathering one round's per-rank window buffers [n, 32, h, w] to rank 0 (RCCL on GPU
    tensors, issued on the current stream; gloo takes host copies).  Returns (the list of world
    receive buffers on rank 0 or None, the async work, the send buffer to keep alive)."""
    import torch.distributed as dist
    cpu = dist.get_backend(group) == "gloo"
    src = buf.cpu() if cpu else buf
    bufs = [torch.empty_like(src) for _ in range(world)] if rank == 0 else None
    work = dist.gather(src, bufs, dst=0, group=group, async_op=True)
    return bufs, work, src


def infer_video_depth(forward: Callable[[torch.Tensor], torch.Tensor], frames, target_fps, input_size: int = 518,
                      device="cuda", windows_per_batch: int = 1, rank: int = 0, world: int = 1, group=None,
                      io=DeviceIO, streams: int = 2, prepare: Optional[Callable[[tuple], None]] = None):
    """Depth for every frame of ``frames`` (uint8 [N, h, w, 3] numpy or tensor).

    ``forward(x[B, 32, 3, H, W]) -> depth[B, 32, H, W]`` is the clip forward (the model, or any
    callable); ``prepare((H, W))``, when given, builds whatever state the forward creates lazily
    (packed weights, the resolution's token bias) on the current stream before any side stream runs
    a forward.  With world > 1, window k runs on rank k % world: round r is windows
    r*world .. r*world + world - 1, one per rank, and each round's (or each ``windows_per_batch``
    rounds') depth maps are gathered to rank 0 by an asynchronous collective, so no rank ever holds
    more than two batches of windows on the device.  Rank 0 hands round r's windows to the host
    stitcher only after round r + 1's forward and gather are enqueued, so the host work never sits
    between two collectives; rank 0 returns (depth, fps), others (None, fps).

    ``streams`` > 1 (GPU): consecutive window batches go round-robin onto that many HIP streams, so
    one window's forward can start while the previous one's tail kernels run (one GPU, two streams:
    the 176-frame ViT-L job in 414-420 ms against 442 ms on one stream and 413 ms for its 8 forwards
    back to back; ``tools/archive/video_probe.py``).  Each rank of a multi-GPU job does the same.
    """
    if not isinstance(frames, torch.Tensor):
        frames = torch.from_numpy(np.ascontiguousarray(frames))
    n = frames.shape[0]
    h, w = int(frames.shape[1]), int(frames.shape[2])
    size = net_input_size(h, w, input_size)
    nwin = len(window_starts(n))
    rounds = (nwin + world - 1) // world
    dev = torch.device(device)
    sink = _HostSink(dev, n) if rank == 0 else None
    source = _HostSource(frames, dev)
    wpb = max(1, int(windows_per_batch))
    if prepare is None and callable(getattr(forward, "prepare", None)):  # the model itself as the forward
        prepare = lambda hw: forward.prepare(dev, hw)  # noqa: E731
    if prepare is not None:
        prepare(size)
    strs = []
    if dev.type == "cuda" and int(streams) > 1:
        strs = [torch.cuda.Stream(device=dev) for _ in range(int(streams))]
        for st in strs:  # after prepare(): the side streams see the packed weights / token bias
            st.wait_stream(torch.cuda.current_stream(dev))
    pending = None  # previous round's (receive buffers, rounds, work, send buffer)

    def land(pend):
        bufs, rr_, work, _ = pend
        work.wait()  # the current stream (or, on gloo, the host) waits for the gather
        if rank == 0:
            if strs:
                # the receive buffers were allocated on a side stream, but the sink's D2H copies run on
                # the current one: without this the caching allocator could hand their blocks to that
                # side stream's next forward while the copies are still queued
                cur_st = torch.cuda.current_stream(dev)
                for b in bufs:
                    if b.is_cuda:
                        b.record_stream(cur_st)
            for src in range(world):
                for j, r in enumerate(rr_):
                    k = r * world + src
                    if k < nwin:
                        sink.put(k, bufs[src][j])

    for bi, r0 in enumerate(range(0, rounds, wpb)):
        rr = list(range(r0, min(rounds, r0 + wpb)))
        ks = [r * world + rank for r in rr if r * world + rank < nwin]
        d = None
        with (torch.cuda.stream(strs[bi % len(strs)]) if strs else contextlib.nullcontext()):
            if ks:
                idx = [window_frame_indices(k, n) for k in ks]
                uniq = sorted(set(i for row in idx for i in row))
                pre = io.preprocess(source.get(uniq), size)
                pos = {f: j for j, f in enumerate(uniq)}
                x = torch.stack([pre[[pos[i] for i in row]] for row in idx], 0)
                del pre
                with torch.no_grad():
                    d = forward(x).float()  # [B, 32, H, W]
                del x
                d = io.resize_depth(d.flatten(0, 1), (h, w)).view(len(ks), INFER_LEN, h, w)
            if world == 1:
                for j, k in enumerate(ks):
                    sink.put(k, d[j])
                continue
            # every rank takes part in every round's gather (a rank without a window sends zeros),
            # enqueued behind this round's forward on its stream
            buf = torch.zeros(len(rr), INFER_LEN, h, w, dtype=torch.float32, device=dev)
            if d is not None:
                buf[:len(ks)] = d
            cur = _gather_round(buf, rank, world, group) + (rr,)
        if pending is not None:
            land(pending)
        pending = (cur[0], cur[3], cur[1], cur[2])
    if pending is not None:
        land(pending)
    if rank != 0:
        return None, target_fps
    return sink.result(), target_fps

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


def stitch(depth_list: List[np.ndarray], n_frames: int) -> np.ndarray:
    """depth_list: per-window depth frames concatenated (32 per window) -> [n_frames, h, w]."""
    aligned: List[np.ndarray] = []
    ref_align: List[np.ndarray] = []
    align_len = OVERLAP - INTERP_LEN
    kf_align = KEYFRAMES[:align_len]
    for fid in range(0, len(depth_list), INFER_LEN):
        if not aligned:
            aligned += depth_list[:INFER_LEN]
            for kf in kf_align:
                ref_align.append(depth_list[fid + kf])
            continue
        cur = [depth_list[fid + i] for i in range(len(kf_align))]
        scale, shift = compute_scale_and_shift(np.concatenate(cur), np.concatenate(ref_align),
                                               np.concatenate(np.ones_like(ref_align) == 1))
        pre = aligned[-INTERP_LEN:]
        post = list(depth_list[fid + align_len: fid + OVERLAP])
        for i in range(len(post)):
            post[i] = post[i] * scale + shift
            post[i][post[i] < 0] = 0
        aligned[-INTERP_LEN:] = interpolate_frames(pre, post)
        for i in range(OVERLAP, INFER_LEN):
            d = depth_list[fid + i] * scale + shift
            d[d < 0] = 0
            aligned.append(d)
        ref_align = ref_align[:1]
        for kf in kf_align[1:]:
            d = depth_list[fid + kf] * scale + shift
            d[d < 0] = 0
            ref_align.append(d)
    return np.stack(aligned[:n_frames], axis=0)


# ---- driver ---------------------------------------------------------------------------------
class _HostSink:
    """Moves each window's resized depth [32, h, w] off the device as soon as it exists (as the
    reference does, video_depth.py:372-373), so device memory stays flat in the video length.  On a
    GPU the copies go through a ring of two pinned staging buffers with non-blocking D2H copies, so
    the next window's forward is enqueued while the previous window drains."""

    def __init__(self, device: torch.device):
        self.gpu = device.type == "cuda"
        self.ring: list = []
        self.pending: list = []  # (window id, staging slot, event)
        self.out = {}

    def _drain(self, keep: int):
        while len(self.pending) > keep:
            k, slot, ev = self.pending.pop(0)
            ev.synchronize()
            self.out[k] = slot.numpy().copy()

    def put(self, k: int, d: torch.Tensor):
        if not self.gpu:
            self.out[k] = d.detach().to("cpu", torch.float32).numpy().copy()
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

    def result(self):
        self._drain(0)
        return self.out


def _gather_round(buf: torch.Tensor, rank: int, world: int, group):
    """Gather one round's per-rank window buffers [n, 32, h, w] to rank 0 (RCCL on GPU tensors; gloo
    takes host copies).  Returns the list of world buffers on rank 0, None elsewhere."""
    import torch.distributed as dist
    cpu = dist.get_backend(group) == "gloo"
    src = buf.cpu() if cpu else buf
    bufs = [torch.empty_like(src) for _ in range(world)] if rank == 0 else None
    dist.gather(src, bufs, dst=0, group=group)
    return bufs


def infer_video_depth(forward: Callable[[torch.Tensor], torch.Tensor], frames, target_fps, input_size: int = 518,
                      device="cuda", windows_per_batch: int = 1, rank: int = 0, world: int = 1, group=None,
                      io=DeviceIO):
    """Depth for every frame of ``frames`` (uint8 [N, h, w, 3] numpy or tensor).

    ``forward(x[B, 32, 3, H, W]) -> depth[B, 32, H, W]`` is the clip forward (the model, or any
    callable).  With world > 1, window k runs on rank k % world: round r is windows
    r*world .. r*world + world - 1, one per rank, and each round's (or each ``windows_per_batch``
    rounds') depth maps are gathered to rank 0 as soon as they exist, so no rank ever holds more than
    one batch of windows on the device.  Rank 0 keeps the windows in host memory and stitches;
    rank 0 returns (depth, fps), others (None, fps).
    """
    if not isinstance(frames, torch.Tensor):
        frames = torch.from_numpy(np.ascontiguousarray(frames))
    n = frames.shape[0]
    h, w = int(frames.shape[1]), int(frames.shape[2])
    size = net_input_size(h, w, input_size)
    nwin = len(window_starts(n))
    rounds = (nwin + world - 1) // world
    dev = torch.device(device)
    sink = _HostSink(dev) if rank == 0 else None
    wpb = max(1, int(windows_per_batch))
    for r0 in range(0, rounds, wpb):
        rr = list(range(r0, min(rounds, r0 + wpb)))
        ks = [r * world + rank for r in rr if r * world + rank < nwin]
        d = None
        if ks:
            idx = [window_frame_indices(k, n) for k in ks]
            uniq = sorted(set(i for row in idx for i in row))
            pre = io.preprocess(frames[uniq].to(dev), size)
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
        # every rank takes part in every round's gather (a rank without a window sends zeros)
        buf = torch.zeros(len(rr), INFER_LEN, h, w, dtype=torch.float32, device=dev)
        if d is not None:
            buf[:len(ks)] = d
        bufs = _gather_round(buf, rank, world, group)
        if rank == 0:
            for src in range(world):
                for j, r in enumerate(rr):
                    k = r * world + src
                    if k < nwin:
                        sink.put(k, bufs[src][j])
    if rank != 0:
        return None, target_fps
    out = sink.result()
    depth_list = []
    for k in range(nwin):
        depth_list += list(out[k])
    return stitch(depth_list, n), target_fps

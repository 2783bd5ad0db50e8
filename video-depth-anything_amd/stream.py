"""Streaming (per-frame) depth: ``infere_single_image`` of the reference fork, on any engine.

Mirrors ``VideoDepthAnything.infere_single_image`` (video_depth.py:91-327).  Every new frame is
encoded alone (T=1 through the DINOv2 encoder and the DPT reassemble), its four reassembled maps
are kept in a feature store of ``inference_length + max(keyframe_list) - 1`` slots, and the
temporal head runs over a context of ``inference_length - 1`` stored frames plus the new one.
Depth is produced for the new frame, and, with ``align_each_new_frame``, also for the context's
alignment frames, which fix a least-squares scale/shift against the depths already emitted.

Host/device split:

* the slot schedule (which stored frames form each context, which of them are alignment frames)
  is pure index bookkeeping, computed once on the host (``StreamSchedule``), a restatement of
  video_depth.py:153-190;
* the feature store lives on the device.  The reference keeps it ordered by shifting every slot
  down one place per frame once it is full (``features[:-1] = features[move]``, :299-307); here
  the store keeps a logical->physical slot map instead, so a shift is a host list operation and
  no feature bytes move;
* the engine does the model work: ``motion_features(x[1,3,H,W]) -> 4 maps`` and
  ``predict(x, context_maps, pred_idx, T, skip_tmp_block) -> (depth[P+1,H,W] fp32, 4 maps)``.
  ``VideoDepthAnything`` provides the libvda engine; ``oracle/vda_oracle.StreamEngine`` is the
  CPU checker used by the tests.

The reference's default configuration (``keyframe_list=[0, 12]`` with alignment) indexes feature
slot ``inference_length`` out of a context of ``inference_length - 1`` rows at the first
prediction and raises ``IndexError`` (dpt_temporal.py:189); this driver reproduces that error
rather than inventing a fix.  Without alignment the same schedule reads never-written slots,
which hold zeros in the reference (``torch.zeros``, :227-230) and here too.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from .video import DeviceIO, compute_scale_and_shift, net_input_size


@dataclass
class StreamSchedule:
    """Slot bookkeeping of video_depth.py:153-190 for one (inference_length, keyframe_list)."""
    length: int
    keyframes: List[int]
    n_slots: int
    contexts: List[List[int]]     # per warm-up prediction: the stored slots feeding the temporal head
    align: List[List[int]]        # per warm-up prediction: context positions used for alignment
    drop_slot: int = 1            # the slot the reference's shift discards (move list skips index 1)

    @classmethod
    def build(cls, length: int, keyframes: Sequence[int]) -> "StreamSchedule":
        keyframes = list(keyframes)
        kmax = max(keyframes)
        nk = len(keyframes)
        # distance of each keyframe from the batch end, and its slot while the store is filling
        dist = [kf + (length - nk) for kf in keyframes]
        fixed = [length - kf if length > kf else j + 1 for j, kf in enumerate(keyframes)]
        if len(fixed) != len(set(fixed)):
            raise AssertionError(f"Setup leads to duplicates in the keyframes: {fixed}")
        contexts, align = [], []
        for f in range(length - 1, length + kmax):
            ctx = list(range(f - (length - 1), f))
            ctx[0] = 0  # the first frame always stays in the context
            al = [0]
            for j, s in enumerate(fixed):
                if s in ctx:
                    al.append(ctx.index(s))
                else:
                    al.append(j + 1)
                    ctx[j + 1] = max(s, f - dist[j])
            contexts.append(ctx)
            align.append(al)
        return cls(length, keyframes, length + kmax - 1, contexts, align)


class FeatureStore:
    """Device store of the four reassembled maps per frame, ``n_slots`` logical slots.

    ``slot_map[logical] = physical`` row of the backing tensors; zero-initialised like the
    reference's ``torch.zeros`` buffers."""

    def __init__(self, n_slots: int, like: Sequence[torch.Tensor]):
        self.n = n_slots
        self.bufs = [torch.zeros((n_slots,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device) for t in like]
        self.slot_map = list(range(n_slots))

    def put(self, logical: int, maps: Sequence[torch.Tensor]):
        p = self.slot_map[logical]
        for b, t in zip(self.bufs, maps):
            b[p].copy_(t[0])

    def shift_in(self, maps: Sequence[torch.Tensor], drop: int = 1):
        """features[:-1] = features[[s for s in range(n) if s != drop]]; features[-1] = new."""
        freed = self.slot_map[drop]
        self.slot_map = self.slot_map[:drop] + self.slot_map[drop + 1:] + [freed]
        self.put(self.n - 1, maps)

    def gather(self, logical: Sequence[int]):
        bad = [i for i in logical if not -self.n <= i < self.n]
        if bad:  # the reference's features_f[use_feature_idx] (video_depth.py:241-244) raises the same
            raise IndexError(f"index {bad[0]} is out of bounds for dimension 0 with size {self.n}")
        idx = torch.tensor([self.slot_map[i] for i in logical], dtype=torch.long, device=self.bufs[0].device)
        return tuple(b.index_select(0, idx) for b in self.bufs)


def infere_single_image(engine, frames, target_fps, input_size: int = 518, device="cuda", warmup: bool = True,
                        inference_length: int = 32, keyframe_list=(0, 12), align_each_new_frame: bool = True,
                        skip_tmp_block: bool = False, io=DeviceIO):
    """Per-frame depth for ``frames`` (uint8 [N, h, w, 3]); returns (depth [N', h, w] float32, fps).

    video_depth.py:91-327: frames 0..L-2 only fill the feature store; from frame L-1 on every frame
    is predicted.  With alignment the first prediction emits the whole context's depths, later
    ones emit the new frame scaled/shifted onto the alignment frames, and the first emitted frame
    is dropped from the result (:322-323); without it one depth per predicted frame is emitted.
    """
    if not warmup:
        raise NotImplementedError  # video_depth.py:318-319
    if not isinstance(frames, torch.Tensor):
        frames = torch.from_numpy(np.ascontiguousarray(frames))
    n = int(frames.shape[0])
    fh, fw = int(frames.shape[1]), int(frames.shape[2])
    size = net_input_size(fh, fw, input_size)
    L = int(inference_length)
    sch = StreamSchedule.build(L, keyframe_list)
    kmax = max(sch.keyframes)
    dev = torch.device(device)
    store: Optional[FeatureStore] = None
    depth_list: List[np.ndarray] = []
    emitted_first = False
    for i in range(n):
        x = io.preprocess(frames[i:i + 1].to(dev), size)  # [1, 3, H, W]
        if i < L - 1:
            maps = engine.motion_features(x)
            if store is None:
                store = FeatureStore(sch.n_slots, maps)
            store.put(i, maps)
            continue
        pred_idx = None
        abs_idx: List[int] = []
        if i < L + kmax:
            step = i - (L - 1)
            ctx = sch.contexts[step]
            if align_each_new_frame:
                # store not shifted yet: logical slot == absolute frame index
                abs_idx = [ctx[t] for t in sch.align[step]]
                pred_idx = list(ctx) if i == L - 1 else list(sch.align[step])
        else:
            ctx = sch.contexts[-1]
            if align_each_new_frame:
                pred_idx = list(sch.align[-1])
                # the store has shifted (i - (L + kmax) + 1) times since the schedule's last row
                abs_idx = [0 if s == 0 else s + (i - (L + kmax)) + 1 for s in (ctx[t] for t in sch.align[-1])]
        if pred_idx is not None and max(pred_idx) >= len(ctx):
            # what the reference's layer_1_old[pred_depth_idx] does (dpt_temporal.py:189)
            raise IndexError(f"index {max(pred_idx)} is out of bounds for dimension 0 with size {len(ctx)}")
        depth, maps = engine.predict(x, store.gather(ctx), pred_idx, L, skip_tmp_block)
        if i < L + kmax - 1:
            store.put(i, maps)
        else:
            store.shift_in(maps, sch.drop_slot)
        d = io.resize_depth(depth, (fh, fw)).cpu().numpy()
        if not align_each_new_frame or not emitted_first:
            depth_list += [d[k] for k in range(d.shape[0])]
            emitted_first = True
            continue
        cur = d[-1]
        cur_kf = [d[k] for k in range(len(pred_idx))]
        old_kf = [depth_list[j] for j in abs_idx]
        scale, shift = compute_scale_and_shift(np.concatenate(cur_kf), np.concatenate(old_kf),
                                               np.concatenate(np.ones_like(old_kf) == 1))
        depth_list.append(cur * scale + shift)
    if align_each_new_frame:
        return np.stack(depth_list[1:n], axis=0), target_fps
    return np.stack(depth_list[:n], axis=0), target_fps

"""Video I/O and output formats around the depth path (utils/dc_utils.py:19-89, run.py:150-166).

The reference decodes with decord (or cv2) and encodes mp4 with imageio/ffmpeg; none of those is
installed in this image, so this module keeps the reference's *semantics* and supplies decoders
and encoders that need only numpy / Pillow:

* ``read_video_frames(path, process_length, target_fps=-1, max_res=-1) -> (frames uint8 [N,h,w,3], fps)``
  (dc_utils.py:19-69).  Containers: YUV4MPEG2 ``.y4m`` (uncompressed 4:2:0 / 4:2:2 / 4:4:4 / mono,
  the format ffmpeg emits with ``-f yuv4mpegpipe``), ``.npy`` / ``.npz`` frame stacks, animated
  GIF / PNG / WebP / multi-page TIFF and directories of images via Pillow; compressed containers
  (.mp4 ...) go through decord when it is importable.  Frame stride = max(round(source_fps / target_fps), 1); at most
  ``process_length`` frames; ``max_res`` scales the longer side down (decord branch: sizes rounded
  and made even, dc_utils.py:22-29).
* ``save_video(frames, path, fps, is_depths, grayscale, spectral)`` (dc_utils.py:72-89): depth is
  min/max-normalised to uint8 over the whole clip and mapped through matplotlib's inferno (or
  Spectral) table; written as ``.y4m`` (4:4:4), or animated GIF / PNG / WebP via Pillow; ``.mp4``
  needs imageio + ffmpeg and raises a clear error without them.
* ``save_npz`` (``depths`` key, run.py:162-164) and ``save_tiff`` (float32 multi-page, :165-166).

YUV <-> RGB uses BT.601 limited range (ffmpeg's default for SD/unknown-matrix y4m); decoded frames
of the reference's decord path are therefore parity-unpinned here (no decoder to compare with).
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np

_IMG_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".webp", ".tif", ".tiff")


def ensure_even(v: int) -> int:
    return v if v % 2 == 0 else v + 1


# ---- YUV4MPEG2 -------------------------------------------------------------------------------
def _yuv_to_rgb(y: np.ndarray, u: np.ndarray, v: np.ndarray) -> np.ndarray:
    """BT.601 limited range -> RGB uint8 (planes already at luma resolution)."""
    yf = (y.astype(np.float32) - 16.0) * (255.0 / 219.0)
    uf = (u.astype(np.float32) - 128.0) * (255.0 / 224.0)
    vf = (v.astype(np.float32) - 128.0) * (255.0 / 224.0)
    r = yf + 1.402 * vf
    g = yf - 0.344136 * uf - 0.714136 * vf
    b = yf + 1.772 * uf
    return np.clip(np.rint(np.stack([r, g, b], -1)), 0, 255).astype(np.uint8)


def _rgb_to_yuv(rgb: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    f = rgb.astype(np.float32)
    r, g, b = f[..., 0], f[..., 1], f[..., 2]
    y = 0.299 * r + 0.587 * g + 0.114 * b
    u = (b - y) / 1.772
    v = (r - y) / 1.402
    q = lambda a: np.clip(np.rint(a), 0, 255).astype(np.uint8)  # noqa: E731
    return q(y * (219.0 / 255.0) + 16.0), q(u * (224.0 / 255.0) + 128.0), q(v * (224.0 / 255.0) + 128.0)


def _parse_ratio(s: str) -> float:
    a, b = s.split(":")
    return float(a) / float(b) if float(b) else 0.0


def read_y4m(path: str) -> Tuple[np.ndarray, float]:
    """All frames of a YUV4MPEG2 file as RGB uint8 [N, h, w, 3], plus its frame rate."""
    with open(path, "rb") as f:
        data = f.read()
    nl = data.index(b"\n")
    head = data[:nl].decode("ascii").split()
    if not head or head[0] != "YUV4MPEG2":
        raise ValueError(f"{path}: not a YUV4MPEG2 stream")
    w = h = None
    fps, cs = 25.0, "420"
    for tok in head[1:]:
        k, val = tok[0], tok[1:]
        if k == "W":
            w = int(val)
        elif k == "H":
            h = int(val)
        elif k == "F":
            fps = _parse_ratio(val)
        elif k == "C":
            cs = val
    if w is None or h is None:
        raise ValueError(f"{path}: y4m header lacks W/H")
    base = cs.split("p")[0]
    if base.startswith("420"):
        cw, ch = (w + 1) // 2, (h + 1) // 2
    elif base == "422":
        cw, ch = (w + 1) // 2, h
    elif base == "444":
        cw, ch = w, h
    elif base == "mono":
        cw = ch = 0
    else:
        raise ValueError(f"{path}: unsupported y4m colourspace C{cs} (8-bit 420/422/444/mono only)")
    fsz = w * h + 2 * cw * ch
    frames = []
    pos = nl + 1
    while pos < len(data):
        e = data.index(b"\n", pos)
        if not data[pos:e].startswith(b"FRAME"):
            raise ValueError(f"{path}: corrupt frame header at byte {pos}")
        pos = e + 1
        buf = np.frombuffer(data, np.uint8, fsz, pos)
        pos += fsz
        y = buf[:w * h].reshape(h, w)
        if cw == 0:
            u = v = np.full((h, w), 128, np.uint8)
        else:
            u = buf[w * h:w * h + cw * ch].reshape(ch, cw)
            v = buf[w * h + cw * ch:].reshape(ch, cw)
            ry, rx = (2 if ch != h else 1), (2 if cw != w else 1)  # nearest chroma upsampling
            u = np.repeat(np.repeat(u, ry, 0), rx, 1)[:h, :w]
            v = np.repeat(np.repeat(v, ry, 0), rx, 1)[:h, :w]
        frames.append(_yuv_to_rgb(y, u, v))
    if not frames:
        return np.zeros((0, h, w, 3), np.uint8), fps
    return np.stack(frames), fps


def write_y4m(path: str, frames: np.ndarray, fps: float):
    """RGB (or grey) uint8 frames -> YUV4MPEG2 4:4:4 (C444), BT.601 limited range."""
    frames = np.asarray(frames)
    if frames.ndim == 3:
        frames = np.repeat(frames[..., None], 3, -1)
    n, h, w, _ = frames.shape
    num, den = (int(round(fps * 1001)), 1001) if abs(fps * 1001 - round(fps * 1001)) < 1e-6 else (int(round(fps * 1000)), 1000)
    with open(path, "wb") as f:
        f.write(f"YUV4MPEG2 W{w} H{h} F{num}:{den} Ip A1:1 C444\n".encode("ascii"))
        for i in range(n):
            y, u, v = _rgb_to_yuv(frames[i])
            f.write(b"FRAME\n")
            f.write(y.tobytes())
            f.write(u.tobytes())
            f.write(v.tobytes())


# ---- readers ---------------------------------------------------------------------------------
def _read_pillow(path: str) -> Tuple[np.ndarray, float]:
    from PIL import Image, ImageSequence
    if os.path.isdir(path):
        names = sorted(n for n in os.listdir(path) if n.lower().endswith(_IMG_EXT))
        frames = [np.asarray(Image.open(os.path.join(path, n)).convert("RGB")) for n in names]
        return np.stack(frames), 30.0
    im = Image.open(path)
    frames, dur = [], []
    for fr in ImageSequence.Iterator(im):
        frames.append(np.asarray(fr.convert("RGB")))
        dur.append(fr.info.get("duration", 0) or 0)
    d = float(np.mean(dur)) if dur and np.mean(dur) > 0 else 0.0
    return np.stack(frames), (1000.0 / d if d > 0 else 30.0)


def _resize_rgb(frames: np.ndarray, height: int, width: int) -> np.ndarray:
    from PIL import Image
    return np.stack([np.asarray(Image.fromarray(f).resize((width, height), Image.BICUBIC)) for f in frames])


def _read_all(path: str) -> Tuple[np.ndarray, float]:
    ext = os.path.splitext(path)[1].lower()
    if ext == ".y4m":
        return read_y4m(path)
    if ext == ".npy":
        return np.load(path, allow_pickle=False), 30.0
    if ext == ".npz":
        z = np.load(path, allow_pickle=False)
        fps = float(z["fps"]) if "fps" in z.files else 30.0
        return z["frames"], fps
    return _read_pillow(path)


def read_video_frames(video_path: str, process_length: int, target_fps: float = -1, max_res: int = -1):
    """dc_utils.py:19-69 semantics on the decoders available (module docstring)."""
    ext = os.path.splitext(video_path)[1].lower()
    if ext in (".mp4", ".mov", ".avi", ".mkv", ".webm"):
        try:
            import decord  # noqa: F401
        except ImportError:
            decord = None
        if decord is None:
            raise RuntimeError(f"{video_path}: compressed video needs decord or cv2, neither is installed; "
                               "convert it to .y4m (ffmpeg -i in.mp4 -f yuv4mpegpipe out.y4m) or a frame stack")
        vr = decord.VideoReader(video_path, ctx=decord.cpu(0))
        oh, ow = vr.get_batch([0]).shape[1:3]
        h, w = oh, ow
        if max_res > 0 and max(h, w) > max_res:
            s = max_res / max(oh, ow)
            h, w = ensure_even(round(oh * s)), ensure_even(round(ow * s))
        vr = decord.VideoReader(video_path, ctx=decord.cpu(0), width=w, height=h)
        src_fps = vr.get_avg_fps()
        fps = src_fps if target_fps == -1 else target_fps
        idx = list(range(0, len(vr), max(round(src_fps / fps), 1)))
        if process_length != -1 and process_length < len(idx):
            idx = idx[:process_length]
        return vr.get_batch(idx).asnumpy(), fps
    frames, src_fps = _read_all(video_path)
    if frames.ndim != 4 or frames.shape[-1] != 3 or frames.dtype != np.uint8:
        raise ValueError(f"{video_path}: expected uint8 frames [N, h, w, 3], got {frames.dtype} {frames.shape}")
    fps = src_fps if target_fps == -1 else target_fps
    idx = list(range(0, len(frames), max(round(src_fps / fps), 1)))
    if process_length != -1 and process_length < len(idx):
        idx = idx[:process_length]
    frames = frames[idx]
    oh, ow = frames.shape[1:3]
    if max_res > 0 and max(oh, ow) > max_res:
        s = max_res / max(oh, ow)
        frames = _resize_rgb(frames, ensure_even(round(oh * s)), ensure_even(round(ow * s)))
    return np.ascontiguousarray(frames), fps


# ---- writers ---------------------------------------------------------------------------------
def colorize_depths(depths: np.ndarray, grayscale: bool = False, spectral: bool = False) -> np.ndarray:
    """dc_utils.py:74-85: clip-wide min/max normalisation to uint8, then inferno / Spectral / grey."""
    d_min, d_max = depths.min(), depths.max()
    norm = ((depths - d_min) / (d_max - d_min) * 255).astype(np.uint8)
    if grayscale:
        return norm
    import matplotlib
    if spectral:
        return (matplotlib.colormaps["Spectral"](norm)[..., :3] * 255).astype(np.uint8)
    table = np.array(matplotlib.colormaps["inferno"].colors)
    return (table[norm] * 255).astype(np.uint8)


def save_video(frames: np.ndarray, output_video_path: str, fps: float = 10, is_depths: bool = False,
               grayscale: bool = False, spectral: bool = False):
    vis = colorize_depths(frames, grayscale, spectral) if is_depths else np.asarray(frames)
    ext = os.path.splitext(output_video_path)[1].lower()
    if ext == ".y4m":
        write_y4m(output_video_path, vis, fps)
        return
    if ext in (".gif", ".png", ".webp", ".apng"):
        from PIL import Image
        ims = [Image.fromarray(f) for f in vis]
        ims[0].save(output_video_path, save_all=True, append_images=ims[1:], duration=int(round(1000 / fps)), loop=0)
        return
    try:
        import imageio
    except ImportError as e:
        raise RuntimeError(f"{output_video_path}: mp4 output needs imageio + ffmpeg (not installed); use .y4m, .gif, "
                           ".png or .webp") from e
    writer = imageio.get_writer(output_video_path, fps=fps, macro_block_size=1, codec="libx264",
                                ffmpeg_params=["-crf", "18"])
    for f in vis:
        writer.append_data(f)
    writer.close()


def save_npz(path: str, depths: np.ndarray):
    np.savez_compressed(path, depths=depths)


def save_tiff(path: str, depths: np.ndarray):
    """float32 multi-page TIFF, one page per frame (run.py:165-166 writes one tifffile stack)."""
    from PIL import Image
    pages = [Image.fromarray(np.ascontiguousarray(d, dtype=np.float32), mode="F") for d in depths]
    pages[0].save(path, save_all=True, append_images=pages[1:])


def load_tiff(path: str) -> np.ndarray:
    from PIL import Image, ImageSequence
    return np.stack([np.asarray(p, dtype=np.float32) for p in ImageSequence.Iterator(Image.open(path))])


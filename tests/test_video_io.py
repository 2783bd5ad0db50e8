"""Video I/O and output formats (utils/dc_utils.py:19-89, run.py:150-166) on numpy / Pillow codecs."""
import os

import numpy as np
import pytest
import torch

from helpers import recipe_state_dict, REPO  # noqa: F401
from vda_amd import video_io as VIO


def _frames(n=12, h=30, w=44, seed=0):
    g = np.random.default_rng(seed)
    base = g.integers(0, 256, (1, h // 2, w // 2, 3)).repeat(2, 1).repeat(2, 2)  # 2x2-constant blocks
    return np.concatenate([np.roll(base, t, 2) for t in range(n)]).astype(np.uint8)


def test_y4m_444_round_trip(tmp_path):
    fr = _frames()
    p = str(tmp_path / "a.y4m")
    VIO.write_y4m(p, fr, 30000 / 1001)
    back, fps = VIO.read_y4m(p)
    assert back.shape == fr.shape and abs(fps - 29.97) < 1e-2
    assert np.abs(back.astype(int) - fr).max() <= 3  # 8-bit limited-range YUV quantisation


def test_y4m_420_reader(tmp_path):
    h, w = 6, 8
    y = np.full((h, w), 126, np.uint8)
    u = np.full((3, 4), 128, np.uint8)
    v = np.full((3, 4), 128, np.uint8)
    v[0, 0] = 200  # a red-shifted 2x2 block top-left
    p = tmp_path / "b.y4m"
    with open(p, "wb") as f:
        f.write(b"YUV4MPEG2 W8 H6 F25:1 Ip A1:1 C420jpeg XYSCSS=420JPEG\n")
        for _ in range(3):
            f.write(b"FRAME\n" + y.tobytes() + u.tobytes() + v.tobytes())
    fr, fps = VIO.read_y4m(str(p))
    assert fr.shape == (3, 6, 8, 3) and fps == 25
    assert (fr[:, :2, :2, 0] > fr[:, :2, :2, 1]).all()  # chroma replicated over its 2x2 block
    assert (fr[:, 2:, 2:, 0] == fr[:, 2:, 2:, 1]).all()  # neutral elsewhere (grey)


def test_read_video_frames_stride_length_maxres(tmp_path):
    fr = _frames(n=20, h=40, w=60)
    p = str(tmp_path / "c.npz")
    np.savez(p, frames=fr, fps=np.float64(30.0))
    out, fps = VIO.read_video_frames(p, -1, 15, -1)  # stride round(30/15) = 2
    assert fps == 15 and np.array_equal(out, fr[::2])
    out, _ = VIO.read_video_frames(p, 4, -1, -1)
    assert np.array_equal(out, fr[:4])
    out, fps = VIO.read_video_frames(p, 3, -1, 45)  # 60 -> 45: 40*0.75 = 30, 45 (even: 46)
    assert out.shape == (3, 30, 46, 3) and fps == 30
    with pytest.raises(RuntimeError):
        VIO.read_video_frames(str(tmp_path / "x.mp4"), -1)


def test_colorize_and_writers(tmp_path):
    d = np.linspace(0, 7, 5 * 12 * 16, dtype=np.float32).reshape(5, 12, 16)
    grey = VIO.colorize_depths(d, grayscale=True)
    assert grey.dtype == np.uint8 and grey.min() == 0 and grey.max() == 255
    inf = VIO.colorize_depths(d)
    spec = VIO.colorize_depths(d, spectral=True)
    assert inf.shape == spec.shape == (5, 12, 16, 3) and inf.dtype == np.uint8
    VIO.save_video(d, str(tmp_path / "v.y4m"), fps=10, is_depths=True)
    back, fps = VIO.read_y4m(str(tmp_path / "v.y4m"))
    assert back.shape == (5, 12, 16, 3) and fps == 10
    VIO.save_video(d, str(tmp_path / "v.gif"), fps=10, is_depths=True, grayscale=True)
    g, _ = VIO.read_video_frames(str(tmp_path / "v.gif"), -1)
    assert g.shape == (5, 12, 16, 3)
    VIO.save_npz(str(tmp_path / "d.npz"), d)
    assert np.array_equal(np.load(str(tmp_path / "d.npz"))["depths"], d)
    VIO.save_tiff(str(tmp_path / "d.tiff"), d)
    assert np.array_equal(VIO.load_tiff(str(tmp_path / "d.tiff")), d)
    with pytest.raises(RuntimeError):
        VIO.save_video(d, str(tmp_path / "v.mp4"), is_depths=True)


@pytest.mark.gpu
@pytest.mark.parametrize("single", [False, True])
def test_cli_end_to_end(tmp_path, single):
    """run.py on a .y4m clip (vits, synthetic weights) == the model's own driver on the decoded frames."""
    import sys
    sys.path.insert(0, REPO)
    import run as cli
    import vda_amd
    fr = _frames(n=40, h=42, w=56)
    p = str(tmp_path / "clip.y4m")
    VIO.write_y4m(p, fr, 24)
    args = ["--input_video", p, "--output_dir", str(tmp_path / "out"), "--encoder", "vits", "--input_size", "56",
            "--synthetic_weights", "--save_npz", "--save_tiff", "--save_vis"]
    if single:
        args += ["--process_single_image", "--keyframe_list", "2", "12", "--align_each_new_frame"]
    d = cli.main(args)
    name = ("Single_" if single else "") + "VideoDepthAny_vits_clip"
    npz = np.load(str(tmp_path / "out" / (name + "_depths.npz")))["depths"]
    assert np.array_equal(npz, d)
    assert os.path.exists(str(tmp_path / "out" / (name + "_vis.y4m")))
    frames, fps = VIO.read_video_frames(p, -1, -1, 1280)
    m = vda_amd.build_model("vits", device="cuda")
    if single:
        ref, _ = m.infere_single_image(frames, fps, input_size=56, keyframe_list=[2, 12], align_each_new_frame=True)
    else:
        ref, _ = m.infer_video_depth(frames, fps, input_size=56)
    assert d.shape == ref.shape == ((39 if single else 40), 42, 56)
    assert np.abs(d - ref).max() <= 1e-6 * max(1.0, np.abs(ref).max())


@pytest.mark.gpu
def test_cli_on_reference_golden_video(tmp_path):
    """run.py end to end vs the REFERENCE's own infer_video_depth output (tests/golden/video_vits_57f.npz,
    made by tests/golden/make_golden.py): the golden's frames as a .npz frame stack -> run.py -> npz."""
    import sys
    sys.path.insert(0, REPO)
    import json
    import run as cli
    z = np.load(os.path.join(REPO, "tests", "golden", "video_vits_57f.npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    p = str(tmp_path / "golden.npz")
    np.savez(p, frames=z["frames"], fps=np.float64(meta["fps"]))
    out = tmp_path / "out"
    d = cli.main(["--input_video", p, "--output_dir", str(out), "--encoder", meta["encoder"], "--input_size",
                  str(meta["input_size"]), "--synthetic_weights", "--save_npz"])
    npz = np.load(str(out / "VideoDepthAny_vits_golden_depths.npz"))["depths"]
    assert np.array_equal(npz, d) and d.shape == z["depth"].shape
    err = float(np.abs(d - z["depth"]).sum() / np.abs(z["depth"]).sum())
    print(f"run.py on the reference golden video: rel-L1 = {err:.3e}")
    assert err <= 1e-3


@pytest.mark.gpu
def test_cli_single_image_wins_over_original(tmp_path):
    """--process_single_image is checked before --original (reference run.py:93-100): the streaming
    driver runs and the outputs are named Single_*."""
    import sys
    sys.path.insert(0, REPO)
    import run as cli
    fr = _frames(n=36, h=42, w=56)
    p = str(tmp_path / "clip.y4m")
    VIO.write_y4m(p, fr, 24)
    base = ["--input_video", p, "--encoder", "vits", "--input_size", "56", "--synthetic_weights", "--save_npz",
            "--process_single_image", "--keyframe_list", "2", "12", "--align_each_new_frame"]
    d1 = cli.main(base + ["--output_dir", str(tmp_path / "a")])
    d2 = cli.main(base + ["--output_dir", str(tmp_path / "b"), "--original"])
    assert d1.shape == d2.shape == (35, 42, 56)  # the streaming driver's frame count
    assert np.array_equal(d1, d2)
    assert os.path.exists(str(tmp_path / "b" / "Single_VideoDepthAny_vits_clip_depths.npz"))

"""bench.py's multi-rank plumbing on the CPU (gloo, world size 2), through the real spawn path:
``python bench.py --gpus 2`` (no WORLD_SIZE) re-launches itself under torch.distributed.run with two
ranks, which count devices, run the (stand-in) clip forward, gather each step's depth to rank 0,
take the max over ranks and print one JSON line.  ``--dry-run`` swaps the HIP forward for a CPU
stand-in, so the numbers are not measurements; the GPU path is covered by the bench runs themselves."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("OMP_NUM_THREADS", "2")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", *args], capture_output=True,
                       text=True, timeout=300, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 prints exactly one line
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_spawns_ranks_and_gathers(gpus):
    d = run_bench("--gpus", str(gpus), "--steps", "3", "--warmup", "1", "--frames", "4", "--size", "28", "28")
    assert d["config"]["ranks"] == gpus and d["n_gpus"] == gpus
    assert d["config"]["depth_gather_to_rank0"] == (gpus > 1)
    assert d["steps"] == 3 and d["unit"] == "frames/s" and d["scaling"] == "weak"
    assert abs(d["value"] - gpus * 3 * 4 / (d["ms_per_step"] * 3 / 1e3)) / d["value"] < 0.01


def test_bench_video_mode_two_ranks():
    d = run_bench("--gpus", "2", "--video", "--video-frames", "30", "--steps", "1", "--warmup", "0",
                  "--size", "28", "28")
    assert d["config"]["windows"] == 2 and d["scaling"] == "strong" and d["unit"] == "video frames/s"


def test_bench_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dry-run", "--gpus", "4"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=REPO)
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr

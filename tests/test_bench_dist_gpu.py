"""bench.py's N-rank path (config 5) run end to end on one GPU:
`--gpus 2 --dist-transport host` launches two ranks under
torch.distributed.run, both on the box's GPU, with the start-up exchange on
the host-staged gf_dist transport (gloo). Every line of the world > 1 branch
runs (relaunch, world / vocabulary / map broadcasts, checksum all-reduces,
the barrier + max-over-ranks timing, the per-rank gather); RCCL itself at
world > 1 needs one GPU per rank (the driver's 8-GPU run)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_host_transport(tmp_path):
    B, steps = 64, 3
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--dist-transport", "host", "--batch", str(B), "--groups", "2",
           "--steps", str(steps), "--warmup", "1", "--scenes", "4", "--keyframes", "8", "--no-cpu-baseline",
           "--lba-batch", "0", "--single-stream-steps", "0", "--isolated-steps", "0", "--budget-steps", "0",
           "--pcie-steps", "0", "--config3-steps", "0", "--kernel-times", "events", "--time-log-steps", "4",
           "--time-log", str(tmp_path / "tl.txt"), "--detail-out", str(tmp_path / "detail.json")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == steps
    rk = line["ranks"]
    assert rk["world"] == 2 and rk["communicator_world"] == 2 and rk["transport"] == "host"
    assert len(rk["frames_per_s"]) == 2 and min(rk["frames_per_s"]) > 0
    assert line["startup_checksums_equal"] is True
    # value = frames of all ranks / the max over ranks of the timed wall time
    d = json.load(open(tmp_path / "detail.json"))
    ms = max(d["ranks"]["ms_per_step"])
    assert abs(line["value"] - 2 * B * steps / (ms * steps / 1e3)) <= 0.01 * line["value"]
    assert rk["min_frames_per_s"] <= rk["max_frames_per_s"]
    assert d["config"]["distinct_frames_per_step"] == B  # 4 scenes x 32 phases >= 64 streams
    tl = open(tmp_path / "tl.txt").read().splitlines()
    assert tl[0].startswith("#frame_time_stamp") and len(tl) == 5

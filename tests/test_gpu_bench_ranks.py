"""The N-rank bench path with real GPU work (BASELINE config 5's 1 -> 8 GPU curve).

`bench.py --gpus 2` spawns one rank process per GPU (before anything touches a GPU), the ranks meet over gloo
for the timing reduction only, and each extracts its own frames: the reference's only concurrency, the per-frame
extraction threads of Frame.cc:124-127, becomes frame sharding with no data-path collective.  On a one-GPU box
ORBGPU_BENCH_ONE_DEVICE=1 puts both ranks on device 0, so the whole path -- spawn, rendezvous, extraction on the
GPU, max / sum reduction, the rank-0 JSON line -- runs as the driver's multi-GPU run will.  The bench runs as a
fresh child process (never an exec of this one)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config,frames_per_rank", [("c3", 256), ("c5", 4)])
def test_bench_two_ranks_one_device(config, frames_per_rank):
    env = dict(os.environ, ORBGPU_BENCH_ONE_DEVICE="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--only-extract",
                        "--steps", "5", "--warmup", "2", "--config", config],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5
    ranks = sorted(d["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == [0, 1]
    assert all(x["device"] == 0 for x in ranks)   # (ORBGPU_BENCH_ONE_DEVICE)
    assert all(x["frames_per_step"] == frames_per_rank for x in ranks)
    # disjoint frames: rank r extracts frames [first, first + B)
    a, b = ranks
    assert a["first_frame"] + a["frames_per_step"] <= b["first_frame"] or \
        b["first_frame"] + b["frames_per_step"] <= a["first_frame"]
    assert all(x["keypoints_per_step"] > 1000 * frames_per_rank for x in ranks)
    # value = every rank's keypoints over the slowest rank's time (the line rounds each rank's time to 1 us: a
    # 5-step C5 run lasts well under a millisecond, hence the relative tolerance)
    tmax = max(x["seconds"] for x in ranks)
    want = sum(x["keypoints_per_step"] for x in ranks) * d["steps"] / tmax
    assert abs(d["value"] - want) <= 5e-6 / tmax * want + 1.0, (d["value"], want)
    assert d["config"]["global_batch"] == 2 * frames_per_rank

"""N>1 path of bench.py on CPU (gloo, world size 2): frames shard across ranks with no overlap, and
the timing reduction takes the max time / summed keypoints the driver's contract asks for.  The data
path has no collective — gloo carries only the barrier and the two reductions."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import bench
    r, w, local = bench.dist_env()
    dist = bench.dist_init(w)
    first, count = bench.frame_range(r, 16)
    bench.barrier(dist)
    tmax, ksum = bench.reduce_max_sum(dist, 1.0 + r, 100.0 * (r + 1))
    _, fsum = bench.reduce_max_sum(dist, 0.0, float(count))
    q.put((r, local, first, count, tmax, ksum, fsum))
    dist.destroy_process_group()


def test_two_rank_sharding_and_reduction():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(2))
    (r0, l0, f0, c0, t0, k0, s0), (r1, l1, f1, c1, t1, k1, s1) = res
    assert (r0, r1) == (0, 1) and (l0, l1) == (0, 1)        # one process per GPU: local rank = device
    assert f0 + c0 <= f1 and c0 == c1 == 16                  # disjoint synthetic frames per rank
    assert t0 == t1 == 2.0                                   # max over ranks
    assert k0 == k1 == 300.0 and s0 == s1 == 32.0            # whole-job sums


def test_single_rank_needs_no_process_group():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.dist_init(1) is None
    assert bench.reduce_max_sum(None, 3.0, 5.0) == (3.0, 5.0)


def _bench_line(out):
    import json
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_flag_spawns_the_ranks_itself():
    """`python bench.py --gpus 2` with no launcher: bench.py starts both ranks before any GPU call, they
    rendezvous on 127.0.0.1 over gloo, and rank 0 alone prints the line with every rank's device."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _bench_line(r.stdout)
    assert d["n_gpus"] == 2
    assert [x["rank"] for x in d["ranks"]] == [0, 1] and [x["device"] for x in d["ranks"]] == [0, 1]
    assert d["value"] == 300.0 / 2.0          # summed work over the max time


def test_launcher_world_must_match_gpus_flag():
    import subprocess
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in (r.stderr + r.stdout)

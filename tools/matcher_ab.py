#!/usr/bin/env python3
"""A/B of the matcher drop-ins' per-call latency (bench.py's matcher leg, tools/matcher_latency) at C2 and C3 under
the environment variants given as arguments (NAME=VALUE,...; "-" = as is)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
import bench  # noqa: E402
from orbgpu.synth import bench_frames  # noqa: E402

for spec in sys.argv[1:] or ["-"]:
    env = {} if spec == "-" else dict(kv.split("=", 1) for kv in spec.split(","))
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    for (w, h, nf) in ((640, 480, 1000), (1280, 720, 2000)):
        out = bench.matcher_leg(bench_frames(w, h, 1)[0], w, h, nf, 0)
        row = {k: (v.get("gpu_us"), v.get("cpu_us"), v.get("equal")) for k, v in out.items() if isinstance(v, dict) and "gpu_us" in v}
        print(json.dumps({"env": spec, "size": f"{w}x{h}/{nf}", "calls": row}), flush=True)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v

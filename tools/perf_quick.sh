#!/bin/bash
# Quick performance check (GPU box): C3 extraction kernels + host path, C5 at one frame per step with
# four in flight (north_star's N = 8 shard per GPU).  Each step has its own limit; stops at the first failure.
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu --no-hamming --no-stereo --no-bird --no-c4 --no-matcher > $OUT/pq_c3.log 2>&1 || { tail -20 $OUT/pq_c3.log; exit 1; }
timeout -k 10 300 python bench.py --config c5 --batch 1 --pipelines 4 --steps 200 --warmup 20 --only-extract > $OUT/pq_c5b1.log 2>&1 || { tail -20 $OUT/pq_c5b1.log; exit 1; }
timeout -k 10 300 python bench.py --config c5 --steps 50 --warmup 5 --only-extract > $OUT/pq_c5.log 2>&1 || { tail -20 $OUT/pq_c5.log; exit 1; }
python3 - <<'PY'
import json
for n in ("pq_c3", "pq_c5b1", "pq_c5"):
    d = json.loads([l for l in open(f"gpurun_out/{n}.log") if l.startswith("{")][-1])
    hp = d.get("host_path") or {}
    print(n, "value %.1f M" % (d["value"] / 1e6), "ms/step", d["ms_per_step"], "kernels", d.get("kernels_ms_per_step"),
          "host_path_ms", hp.get("ms_per_frame"))
PY

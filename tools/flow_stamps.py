#!/usr/bin/env python3
"""Where the dataflow launch (k_extract_flow) spends its time (diagnostic, GPU): runs one-frame C5 launches with
ORBGPU_FLOW_STAMPS=1 and prints, per stage and level, when its tasks started and ended (us after the launch's first
ticket) and how long they waited and ran.  Usage: tools/flow_stamps.py [frames per launch] [features] [blocks]"""
import os
import sys

os.environ["ORBGPU_FLOW_STAMPS"] = "1"
os.environ.setdefault("ORBGPU_FLOW", "1")
if len(sys.argv) > 3:
    os.environ["ORBGPU_FLOW_BLOCKS"] = sys.argv[3]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
import numpy as np  # noqa: E402

import orbgpu  # noqa: E402
from orbgpu.synth import bench_frames  # noqa: E402

KINDS = ["resize", "fast", "octree", "describe", "chain"]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    NF = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    bx = orbgpu.BatchExtractor(NF, 1280, 720, B)
    bx.upload(bench_frames(1280, 720, B))
    runs = []
    for _ in range(20):
        bx.launch()
        bx.sync()
        cap = 4 * 4096
        st = np.zeros(cap, np.uint64)
        n = orbgpu._lib.lib().orb_debug_fast_stamps(bx.h, st.ctypes.data, cap)
        runs.append(st[:n].reshape(-1, 4).astype(np.int64))
    ids = runs[0][:, 3]
    nt = int(np.count_nonzero(ids))   # (tasks past ntasks are zero)
    spans, rows = [], {}
    for r in runs[5:]:
        r = r[:nt]
        t0 = r[:, 0].min()
        spans.append((r[:, 2].max() - t0) / 100.0)
        for i in range(nt):
            klf = int(r[i, 3]) & 0xFFFFFFFF
            key = (KINDS[klf & 0xFF], (klf >> 8) & 0xFF)
            rows.setdefault(key, []).append(((r[i, 0] - t0) / 100.0, (r[i, 1] - t0) / 100.0, (r[i, 2] - t0) / 100.0))
    blocks = len(set(int(x) >> 32 for x in ids[:nt]))
    print(f"tasks {nt}  workgroups used {blocks}  launch span (first ticket -> last done) median {np.median(spans):.1f} us"
          f"  min {np.min(spans):.1f}")
    print(f"{'stage':9s} lv  tasks  ticket..   start..end (us, medians over runs)   wait  run")
    for (k, lv), v in sorted(rows.items(), key=lambda kv: np.median([x[1] for x in kv[1]])):
        v = np.array(v)
        ntask = len(v) // (len(runs) - 5)
        print(f"{k:9s} {lv:2d} {ntask:5d}  {np.median(v[:, 0]):6.1f}  {np.min(v[:, 1]):6.1f}..{np.max(v[:, 2]):6.1f}"
              f"   {np.median(v[:, 1] - v[:, 0]):5.1f} {np.median(v[:, 2] - v[:, 1]):5.1f}")
    bx.close()


if __name__ == "__main__":
    main()

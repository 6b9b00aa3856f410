#!/usr/bin/env python3
"""Where a k_fast_wave wavefront spends its time (diagnostic, GPU): runs one C3 batch with
ORBGPU_FAST_STAMPS=1 and prints the mean s_memtime cycles of each phase per (frame, cell) wave,
overall and per pyramid level.  Phases: ROI wait + LDS store, score-map zeroing, prefilter +
compaction, exact arc strength, NMS (+ fallback), emission.
Needs a library built with kernel stamps: make -B -C orb-slam-birdview_amd STAMPS=1 (then make -B again without it)."""
import os
import sys

os.environ["ORBGPU_FAST_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
import numpy as np  # noqa: E402

import orbgpu  # noqa: E402
from orbgpu.synth import synth_batch  # noqa: E402


def main():
    B = 64
    bx = orbgpu.BatchExtractor(2000, 1280, 720, B)
    bx.upload(synth_batch(1280, 720, B))
    for _ in range(3):
        bx.launch()
    bx.sync()
    L = orbgpu._lib.lib()
    cap = 8 * 2656 * B
    st = np.zeros(cap, np.uint64)
    n = L.orb_debug_fast_stamps(bx.h, st.ctypes.data, cap)
    st = st[:n].reshape(-1, 8).astype(np.int64)
    st = st[:, [0, 6, 1, 2, 3, 4, 5]]   # slot 6 = end of the cell decode
    valid = (st[:, 6] > st[:, 0]) & (st[:, 0] > 0) & (st[:, 1] >= st[:, 0])
    d = np.diff(st[valid], axis=1)
    names = ["roi_wait_store", "zero_maps", "prefilter", "arc_strength", "nms", "emission"]
    print("waves", int(valid.sum()), "mean lifetime cycles", round(float((st[valid, 6] - st[valid, 0]).mean()), 1))
    for i, nm in enumerate(names):
        print(f"  {nm:14s} {d[:, i].mean():9.1f}  p50 {np.median(d[:, i]):9.1f}  p90 {np.percentile(d[:, i], 90):9.1f}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where a k_describe wavefront spends its time (diagnostic, GPU): runs one C3 batch with
ORBGPU_FAST_STAMPS=1 and prints the mean s_memtime cycles of each phase per keypoint wave:
window load, IC angle, blur row pass, blur column pass, sin/cos, BRIEF tests + output.
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
    B, NL, NCELLS = 64, 8, 2656
    bx = orbgpu.BatchExtractor(2000, 1280, 720, B)
    bx.upload(synth_batch(1280, 720, B))
    for _ in range(3):
        bx.launch()
    bx.sync()
    L = orbgpu._lib.lib()
    kcap = bx.kp_cap
    off = B * (NCELLS * 8 + NL * 32)
    cap = off + B * kcap * 8
    st = np.zeros(cap, np.uint64)
    n = L.orb_debug_fast_stamps(bx.h, st.ctypes.data, cap)
    assert n >= cap, (n, cap)
    d = st[off:].reshape(-1, 8).astype(np.int64)
    ok = (d[:, 0] > 0) & (d[:, 6] >= d[:, 0])
    d = d[ok]
    ph = np.diff(d[:, :7], axis=1)
    names = ["window", "ic_angle", "row_pass", "col_pass", "sincos", "brief_out"]
    print("waves", len(d), "mean lifetime", round(float((d[:, 6] - d[:, 0]).mean()), 1), "cycles")
    for i, nm in enumerate(names):
        print(f"  {nm:10s} {ph[:, i].mean():9.1f}  p50 {np.median(ph[:, i]):9.1f}  p90 {np.percentile(ph[:, i], 90):9.1f}")
    span = (d[:, 6].max() - d[:, 0].min())
    print("kernel span (cycles)", int(span))


if __name__ == "__main__":
    main()

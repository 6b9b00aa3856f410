#!/usr/bin/env python3
"""Birdview stream timing (diagnostic, GPU): orb_bird_extract_device on one resident 1280x720 frame +
mask, N calls; prints ms per call.  Run under `rocprofv3 --kernel-trace --stats` for the kernel split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
import numpy as np  # noqa: E402

import orbgpu  # noqa: E402
from orbgpu.synth import synth_bird_mask, synth_frame  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    w, h = 1280, 720
    img, mask = synth_frame(w, h, 3), synth_bird_mask(w, h, 3)
    bx = orbgpu.BatchExtractor(2000, w, h, 1)
    L = orbgpu._lib.lib()
    di, dm = bx._alloc(w * h), bx._alloc(w * h)
    orbgpu._lib.check(L.orb_memcpy_h2d(bx.h, di, img.ctypes.data, w * h))
    orbgpu._lib.check(L.orb_memcpy_h2d(bx.h, dm, mask.ctypes.data, w * h))
    b = orbgpu.BirdORB(2000)
    for _ in range(3):
        b.extract_device(di, w, h, dm)
    t0 = time.perf_counter()
    for _ in range(n):
        k, d = b.extract_device(di, w, h, dm)
    t1 = time.perf_counter()
    print(f"bird extract: {(t1 - t0) / n * 1e3:.3f} ms/frame, {len(k)} keypoints")


if __name__ == "__main__":
    main()

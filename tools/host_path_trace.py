#!/usr/bin/env python3
"""Per-frame host-path latency breakdown (diagnostic, GPU): ORBextractor on host images one frame at
a time, as Frame::ExtractORB calls it.  Run under rocprofv3 --kernel-trace to see kernel times vs gaps."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
import orbgpu  # noqa: E402
from orbgpu.synth import synth_batch  # noqa: E402

frames = synth_batch(1280, 720, 8)
ex = orbgpu.ORBextractor(2000, 1.2, 8, 20, 7)
for f in frames[:2]:
    ex(f)
t0 = time.perf_counter()
for _ in range(4):
    for f in frames:
        ex(f)
t1 = time.perf_counter()
print(f"host path: {(t1 - t0) / 32 * 1e3:.3f} ms/frame")

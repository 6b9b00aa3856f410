import os, sys, time
sys.path.insert(0, '/root/repo/orb-slam-birdview_amd'); sys.path.insert(0, '/root/repo/oracle')
import numpy as np, orbgpu
from orbgpu.synth import synth_frame
img = synth_frame(1280, 720, 3)
b = orbgpu.BirdORB(2000)
k = b.detect(img)
pts = np.stack([k['x'], k['y']], 1).astype(np.float32)
for it in (1, 2, 3, 5, 10, 20, 40):
    b.cornerSubPix(img, pts, maxCount=it)
    t0 = time.perf_counter()
    for _ in range(20): p = b.cornerSubPix(img, pts, maxCount=it)
    t1 = time.perf_counter()
    prev = b.cornerSubPix(img, pts, maxCount=it - 1) if it > 1 else pts
    moved = (np.abs(p - prev).sum(1) > 0).sum()
    print(f"max_iter {it:3d}: {(t1 - t0) / 20 * 1e6:8.1f} us/call, points still moving at this iteration: {moved}")

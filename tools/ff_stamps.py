#!/usr/bin/env python3
"""Octree phase-1 fast-forward sub-steps (diagnostic, GPU; STAMPS=1 build via ORBGPU_LIB_PATH):
per level the mean cycles of gather, zero, A (path codes), B (count tables), C (bookkeeping),
D (list scan), E (key nodes) and the rest.  Usage: python3 tools/ff_stamps.py [B]"""
import os
import sys

os.environ["ORBGPU_FAST_STAMPS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
import numpy as np  # noqa: E402

import orbgpu  # noqa: E402
from orbgpu.synth import synth_batch  # noqa: E402

B, NL, NCELLS = int(sys.argv[1]) if len(sys.argv) > 1 else 1, 8, 2656
bx = orbgpu.BatchExtractor(2000, 1280, 720, B)
bx.upload(synth_batch(1280, 720, B))
for _ in range(3):
    bx.launch()
bx.sync()
cap = B * (NCELLS * 8 + NL * 32)
st = np.zeros(cap, np.uint64)
orbgpu._lib.lib().orb_debug_fast_stamps(bx.h, st.ctypes.data, cap)
o = st[B * NCELLS * 8:].reshape(B, NL, 32).astype(np.int64)
for lv in range(NL):
    s = o[:, lv]
    seq = [0, 1, 12, 13, 14, 15, 16, 2]
    d = [np.mean(s[:, b] - s[:, a]) for a, b in zip(seq, seq[1:])]
    # rounds after the fast-forward: stamps 3 + round at each round's end (round0 = R); the last one set
    ends = [max(int(np.max(np.nonzero(r[3:12])[0])) if np.any(r[3:12]) else -1, -1) for r in s]
    last = np.array([r[3 + e] if e >= 0 else r[2] for r, e in zip(s, ends)])
    print(f"level {lv}: C {s[:, 29].mean():6.0f} total {np.mean(s[:, 31] - s[:, 0]):7.0f}  gather {d[0]:6.0f} zero {d[1]:5.0f} "
          f"A {d[2]:5.0f} B {d[3]:5.0f} C {d[4]:5.0f} D {d[5]:5.0f} E+prep {d[6]:5.0f} rounds {np.mean(last - s[:, 2]):6.0f} "
          f"best {np.mean(s[:, 31] - last):6.0f}")

#!/usr/bin/env python3
"""Where a k_octree workgroup spends its time (diagnostic, GPU): runs one C3 batch with
ORBGPU_FAST_STAMPS=1 and prints, per pyramid level, the mean s_memtime cycles of the candidate
gather, the root setup, each division round and the final best-key pass, with the candidate
count and the round at which phase 2 (sorted division) starts.
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
    B, NL, NCELLS = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 8, 2656
    NF = int(sys.argv[2]) if len(sys.argv) > 2 else 2000   # features (C5: 4000)
    bx = orbgpu.BatchExtractor(NF, 1280, 720, B)
    bx.upload(synth_batch(1280, 720, B))
    for _ in range(3):
        bx.launch()
    bx.sync()
    L = orbgpu._lib.lib()
    cap = B * (NCELLS * 8 + NL * 32)
    st = np.zeros(cap, np.uint64)
    n = L.orb_debug_fast_stamps(bx.h, st.ctypes.data, cap)
    assert n >= cap, (n, cap)
    o = st[B * NCELLS * 8:].reshape(B, NL, 32).astype(np.int64)
    t0 = o[:, :, 0].min()
    for lv in range(NL):
        s = o[:, lv]
        tot = s[:, 31] - s[:, 0]
        nr = [int(np.count_nonzero(r[3:12])) for r in s]
        rounds = np.array([np.diff(np.concatenate([[r[2]], r[3:3 + k]])) for r, k in zip(s, nr)], dtype=object)
        mr = max(nr)
        per_round = [float(np.mean([x[i] for x in rounds if len(x) > i])) for i in range(mr)]
        last = np.array([r[2 + k] for r, k in zip(s, nr)])
        print(f"level {lv}: C {s[:, 29].mean():7.0f}  total {tot.mean():8.0f} cyc  start +{(s[:, 0] - t0).mean():7.0f}"
              f"  gather {(s[:, 1] - s[:, 0]).mean():6.0f}  roots {(s[:, 2] - s[:, 1]).mean():6.0f}"
              f"  rounds {np.mean(nr):4.1f} (phase2 at {s[:, 30].mean():4.1f})  best {(s[:, 31] - last).mean():6.0f}")
        print("         per round:", " ".join(f"{x:.0f}" for x in per_round))
        r0 = np.diff(np.concatenate([s[:, 2:3], s[:, 12:17]], axis=1), axis=1).mean(axis=0)
        print("         round 0 steps (zero, quad counts, scan, moves, knode):", " ".join(f"{x:.0f}" for x in r0))
        p2 = s[:, 20:29]
        ok = p2[:, 0] > 0
        if ok.any():
            d = np.diff(p2[ok], axis=1).mean(axis=0)
            print("         phase-2 steps (quad counts, dense keys, ranks, cut, assign, undivided, moves, knode):",
                  " ".join(f"{x:.0f}" for x in d))


if __name__ == "__main__":
    main()

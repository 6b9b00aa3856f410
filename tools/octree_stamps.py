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
    # slots: 0 start, 1 gathered, 2 fast-forward done, 3 + r end of round r (r < 9; rounds start at the fast-forward
    # depth R), 12..16 fast-forward sub-steps, 20..28 the first phase-2 round's sub-steps, 29 C, 30 phase-2 start, 31 done
    for lv in range(NL):
        s = o[:, lv]
        tot = s[:, 31] - s[:, 0]
        ends = [sorted(int(x) for x in r[3:12] if x > 0) for r in s]
        nr = np.mean([len(e) for e in ends])
        rounds = [np.diff([int(r[2])] + e) for r, e in zip(s, ends)]
        mr = max(len(x) for x in rounds)
        per_round = [float(np.mean([x[i] for x in rounds if len(x) > i])) for i in range(mr)]
        last = np.array([e[-1] if e else int(r[2]) for r, e in zip(s, ends)])
        ff = np.diff(np.concatenate([s[:, 1:2], s[:, 12:17], s[:, 2:3]], axis=1), axis=1).mean(axis=0)
        print(f"level {lv}: C {s[:, 29].mean():6.0f}  total {tot.mean():7.0f} cyc  gather {(s[:, 1] - s[:, 0]).mean():6.0f}"
              f"  fast-forward {(s[:, 2] - s[:, 1]).mean():6.0f}  rounds {nr:3.1f}: {' '.join(f'{x:.0f}' for x in per_round)}"
              f"  best+out {(s[:, 31] - last).mean():6.0f} (zero {(s[:, 17] - last).mean():.0f}, max {(s[:, 18] - s[:, 17]).mean():.0f},"
              f" out {(s[:, 31] - s[:, 18]).mean():.0f})")
        print("         fast-forward steps (zero, codes, depth sums, stop, list scan, key nodes + quads):",
              " ".join(f"{x:.0f}" for x in ff))
        p2 = s[:, 20:29]
        ok = p2[:, 0] > 0
        if ok.any():
            d = np.diff(p2[ok], axis=1).mean(axis=0)
            print("         phase-2 steps (quad counts, dense keys, ranks, cut, assign, undivided, moves, knode):",
                  " ".join(f"{x:.0f}" for x in d))


if __name__ == "__main__":
    main()

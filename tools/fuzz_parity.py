"""Randomised extraction parity (test infrastructure: the oracle is the checker): N configurations drawn from a
seeded generator -- frame size (odd sizes included), nfeatures, scale factor, levels, FAST thresholds, OpenCV variant
bits, frame content -- each extracted by liborbgpu (orbgpu.ORBextractor: the drop-in operator()) and by the oracle
restatement of ORBextractor.cc:1043-1132; keypoints (all 28 bytes) and descriptors must be equal byte for byte.
A configuration the library refuses as geometry (ORB_ERR_GEOMETRY: a level below the FAST border or beyond the
LDS-sized limits) must be refused by a documented bound, and is counted separately.
usage: python3 tools/fuzz_parity.py <n> [seed0]   (prints one line per failure and a summary line).
tests/test_gpu_fuzz.py runs a few of the same seeded cases through extract_case()."""
import sys

import numpy as np

sys.path.insert(0, "orb-slam-birdview_amd")
sys.path.insert(0, "oracle")
import oracle  # noqa: E402
import orbgpu  # noqa: E402
from orbgpu.synth import synth_frame  # noqa: E402


def config(s):
    """The seeded configuration of case s: (w, h, nfeatures, scale, nlevels, iniTh, minTh, variant, kind)."""
    rng = np.random.default_rng(1000 + s)
    w = int(rng.integers(160, 1921))
    h = int(rng.integers(120, 1081))
    nf = int(rng.choice([300, 500, 1000, 2000, 3000, 4000]))
    sf = float(rng.choice([1.1, 1.2, 1.2, 1.25, 1.3, 1.5]))
    nl = int(rng.integers(1, 13))
    ini, mn = [(20, 7), (20, 7), (12, 7), (30, 10), (15, 5)][int(rng.integers(0, 5))]
    variant = 0 if rng.random() < 0.7 else int(rng.integers(1, 16))
    kind = "noise" if rng.random() < 0.1 else "scene"
    return w, h, nf, sf, nl, ini, mn, variant, kind


def level0_target(nf, sf, nl):
    """Level 0's feature target (ORBextractor.cc:436-446): the largest per-level N of the pyramid."""
    f = 1.0 / sf
    return nf * (1 - f) / (1 - f ** nl) if nl > 1 else float(nf)


# orbgpu.h, ORB_ERR_GEOMETRY: a level whose octree node tables exceed one CU's LDS (N per level above ~2,550)
LDS_LEVEL_BOUND = 2500


def extract_case(s):
    """Case s through liborbgpu and the oracle.  Returns (status, cfg, nkeypoints): status "equal", "mismatch",
    "refused" (both refuse: the reference's degenerate geometry), "refused_bound" (the GPU refuses a level above
    the documented LDS bound, the oracle runs) or "refused_unexplained" (the GPU refuses anything else)."""
    cfg = config(s)
    w, h, nf, sf, nl, ini, mn, variant, kind = cfg
    img = synth_frame(w, h, s, kind)
    o = oracle.OracleExtractor(nf, sf, nl, ini, mn, flags=variant)
    on = o.run(img)
    try:
        g = orbgpu.ORBextractor(nf, sf, nl, ini, mn, variant=variant)
        gk, gd = g(img)
    except orbgpu.OrbError:
        if on < 0:
            return "refused", cfg, 0
        return ("refused_bound" if level0_target(nf, sf, nl) > LDS_LEVEL_BOUND else "refused_unexplained"), cfg, 0
    if on < 0:
        return "mismatch", cfg, 0   # the reference cannot run this geometry, the GPU claims it can
    ok_k, ok_d = o.output()
    if len(gk) == len(ok_k) and gk.tobytes() == ok_k.tobytes() and np.array_equal(gd, ok_d):
        return "equal", cfg, len(gk)
    return "mismatch", cfg, len(gk)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    ok = fail = refused = 0
    kps_total = 0
    for s in range(seed0, seed0 + n):
        st, cfg, nk = extract_case(s)
        if st == "equal":
            ok += 1
            kps_total += nk
        elif st.startswith("refused") and st != "refused_unexplained":
            refused += 1
            print("refused", cfg, st)
        else:
            fail += 1
            print("MISMATCH", cfg, st, nk)
    print(f"SUMMARY configurations={n} equal={ok} mismatched={fail} refused={refused} keypoints_compared={kps_total}")
    return 1 if fail else 0


if __name__ == "__main__":
    sys.exit(main())

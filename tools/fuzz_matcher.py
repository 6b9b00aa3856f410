"""Randomised matcher parity (test infrastructure: the oracle is the checker).  Per iteration: two frames extracted
by the GPU extractor (its parity is fuzz_parity.py's) at a random size / feature count, random FeatureVectors (node =
a random function of the descriptor, random node counts), random map-point and stereo masks, random ratio /
orientation check; the GPU calls -- SearchByBoW (KF,F) and (KF,KF), SearchForTriangulation, and their batched forms
over 1-6 keyframes -- against the oracle's restatements of ORBmatcher.cc:159-288, 522-655, 657-823.
usage: python3 tools/fuzz_matcher.py <n> [seed0]; tests/test_gpu_fuzz.py runs a few seeded cases through matcher_case()."""
import sys

import numpy as np

sys.path.insert(0, "orb-slam-birdview_amd")
sys.path.insert(0, "oracle")
import oracle  # noqa: E402
import orbgpu  # noqa: E402
from orbgpu.synth import synth_frame  # noqa: E402


def featvec(desc, rng):
    nodes = int(rng.integers(1, 300))
    salt = int(rng.integers(0, 32))
    fv = {}
    for i, d in enumerate(desc):
        fv.setdefault((int(d[salt % 32]) * 7 + int(d[(salt + 5) % 32])) % nodes * 3 + 1, []).append(i)
    return fv


def ofv(fv):
    ids = sorted(fv)
    return oracle.make_featvec(ids, [fv[i] for i in ids])


def matcher_case(s):
    """Case s: returns (status, info, bad) with status "equal", "mismatch" or "refused" (a frame geometry both the
    oracle and the GPU refuse) and bad the list of calls that differed from the oracle."""
    rng = np.random.default_rng(5000 + s)
    w, h = int(rng.integers(320, 1281)), int(rng.integers(240, 721))
    nf = int(rng.choice([500, 1000, 2000]))
    img = synth_frame(w, h, s)
    shift = (int(rng.integers(-4, 5)), int(rng.integers(-4, 5)))
    ex_ = oracle.OracleExtractor(nf)
    ext = orbgpu.ORBextractor(nf, 1.2, 8, 20, 7)  # frames are inputs here; extraction parity is fuzz_parity.py's
    if ex_.run(img) < 0:  # a geometry the reference cannot run (a level's cell grid degenerates): both refuse
        try:
            ext(img)
        except orbgpu.OrbError:
            return "refused", (w, h, nf), []
        return "mismatch", (w, h, nf), [("oracle refuses, GPU extracts",)]
    ka, da = ext(img)
    kb, db = ext(np.ascontiguousarray(np.roll(img, shift, axis=(0, 1))))
    ratio = float(rng.choice([0.6, 0.7, 0.75, 0.9]))
    ori = bool(rng.random() < 0.6)
    m = orbgpu.ORBmatcher(ratio, ori)
    bad = []
    # SearchByBoW (KF, F) and its batch over several keyframes
    kfs = []
    for _ in range(int(rng.integers(1, 7))):
        d, k = (da, ka) if rng.random() < 0.5 else (db, kb)
        kfs.append(dict(desc=d, angle=k["angle"], mp=(rng.random(len(d)) < rng.random()).astype(np.uint8),
                        featvec=featvec(d, rng)))
    fvf = featvec(db, rng)
    off, keep = ofv(fvf)
    got = m.SearchByBoW_KF_F_batch(kfs, db, kb["angle"], fvf)
    for i, (kf, (gn, gm)) in enumerate(zip(kfs, got)):
        oa, keep_a = ofv(kf["featvec"])
        on, om = oracle.search_by_bow_kf_f(ratio, ori, kf["desc"], kf["angle"], kf["mp"], oa, db, kb["angle"], off)
        if gn != on or not np.array_equal(gm, om):
            bad.append(("bow_kf_f", i))
        if i == 0:
            sn, sm = m.SearchByBoW_KF_F(kf["desc"], kf["angle"], kf["mp"], kf["featvec"], db, kb["angle"], fvf)
            if sn != on or not np.array_equal(sm, om):
                bad.append(("bow_kf_f_single",))
    # SearchByBoW (KF, KF) batch, and the single call on the first keyframe
    mp1 = (rng.random(len(da)) < rng.random()).astype(np.uint8)
    fv1 = featvec(da, rng)
    o1, keep1 = ofv(fv1)
    got = m.SearchByBoW_KF_KF_batch(da, ka["angle"], mp1, fv1, kfs)
    for i, (kf, (gn, gm)) in enumerate(zip(kfs, got)):
        ob, keep_b = ofv(kf["featvec"])
        on, om = oracle.search_by_bow_kf_kf(ratio, ori, da, ka["angle"], mp1, o1, kf["desc"], kf["angle"], kf["mp"], ob)
        if gn != on or not np.array_equal(gm, om):
            bad.append(("bow_kf_kf", i))
        if i == 0:
            sn, sm = m.SearchByBoW_KF_KF(da, ka["angle"], mp1, fv1, kf["desc"], kf["angle"], kf["mp"], kf["featvec"])
            if sn != on or not np.array_equal(sm, om):
                bad.append(("bow_kf_kf_single",))
    # SearchForTriangulation batch (random F near a horizontal epipolar geometry, random epipoles), and the single
    # call on the first neighbour
    t = ex_.tables()
    ur1 = np.where(rng.random(len(da)) < 0.3, 10.0, -1.0).astype(np.float32)
    others = []
    for _ in range(int(rng.integers(1, 7))):
        d, k = (db, kb) if rng.random() < 0.7 else (da, ka)
        F = (np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)
             + rng.normal(0, 10 ** rng.uniform(-6, -3), (3, 3)).astype(np.float32))
        ex, ey = float(rng.uniform(-2000, 2000)), float(rng.uniform(-2000, 2000))
        others.append(dict(desc2=d, kps2=k, has_mp2=(rng.random(len(d)) < rng.random()).astype(np.uint8),
                           uright2=np.where(rng.random(len(d)) < 0.3, 10.0, -1.0).astype(np.float32),
                           featvec2=featvec(d, rng), F12=F, ex=ex, ey=ey, scale_factors2=t["scale"],
                           level_sigma2_2=t["sigma2"]))
    stereo = bool(rng.random() < 0.2)
    got = m.SearchForTriangulationBatch(da, ka, mp1, ur1, fv1, others, stereo)
    for i, (o, gp) in enumerate(zip(others, got)):
        ob, keep_b = ofv(o["featvec2"])
        op = oracle.search_for_triangulation(ori, stereo, da, ka, mp1, ur1, o1, o["desc2"], o["kps2"], o["has_mp2"],
                                             o["uright2"], ob, o["F12"], o["ex"], o["ey"], t["scale"], t["sigma2"])
        if not np.array_equal(gp, op):
            bad.append(("triangulation", i))
        if i == 0:
            sp = m.SearchForTriangulation(da, ka, mp1, ur1, fv1, o["desc2"], o["kps2"], o["has_mp2"], o["uright2"],
                                          o["featvec2"], o["F12"], o["ex"], o["ey"], t["scale"], t["sigma2"], stereo)
            if not np.array_equal(sp, op):
                bad.append(("triangulation_single",))
    return ("mismatch" if bad else "equal"), (w, h, nf, ratio, ori), bad


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    ok = fail = refused = 0
    for s in range(seed0, seed0 + n):
        st, info, bad = matcher_case(s)
        if st == "equal":
            ok += 1
        elif st == "refused":
            refused += 1
        else:
            fail += 1
            print("MISMATCH seed", s, info, bad)
        if (s - seed0) % 10 == 9:
            print(f"progress {s - seed0 + 1}/{n} equal={ok} mismatched={fail} refused={refused}", flush=True)
    print(f"SUMMARY iterations={n} equal={ok} mismatched={fail} refused={refused}", flush=True)
    return 1 if fail else 0


if __name__ == "__main__":
    sys.exit(main())

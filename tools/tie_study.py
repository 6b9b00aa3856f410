#!/usr/bin/env python3
"""DistributeOctTree tie-order study (VERDICT r01 'Next' 1a).

ORBextractor.cc:684 sorts std::pair<int, ExtractorNode*>: nodes of equal size are ordered by their heap
ADDRESS, which decides which of them are split before the list reaches N (:730).  The oracle's
ORACLE_TIE_LITERAL mode runs that algorithm with the reference's own data structures, so the addresses
are the ones glibc malloc hands out in the running process.  This tool runs it over seeded C3 frames
in three heap contexts (tools/tie_driver.cpp: a fresh process per frame, one warm process, a fresh
thread per frame) and compares the keypoints with the oracle's pinned policies:

  seq      creation sequence (later-created = larger pointer; the kernel's policy)
  rev      reverse creation sequence (ORACLE_TIE_REVERSE_SEQ)

Prints one JSON object (per-frame keypoint deltas |A xor B| over (octave, x, y), agreement rates).
Usage: python3 tools/tie_study.py [--frames 64] [--w 1280 --h 720 --nf 2000] [--kind scene]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def build_driver(tmp):
    import oracle
    oracle.lib()
    exe = os.path.join(tmp, "tie_driver")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(ROOT, "tools", "tie_driver.cpp"),
                           "-L" + os.path.join(ROOT, "oracle"), "-lorb_oracle", "-Wl,-rpath," + os.path.join(ROOT, "oracle"),
                           "-lpthread"])
    return exe


def read_out(path, n):
    import oracle
    res = []
    with open(path, "rb") as f:
        for _ in range(n):
            m = int(np.frombuffer(f.read(4), np.int32)[0])
            res.append(np.frombuffer(f.read(28 * m), oracle.KP_DTYPE) if m else np.zeros(0, oracle.KP_DTYPE))
    return res


def kset(k):
    return set(zip(k["octave"].tolist(), k["x"].tolist(), k["y"].tolist()))


def delta(a, b):
    return len(kset(a) ^ kset(b))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--w", type=int, default=1280)
    ap.add_argument("--h", type=int, default=720)
    ap.add_argument("--nf", type=int, default=2000)
    ap.add_argument("--kind", default="scene")
    ap.add_argument("--first", type=int, default=0)
    args = ap.parse_args()
    import oracle
    from orbgpu.synth import synth_frame
    frames = [synth_frame(args.w, args.h, args.first + i, args.kind) for i in range(args.frames)]
    with tempfile.TemporaryDirectory() as tmp:
        exe = build_driver(tmp)
        raw = os.path.join(tmp, "frames.raw")
        np.ascontiguousarray(np.stack(frames)).tofile(raw)
        common = [raw, str(args.w), str(args.h), str(args.nf)]
        lit = {}
        for mode in ("warm", "thread"):
            out = os.path.join(tmp, mode + ".bin")
            subprocess.check_call([exe] + common + [mode, "0", str(args.frames), out])
            lit[mode] = read_out(out, args.frames)
        fresh = []
        for i in range(args.frames):
            out = os.path.join(tmp, f"fresh{i}.bin")
            subprocess.check_call([exe] + common + ["fresh", str(i), "1", out])
            fresh += read_out(out, 1)
        lit["fresh"] = fresh
    seq = [oracle.OracleExtractor(args.nf, flags=0)(f)[0] for f in frames]
    rev = [oracle.OracleExtractor(args.nf, flags=oracle.TIE_REVERSE_SEQ)(f)[0] for f in frames]
    rep = {"frames": args.frames, "config": f"{args.w}x{args.h} {args.nf} features, {args.kind}, seeds {args.first}..",
           "seq_vs_rev": {"frames_equal": int(sum(s.tobytes() == r.tobytes() for s, r in zip(seq, rev))),
                          "delta_mean": float(np.mean([delta(s, r) for s, r in zip(seq, rev)])),
                          "delta_max": int(max(delta(s, r) for s, r in zip(seq, rev)))}}
    for mode, L in lit.items():
        d_seq = [delta(a, s) for a, s in zip(L, seq)]
        d_rev = [delta(a, r) for a, r in zip(L, rev)]
        rep[mode] = {"frames_equal_seq": int(sum(a.tobytes() == s.tobytes() for a, s in zip(L, seq))),
                     "frames_equal_rev": int(sum(a.tobytes() == r.tobytes() for a, r in zip(L, rev))),
                     "delta_seq_mean": float(np.mean(d_seq)), "delta_seq_max": int(max(d_seq)),
                     "delta_rev_mean": float(np.mean(d_rev)), "delta_rev_max": int(max(d_rev)),
                     "count_diff_seq_max": int(max(abs(len(a) - len(s)) for a, s in zip(L, seq)))}
    modes = list(lit)
    rep["contexts_agree"] = {f"{a}_vs_{b}": int(sum(x.tobytes() == y.tobytes() for x, y in zip(lit[a], lit[b])))
                             for i, a in enumerate(modes) for b in modes[i + 1:]}
    rep["contexts_delta"] = {f"{a}_vs_{b}": {"mean": float(np.mean([delta(x, y) for x, y in zip(lit[a], lit[b])])),
                                             "max": int(max(delta(x, y) for x, y in zip(lit[a], lit[b])))}
                             for i, a in enumerate(modes) for b in modes[i + 1:]}
    print(json.dumps(rep))


if __name__ == "__main__":
    main()

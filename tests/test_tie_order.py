"""DistributeOctTree's pointer tie (ORBextractor.cc:684) — what the pin can and cannot claim.

The oracle's ORACLE_TIE_LITERAL mode runs the reference's std::list / pair<int, ExtractorNode*> algorithm,
so ties fall to glibc heap addresses.  These tests check the facts DESIGN.md quotes, on a small sample
(tools/tie_study.py measures 64 frames per config into profiles/r02/tie_study_*.json):
  * the literal run is reproducible for a given heap history (same frame, fresh process, twice);
  * it depends on the heap history (the same frames in one warm process differ from fresh processes);
  * the pinned creation-sequence policy differs from the literal runs by about as much as the literal
    runs differ from each other, and every policy keeps the keypoint count within a few of the others.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def study(tmp_path_factory, oracle_mod):
    import tie_study
    from orbgpu.synth import synth_frame
    d = str(tmp_path_factory.mktemp("tie"))
    exe = tie_study.build_driver(d)
    frames = [synth_frame(1280, 720, 40 + i) for i in range(4)]
    raw = os.path.join(d, "frames.raw")
    np.ascontiguousarray(np.stack(frames)).tofile(raw)
    common = [exe, raw, "1280", "720", "2000"]

    def run(mode, first, count, tag):
        out = os.path.join(d, tag + ".bin")
        subprocess.check_call(common + [mode, str(first), str(count), out], timeout=300)
        return tie_study.read_out(out, count)
    fresh_a = [run("fresh", i, 1, f"a{i}")[0] for i in range(4)]
    fresh_b = [run("fresh", i, 1, f"b{i}")[0] for i in range(4)]
    warm = run("warm", 0, 4, "warm")
    seq = [oracle_mod.OracleExtractor(2000)(f)[0] for f in frames]
    return dict(fresh_a=fresh_a, fresh_b=fresh_b, warm=warm, seq=seq, delta=tie_study.delta)


def test_literal_run_reproducible_for_a_fixed_heap_history(study):
    for a, b in zip(study["fresh_a"], study["fresh_b"]):
        assert a.tobytes() == b.tobytes()


def test_literal_run_depends_on_heap_history(study):
    # frame 0 of the warm process sees the same heap as a fresh process; later frames do not
    assert study["warm"][0].tobytes() == study["fresh_a"][0].tobytes()
    assert any(w.tobytes() != f.tobytes() for w, f in zip(study["warm"][1:], study["fresh_a"][1:]))


def test_pinned_policy_within_the_literal_spread(study):
    d = study["delta"]
    between = [d(w, f) for w, f in zip(study["warm"][1:], study["fresh_a"][1:])]
    to_seq = [d(f, s) for f, s in zip(study["fresh_a"], study["seq"])]
    assert max(to_seq) <= 3 * max(max(between), 20)   # ~2 % of 2000 keypoints either way
    for f, s in zip(study["fresh_a"], study["seq"]):
        assert abs(len(f) - len(s)) <= 8

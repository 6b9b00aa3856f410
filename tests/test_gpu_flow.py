"""GPU parity of the small-batch dataflow launch (k_extract_flow).

Batches of one or two frames (C5 at one frame per GPU, BASELINE config 5) run the whole extraction as ONE
persistent launch: 1024-thread workgroups take (stage, level, frame) tasks from a device ticket in a host-built
topological order and hand the pyramid levels, FAST candidate records and octree outputs to each other inside the
launch with write-through (sc1) stores and loads and per-(frame, level) counters.  A wrong hand-off reads stale
bytes, so every test here compares keypoints, descriptors and pyramid levels byte for byte with the oracle
(ORBextractor.cc:1043-1105 restated), over many launches on the same buffers, under uneven load (several
contexts in flight) and with the launch shrunk to one workgroup (every task in ticket order) or grown to one per CU.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _flow_on(monkeypatch):
    monkeypatch.setenv("ORBGPU_FLOW", "1")   # (read at orb_create)
    monkeypatch.delenv("ORBGPU_FLOW_CHAIN", raising=False)


def _check(e, o, frames, B, levels=True):
    for f in range(B):
        ok, od = o(frames[f])
        gk, gd = e.results(f)
        assert len(gk) == len(ok) and gk.tobytes() == ok.tobytes(), (f, len(gk), len(ok))
        assert np.array_equal(gd, od), f
        if levels:
            for lv in range(1, 8):
                assert np.array_equal(e.debug_level_image(lv, f), o.level(lv)), (f, lv)


@pytest.mark.parametrize("w,h,nf,B", [(1280, 720, 4000, 1), (1280, 720, 4000, 2), (1280, 720, 2000, 1),
                                      (1280, 720, 2000, 2), (640, 480, 1000, 1), (640, 480, 1000, 2)])
def test_flow_bit_exact(orbgpu_mod, oracle_mod, w, h, nf, B):
    """C5 / C3 / C2 at one and two frames per launch: the graph's capture, then replays on new frames in the same
    buffers (a stale hand-off would show the previous frame's bytes)."""
    from orbgpu.synth import bench_frames
    e = orbgpu_mod.BatchExtractor(nf, w, h, B)
    o = oracle_mod.OracleExtractor(nf)
    for rnd in range(3):
        frames = bench_frames(w, h, B, first=5 + 7 * rnd)
        e.upload(frames)
        for _ in range(2):
            e.launch()
            e.sync()
        _check(e, o, frames, B)
    e.close()


@pytest.mark.parametrize("w,h,nf,B", [(1280, 720, 4000, 1), (1280, 720, 2000, 2), (640, 480, 1000, 1)])
def test_flow_chain_pyramid_tasks(orbgpu_mod, oracle_mod, monkeypatch, w, h, nf, B):
    """ORBGPU_FLOW_CHAIN=1: the pyramid as chain-job tasks (every tile's region chain recomputed from the segment base,
    k_pyramid_chain's arithmetic) instead of per-level resize tasks; the same bytes."""
    from orbgpu.synth import bench_frames
    monkeypatch.setenv("ORBGPU_FLOW_CHAIN", "1")
    e = orbgpu_mod.BatchExtractor(nf, w, h, B)
    o = oracle_mod.OracleExtractor(nf)
    for rnd in range(2):
        frames = bench_frames(w, h, B, first=11 + 5 * rnd)
        e.upload(frames)
        e.launch()
        e.sync()
        _check(e, o, frames, B)
    e.close()


def test_flow_matches_per_kernel_launches(orbgpu_mod, monkeypatch):
    """The dataflow launch and the per-kernel launches (ORBGPU_FLOW=0) give identical outputs for the same frames."""
    from orbgpu.synth import bench_frames
    frames = bench_frames(1280, 720, 2, first=40)
    out = []
    for flow in ("1", "0"):
        monkeypatch.setenv("ORBGPU_FLOW", flow)
        e = orbgpu_mod.BatchExtractor(4000, 1280, 720, 2)
        e.upload(frames)
        e.launch()
        e.sync()
        out.append([e.results(f) for f in range(2)])
        e.close()
    for (ka, da), (kb, db) in zip(*out):
        assert ka.tobytes() == kb.tobytes() and np.array_equal(da, db)


@pytest.mark.parametrize("blocks", ["1", "3", "256"])
def test_flow_workgroup_counts(orbgpu_mod, oracle_mod, monkeypatch, blocks):
    """One workgroup (every task in ticket order, no waits), three (most tasks wait on another workgroup), one per
    CU: the same outputs."""
    from orbgpu.synth import bench_frames
    monkeypatch.setenv("ORBGPU_FLOW_BLOCKS", blocks)
    frames = bench_frames(1280, 720, 1, first=3)
    e = orbgpu_mod.BatchExtractor(4000, 1280, 720, 1)
    e.upload(frames)
    for _ in range(2):
        e.launch()
        e.sync()
        _check(e, oracle_mod.OracleExtractor(4000), frames, 1, levels=False)
    e.close()


def test_flow_uneven_load(orbgpu_mod, oracle_mod):
    """Four contexts in flight (the bench's C5 form, one frame each, different frames) replayed 40 times without a
    host synchronisation in between, then each checked: hand-offs under contention and uneven arrival."""
    from orbgpu.synth import bench_frames
    frames = bench_frames(1280, 720, 4, first=21)
    es = []
    for i in range(4):
        e = orbgpu_mod.BatchExtractor(4000, 1280, 720, 1)
        e.upload(frames[i:i + 1])
        es.append(e)
    for _ in range(40):
        for e in es:
            e.launch()
    for e in es:
        e.sync()
    o = oracle_mod.OracleExtractor(4000)
    for i, e in enumerate(es):
        _check(e, o, frames[i:i + 1], 1, levels=False)
        e.close()


@pytest.mark.parametrize("variant", [1, 2, 4, 8, 15])
def test_flow_variants(orbgpu_mod, oracle_mod, variant):
    """Every OpenCV arithmetic variant bit (include/orbgpu.h ORB_VARIANT_*) through the dataflow launch, against the
    oracle under the same flag, at one and two frames."""
    from orbgpu.synth import bench_frames
    for B in (1, 2):
        frames = bench_frames(1280, 720, B, first=60 + B)
        e = orbgpu_mod.BatchExtractor(2000, 1280, 720, B, variant=variant)
        e.upload(frames)
        e.launch()
        e.sync()
        _check(e, oracle_mod.OracleExtractor(2000, flags=variant), frames, B, levels=(variant & 2) != 0)
        e.close()


def test_flow_edge_frames(orbgpu_mod, oracle_mod):
    """A flat frame (no corner anywhere: every cell runs the minThFAST pass, every level's octree gets no key), a
    noise frame (the densest candidate lists) and a scene frame in one two-frame launch, then swapped."""
    from orbgpu.synth import synth_frame
    flat = np.full((720, 1280), 128, np.uint8)
    noise = synth_frame(1280, 720, 3, "noise")
    scene = synth_frame(1280, 720, 4, "scene")
    o = oracle_mod.OracleExtractor(4000)
    e = orbgpu_mod.BatchExtractor(4000, 1280, 720, 2)
    for pair in ((flat, noise), (noise, scene), (scene, flat)):
        fr = np.stack(pair)
        e.upload(fr)
        e.launch()
        e.sync()
        _check(e, o, fr, 2, levels=False)
    assert e.counts()[1] == 0
    e.close()

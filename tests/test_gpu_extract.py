"""GPU parity: liborbgpu's HIP extractor vs the oracle restatement of ORBextractor.cc, bit-exact
(keypoint structs byte-for-byte, descriptors byte-for-byte), stage by stage where it fails."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [  # (w, h, nfeatures, frame idx, kind) — BASELINE configs C2/C3/C5 at full size + edges
    (320, 240, 500, 0, "scene"),
    (640, 480, 1000, 0, "scene"),      # C2
    (640, 480, 1000, 11, "scene"),
    (1280, 720, 2000, 0, "scene"),     # C3
    (1280, 720, 2000, 7, "scene"),
    (1280, 720, 4000, 4, "scene"),     # C5 per-frame workload
    (641, 479, 1000, 2, "scene"),      # odd sizes: blur tail columns, resize edges
    (950, 400, 2000, 5, "scene"),      # mono_fisheye driver size (mono_fisheye.cc:111-116)
    (640, 480, 1000, 0, "flat"),       # zero keypoints, released descriptors
    (640, 480, 1000, 3, "noise"),      # maximum candidates: octree phase-2 stress
    (1280, 720, 2000, 9, "noise"),
    (640, 480, 100, 1, "scene"),       # tiny N per level
    (640, 480, 8000, 1, "scene"),      # more features than candidates on some levels
]


def _stage_report(o, g):
    msgs = []
    pyr = g.mvImagePyramid
    for l in range(8):
        if not np.array_equal(o.level(l), pyr[l]):
            msgs.append(f"pyramid level {l}")
            break
        if not np.array_equal(o.candidates(l), g.debug_candidates(l)):
            msgs.append(f"FAST candidates level {l}")
            break
        ok = o.level_keypoints(l)
        okx = np.stack([ok["x"], ok["y"], ok["response"]], 1).astype(np.int32)
        if not np.array_equal(okx, g.debug_level_keypoints(l)):
            msgs.append(f"octree level {l}")
            break
    return msgs


@pytest.mark.parametrize("w,h,nf,idx,kind", CASES)
def test_extract_bit_exact(orbgpu_mod, oracle_mod, w, h, nf, idx, kind):
    from orbgpu.synth import synth_frame
    img = synth_frame(w, h, idx, kind)
    o = oracle_mod.OracleExtractor(nf)
    ok_k, ok_d = o(img)
    g = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7)
    gk, gd = g(img)
    if len(gk) != len(ok_k) or gk.tobytes() != ok_k.tobytes() or not np.array_equal(gd, ok_d):
        pytest.fail(f"mismatch ({len(gk)} vs {len(ok_k)} keypoints); first failing stage: {_stage_report(o, g)}")


def test_scale_tables_match_oracle(orbgpu_mod, oracle_mod):
    for nf in (1000, 2000, 4000):
        g = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7)
        t = oracle_mod.OracleExtractor(nf).tables()
        assert np.array_equal(g.GetScaleFactors(), t["scale"])
        assert np.array_equal(g.GetInverseScaleFactors(), t["inv_scale"])
        assert np.array_equal(g.GetScaleSigmaSquares(), t["sigma2"])
        assert np.array_equal(g.GetInverseScaleSigmaSquares(), t["inv_sigma2"])
        assert np.array_equal(g.mnFeaturesPerLevel, t["n_per_level"])
        assert np.array_equal(g.umax, t["umax"])
        assert g.GetLevels() == 8 and abs(g.GetScaleFactor() - 1.2) < 1e-6


def test_other_parameters(orbgpu_mod, oracle_mod):
    # fisheye.yaml (2000 / 1.2 / 8 / 15 / 5) and KITTI04-12 stereo (iniTh 12)
    from orbgpu.synth import synth_frame
    img = synth_frame(640, 480, 21)
    # large scale factors: longer 4-pixel source spans in the tiled resize (1.6), the untiled resize (2.3)
    for params in [(2000, 1.2, 8, 15, 5), (1000, 1.2, 8, 12, 7), (1500, 1.3, 6, 20, 7), (1000, 1.6, 5, 20, 7),
                   (800, 2.3, 3, 20, 7)]:
        o = oracle_mod.OracleExtractor(params[0], params[1], params[2], params[3], params[4])
        ok, od = o(img)
        gk, gd = orbgpu_mod.ORBextractor(*params)(img)
        assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), params


@pytest.mark.parametrize("w,h,params", [
    (640, 480, (1000, 1.2, 1, 20, 7)),    # one level: no pyramid launches, every feature on level 0
    (640, 480, (1000, 1.2, 12, 20, 7)),   # 12 levels: the top one is 86x64, one FAST cell
    (1280, 720, (3000, 1.2, 12, 20, 7)),
    (1280, 720, (2000, 1.1, 16, 20, 7)),  # ORBGPU_MAX_LEVELS levels
])
def test_level_counts(orbgpu_mod, oracle_mod, w, h, params):
    # nlevels away from the default 8 (ORBextractor.cc:410-470 tables, :1107-1132 pyramid chain)
    from orbgpu.synth import synth_frame
    img = synth_frame(w, h, 13)
    ok, od = oracle_mod.OracleExtractor(*params)(img)
    gk, gd = orbgpu_mod.ORBextractor(*params)(img)
    assert len(gk) > 0
    assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), params


def test_host_path_frame_sequence(orbgpu_mod, oracle_mod):
    """One extractor (the host path: few-launch pyramid, direct launches, outputs written into pinned
    memory) over a run of frames with image-size changes in between (the geometry, coefficient tables and
    chain plan are rebuilt, the buffers regrown): every frame equal to the oracle (Frame.cc:414-420 calls
    one ORBextractor per camera for the whole sequence)."""
    from orbgpu.synth import synth_frame
    g = orbgpu_mod.ORBextractor(2000, 1.2, 8, 20, 7)
    o = oracle_mod.OracleExtractor(2000)
    seq = [(1280, 720)] * 6 + [(640, 480)] * 3 + [(1280, 720)] * 3 + [(641, 479)] * 2
    for i, (w, h) in enumerate(seq):
        img = synth_frame(w, h, 30 + i)
        ok, od = o(img)
        gk, gd = g(img)
        assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), (i, w, h)


def test_threshold_edges(orbgpu_mod, oracle_mod):
    # iniThFAST / minThFAST of 0 and 1 on a low-contrast frame, where arc strengths M of 1 and 2 decide
    # corners and the NMS (k_fast_wave keeps a corner iff M > max(neighbour M, 1): score M - 1 > 0 at
    # threshold 0, ORBextractor.cc:812-816 / cv::FAST nonmax)
    from orbgpu.synth import synth_frame
    img = (synth_frame(640, 480, 5) // 24 + 100).astype(np.uint8)
    for params in [(1000, 1.2, 8, 1, 0), (1000, 1.2, 8, 0, 0), (1000, 1.2, 8, 2, 1)]:
        ok, od = oracle_mod.OracleExtractor(*params)(img)
        gk, gd = orbgpu_mod.ORBextractor(*params)(img)
        assert len(gk) > 100, params
        assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), params


def test_empty_image_leaves_outputs_untouched(orbgpu_mod):
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    sentinel_k, sentinel_d = object(), object()
    k, d = g(np.zeros((0, 0), np.uint8), None, sentinel_k, sentinel_d)
    assert k is sentinel_k and d is sentinel_d
    from orbgpu import _lib
    n = ctypes.c_int(12345)
    assert _lib.lib().orb_extract(g.h, None, 0, 0, 0, None, 0, ctypes.byref(n), None) == 0
    assert n.value == 12345


def test_flat_image_zero_keypoints(orbgpu_mod):
    k, d = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)(np.full((480, 640), 77, np.uint8))
    assert len(k) == 0 and d.shape == (0, 32)


def test_too_small_image_is_an_error(orbgpu_mod):
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    with pytest.raises(orbgpu_mod.OrbError):
        g(np.full((120, 160), 50, np.uint8))


def test_strided_input(orbgpu_mod, oracle_mod):
    from orbgpu import _lib
    from orbgpu.synth import synth_frame
    img = synth_frame(640, 480, 6)
    big = np.zeros((480, 777), np.uint8)
    big[:, 5:645] = img
    view = big[:, 5:645]
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    kps = np.zeros(4000, orbgpu_mod.KP_DTYPE)
    desc = np.zeros((4000, 32), np.uint8)
    n = ctypes.c_int()
    st = _lib.lib().orb_extract(g.h, ctypes.c_void_p(view.ctypes.data), 640, 480, 777,
                                ctypes.c_void_p(kps.ctypes.data), 4000, ctypes.byref(n),
                                ctypes.c_void_p(desc.ctypes.data))
    assert st == 0
    ok, od = oracle_mod.OracleExtractor(1000)(img)
    assert kps[:n.value].tobytes() == ok.tobytes() and np.array_equal(desc[:n.value], od)


def test_capacity_error_reports_count(orbgpu_mod):
    from orbgpu import _lib
    from orbgpu.synth import synth_frame
    img = synth_frame(640, 480, 0)
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    kps = np.zeros(10, orbgpu_mod.KP_DTYPE)
    desc = np.zeros((10, 32), np.uint8)
    n = ctypes.c_int()
    st = _lib.lib().orb_extract(g.h, ctypes.c_void_p(img.ctypes.data), 640, 480, 640,
                                ctypes.c_void_p(kps.ctypes.data), 10, ctypes.byref(n),
                                ctypes.c_void_p(desc.ctypes.data))
    assert st == -3 and n.value > 10


def test_size_changes_reuse_context(orbgpu_mod, oracle_mod):
    from orbgpu.synth import synth_frame
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    o = oracle_mod.OracleExtractor(1000)
    for (w, h, i) in [(640, 480, 1), (1280, 720, 2), (320, 240, 3), (640, 480, 4)]:
        img = synth_frame(w, h, i)
        ok, od = o(img)
        gk, gd = g(img)
        assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od)


def test_batch_device_path_matches_single(orbgpu_mod, oracle_mod):
    from orbgpu.synth import synth_batch
    frames = synth_batch(1280, 720, 5, first=30)
    b = orbgpu_mod.BatchExtractor(2000, 1280, 720, 5)
    b.upload(frames)
    b.launch()
    b.sync()
    o = oracle_mod.OracleExtractor(2000)
    for f in range(5):
        gk, gd = b.results(f)
        ok, od = o(frames[f])
        assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), f
    # relaunch is idempotent
    c0 = b.counts().copy()
    b.launch()
    b.sync()
    assert np.array_equal(b.counts(), c0)
    b.close()


def test_mv_image_pyramid(orbgpu_mod, oracle_mod):
    from orbgpu.synth import synth_frame
    img = synth_frame(640, 480, 8)
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    g(img)
    o = oracle_mod.OracleExtractor(1000)
    o(img)
    pyr = g.mvImagePyramid
    assert len(pyr) == 8
    for l in range(8):
        assert np.array_equal(pyr[l], o.level(l))


def test_two_contexts_interleaved(orbgpu_mod, oracle_mod):
    # stereo: left/right extractors are independent instances (Frame.cc:124-127)
    from orbgpu.synth import synth_frame, synth_stereo_right
    left = synth_frame(1280, 720, 12)
    right = synth_stereo_right(left, 12)
    gl = orbgpu_mod.ORBextractor(2000, 1.2, 8, 20, 7)
    gr = orbgpu_mod.ORBextractor(2000, 1.2, 8, 20, 7)
    kl, dl = gl(left)
    kr, dr = gr(right)
    o = oracle_mod.OracleExtractor(2000)
    ol, odl = o(left)
    orr, odr = o(right)
    assert kl.tobytes() == ol.tobytes() and np.array_equal(dl, odl)
    assert kr.tobytes() == orr.tobytes() and np.array_equal(dr, odr)
    # each context keeps its own mvImagePyramid (instance state, ORBextractor.h:85)
    ol3 = oracle_mod.OracleExtractor(2000)
    ol3(left)
    assert np.array_equal(gl.mvImagePyramid[3], ol3.level(3))
    assert np.array_equal(gr.mvImagePyramid[3], o.level(3))


def test_device_sincosf_matches_glibc_restatement(orbgpu_mod, oracle_mod):
    """csrc/glibc_trig.h on the GPU == oracle/glibc_sincosf.inc (== libm, tests/test_trig_pin.py) on a
    strided sweep of every float in [0, 2*pi] plus every float degree value the BRIEF path can form."""
    from orbgpu import _lib
    u = np.arange(0, 0x40C90FDB, 97, dtype=np.uint32)
    x = np.concatenate([u.view(np.float32),
                        (np.arange(0, 360 * 4096, dtype=np.float32) / np.float32(4096)) * np.float32(np.pi / 180)])
    x = np.ascontiguousarray(x, np.float32)
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    s, c = np.zeros_like(x), np.zeros_like(x)
    assert _lib.lib().orb_debug_sincosf(g.h, x.ctypes.data, len(x), s.ctypes.data, c.ctypes.data) == 0
    os_, oc = oracle_mod.sincosf(x)
    assert np.array_equal(s.view(np.uint32), os_.view(np.uint32))
    assert np.array_equal(c.view(np.uint32), oc.view(np.uint32))


@pytest.mark.parametrize("env", [{"ORBGPU_GRAPH": "0"}, {"ORBGPU_FAST_STAMPS": "1"}])
def test_diagnostic_switches_leave_results_unchanged(orbgpu_mod, oracle_mod, monkeypatch, env):
    """The two environment switches liborbgpu still reads are diagnostics: direct launches instead of
    graph replay, and kernel phase timestamps.  Both must give the default path's bytes (three frames,
    launched twice)."""
    from orbgpu.synth import synth_batch
    frames = synth_batch(1280, 720, 3, first=50)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    b = orbgpu_mod.BatchExtractor(2000, 1280, 720, 3)
    b.upload(frames)
    b.launch()
    b.launch()
    b.sync()
    o = oracle_mod.OracleExtractor(2000)
    for f in range(3):
        gk, gd = b.results(f)
        ok, od = o(frames[f])
        assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), (env, f)
    b.close()


@pytest.mark.parametrize("env", [{"ORBGPU_FORK": "1"}, {"ORBGPU_UPLOAD": "1"}, {"ORBGPU_FORK": "1", "ORBGPU_UPLOAD": "1"}])
def test_host_path_switches_bit_exact(orbgpu_mod, oracle_mod, monkeypatch, env):
    """The host path's (orb_extract, one frame in flight) A/B switches: level 0 forked onto a second stream, and the
    streamed image upload (host band copy + flags polled by k_upload_stream).  Both off by default;
    each must give the oracle's bytes, over consecutive frames of two sizes on one extractor (flag sequence numbers
    and the pinned staging reused across calls)."""
    from orbgpu.synth import synth_frame
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = orbgpu_mod.ORBextractor(2000, 1.2, 8, 20, 7)
    o = oracle_mod.OracleExtractor(2000)
    for i, (w, h) in enumerate([(1280, 720), (1280, 720), (641, 479), (1280, 720)]):
        img = synth_frame(w, h, 70 + i)
        gk, gd = g(img)
        ok, od = o(img)
        assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), (env, w, h)


def test_bench_configuration_bit_exact(orbgpu_mod, oracle_mod):
    """The exact configuration bench.py times: C3, B = 256 frames per batch, two extractor contexts
    (own stream and buffers) launched alternately with several batches in flight, through the hipGraph
    path.  Frames {0, 63, 64, 127, 255} of both contexts' last batch vs the oracle, byte for byte."""
    from orbgpu.synth import bench_frames
    B = 256
    frames = bench_frames(1280, 720, B, first=0)
    exs = [orbgpu_mod.BatchExtractor(2000, 1280, 720, B) for _ in range(2)]
    for e in exs:
        e.upload(frames)
    for step in range(5):   # bench: warm-up, then steps alternate over the contexts without syncing
        exs[step % 2].launch()
    for e in exs:
        e.sync()
    o = oracle_mod.OracleExtractor(2000)
    ref = {f: o(frames[f]) for f in (0, 63, 64, 127, 255)}
    for e in exs:
        counts = e.counts()
        for f, (ok, od) in ref.items():
            gk, gd = e.results(f)
            assert counts[f] == len(ok)
            assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), f
    for e in exs:
        e.close()


def test_c5_bench_configuration_bit_exact(orbgpu_mod, oracle_mod):
    """bench.py --config c5: BASELINE config 5's 8-frame batch at 4,000 features, four extractor contexts
    in flight (one per hardware queue) through the hipGraph path, the small-batch kernel shapes (1024-thread
    octree blocks).  Every frame of every context vs the oracle, byte for byte."""
    from orbgpu.synth import bench_frames
    B, NF = 8, 4000
    frames = bench_frames(1280, 720, B, first=0)
    exs = [orbgpu_mod.BatchExtractor(NF, 1280, 720, B) for _ in range(4)]
    for e in exs:
        e.upload(frames)
    for step in range(10):
        exs[step % 4].launch()
    for e in exs:
        e.sync()
    o = oracle_mod.OracleExtractor(NF)
    ref = [o(frames[f]) for f in range(B)]
    for e in exs:
        for f, (ok, od) in enumerate(ref):
            gk, gd = e.results(f)
            assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), f
    for e in exs:
        e.close()


def test_c2_bench_configuration_bit_exact(orbgpu_mod, oracle_mod):
    """bench.py --config c2: 640x480 at 1,000 features, B = 256, two contexts through the graph path."""
    from orbgpu.synth import bench_frames
    B = 256
    frames = bench_frames(640, 480, B, first=0)
    exs = [orbgpu_mod.BatchExtractor(1000, 640, 480, B) for _ in range(2)]
    for e in exs:
        e.upload(frames)
    for step in range(5):
        exs[step % 2].launch()
    for e in exs:
        e.sync()
    o = oracle_mod.OracleExtractor(1000)
    ref = {f: o(frames[f]) for f in (0, 100, 255)}
    for e in exs:
        for f, (ok, od) in ref.items():
            gk, gd = e.results(f)
            assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), f
    for e in exs:
        e.close()


@pytest.mark.parametrize("w,h,nf,kind,batch", [
    (3840, 2160, 8000, "scene", False),   # level 0 has >4 chunks of cells: the octree's two-pass gather
    (4096, 4096, 8000, "noise", False),   # kMaxDim: 12-bit candidate coordinates at their limit
    (3840, 2160, 8000, "scene", True),    # the batch (graph) path at the same size
])
def test_maximum_sizes_bit_exact(orbgpu_mod, oracle_mod, w, h, nf, kind, batch):
    from orbgpu.synth import synth_frame
    img = synth_frame(w, h, 1, kind)
    ok, od = oracle_mod.OracleExtractor(nf)(img)
    if batch:
        e = orbgpu_mod.BatchExtractor(nf, w, h, 2)
        e.upload(np.stack([img, img]))
        e.launch()
        e.sync()
        for f in range(2):
            gk, gd = e.results(f)
            assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), f
        e.close()
    else:
        g = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7)
        gk, gd = g(img)
        assert len(gk) == len(ok) and gk.tobytes() == ok.tobytes() and np.array_equal(gd, od)


def test_geometry_limits_are_errors(orbgpu_mod):
    """The documented limits (include/orbgpu.h): a side above 4096 pixels, and a level whose
    octree node tables would not fit one CU's LDS (level-0 N above ~2,550: nfeatures > ~11,700 at 1.2/8)."""
    from orbgpu._lib import OrbError
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    with pytest.raises(OrbError):
        g(np.zeros((480, 4097), np.uint8))
    g = orbgpu_mod.ORBextractor(12000, 1.2, 8, 20, 7)
    with pytest.raises(OrbError):
        g(np.zeros((2160, 3840), np.uint8))


@pytest.mark.parametrize("w,h,nf,B", [(1280, 720, 4000, 1), (1280, 720, 2000, 2), (640, 480, 1000, 1)])
def test_small_batch_pyramid_plan_bit_exact(orbgpu_mod, oracle_mod, w, h, nf, B):
    """Batches of one or two frames (C5 at one frame per GPU) take the small-batch pyramid plan (orbgpu_abi.hip
    build_chain: the first levels per launch, the rest chained from the last of them in one k_pyramid_chain launch);
    keypoints, descriptors and every pyramid level are byte-identical to the oracle's."""
    from orbgpu.synth import bench_frames
    frames = bench_frames(w, h, B, first=11)
    e = orbgpu_mod.BatchExtractor(nf, w, h, B)
    e.upload(frames)
    for _ in range(2):   # the graph's capture, then a replay
        e.launch()
        e.sync()
        o = oracle_mod.OracleExtractor(nf)
        for f in range(B):
            ok, od = o(frames[f])
            gk, gd = e.results(f)
            assert gk.tobytes() == ok.tobytes() and np.array_equal(gd, od), (B, f)
            for l in range(1, 8):
                assert np.array_equal(e.debug_level_image(l, f), o.level(l)), (f, l)
    e.close()


def test_extract_capacity_contract(orbgpu_mod):
    """orb_extract with a too-small output buffer (include/orbgpu.h: ORB_ERR_CAPACITY with *n set to the required
    count, outputs untouched), then again with exactly that capacity: the same keypoints and descriptors as the
    wrapper's call."""
    import ctypes
    from orbgpu import _lib
    from orbgpu.synth import synth_frame
    img = np.ascontiguousarray(synth_frame(320, 240, 0, "scene"))
    g = orbgpu_mod.ORBextractor(500, 1.2, 8, 20, 7)
    ref_k, ref_d = g(img)
    assert len(ref_k) > 10
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    for cap in (0, 10, len(ref_k) - 1):
        kps = np.zeros(max(cap, 1), orbgpu_mod.KP_DTYPE)
        desc = np.full((max(cap, 1), 32), 7, np.uint8)
        n = ctypes.c_int(-1)
        st = _lib.lib().orb_extract(g.h, p(img), 320, 240, img.strides[0], p(kps), cap, ctypes.byref(n), p(desc))
        assert _lib.STATUS.get(st) == "ORB_ERR_CAPACITY", st
        assert n.value == len(ref_k)
        assert (desc == 7).all()
    kps = np.zeros(len(ref_k), orbgpu_mod.KP_DTYPE)
    desc = np.zeros((len(ref_k), 32), np.uint8)
    n = ctypes.c_int(-1)
    st = _lib.lib().orb_extract(g.h, p(img), 320, 240, img.strides[0], p(kps), len(ref_k), ctypes.byref(n), p(desc))
    assert st == 0 and n.value == len(ref_k)
    assert kps.tobytes() == ref_k.tobytes() and np.array_equal(desc, ref_d)


@pytest.mark.parametrize("w,h", [(160, 120), (4100, 64), (64, 4100)])
def test_extract_geometry_outside_the_reference_domain(orbgpu_mod, w, h):
    """Frames the reference's grid cannot handle are refused with ORB_ERR_GEOMETRY, not computed: at 160 x 120 the
    top level's border-trimmed width is below one 30-px cell (ComputeKeyPointsOctTree divides by nCols = 0,
    ORBextractor.cc:784-786, and DistributeOctTree by nIni = 0, :543-545); past 4096 px the candidates' packed 12-bit
    coordinates do not fit.  The context stays usable afterwards."""
    from orbgpu.synth import synth_frame
    g = orbgpu_mod.ORBextractor(500, 1.2, 8, 20, 7)
    img = np.zeros((h, w), np.uint8)
    img[::7, ::5] = 200
    with pytest.raises(orbgpu_mod.OrbError) as ei:
        g(img)
    assert ei.value.status == -4   # ORB_ERR_GEOMETRY
    k, d = g(np.ascontiguousarray(synth_frame(320, 240, 0, "scene")))
    assert len(k) > 0 and d.shape == (len(k), 32)

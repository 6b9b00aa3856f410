"""GPU parity: the birdview ORB stream (Frame.cc:318-342) — cv::ORB(HARRIS) detect,
cornerSubPix and compute through liborbgpu's bird kernels (csrc/bird.hip) vs the oracle restatement
(oracle/cvorb_oracle.inc).  Bit-exact: every KeyPoint field (float bytes) and every descriptor byte, in
order.  Parity against OpenCV itself is unpinned (tests/test_bird_oracle.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _frame(w, h, idx, kind="scene"):
    from orbgpu.synth import synth_frame
    return synth_frame(w, h, idx, kind)


def _mask(w, h, idx):
    from orbgpu.synth import synth_bird_mask
    return synth_bird_mask(w, h, idx)


@pytest.fixture(scope="module")
def bird(orbgpu_mod):
    b = orbgpu_mod.BirdORB(2000)
    yield b
    b.close()


@pytest.mark.parametrize("w,h,idx,masked", [(1280, 720, 0, False), (1280, 720, 1, True), (640, 480, 4, True)])
def test_bird_pyramid_and_candidates(orbgpu_mod, oracle_mod, bird, w, h, idx, masked):
    img = _frame(w, h, idx)
    mask = oracle_mod.bird_footprint_mask(_mask(w, h, idx)) if masked else None
    o = oracle_mod.OracleCvORB(2000)
    ko = o.detect(img, mask)
    kg = bird.detect(img, mask)
    for l in range(8):
        assert np.array_equal(bird.debug_level(l), o.level(l)), f"level {l}"
        co, cg = o.candidates(l), bird.debug_candidates(l)
        assert len(cg) == len(co), f"level {l}: {len(cg)} vs {len(co)}"
        for f in ("x", "y", "octave", "class_id"):
            assert np.array_equal(cg[f], co[f]), (l, f)
        assert cg["response"].tobytes() == co["response"].tobytes(), f"Harris level {l}"
    assert kg.tobytes() == ko.tobytes()


@pytest.mark.parametrize("w,h,idx,kind,nf", [
    (1280, 720, 2, "scene", 2000),
    (1280, 720, 3, "noise", 2000),      # maximum candidate count: large nth_element inputs
    (640, 480, 5, "scene", 500),
    (200, 150, 6, "scene", 300),         # small: the top levels fall under 2*edgeThreshold
    (641, 479, 14, "scene", 1000),       # odd sizes: unaligned rows, blur tail columns
    (1280, 720, 7, "flat", 2000),        # no corners at all
])
def test_bird_detect_bit_exact(orbgpu_mod, oracle_mod, w, h, idx, kind, nf):
    img = _frame(w, h, idx, kind)
    o = oracle_mod.OracleCvORB(nf)
    b = orbgpu_mod.BirdORB(nf)
    try:
        ko, kg = o.detect(img), b.detect(img)
        assert len(kg) == len(ko)
        assert kg.tobytes() == ko.tobytes()
    finally:
        b.close()


def test_corner_subpix_bit_exact(orbgpu_mod, oracle_mod, bird):
    img = _frame(1280, 720, 8)
    k = oracle_mod.OracleCvORB(2000).detect(img)
    pts = np.stack([k["x"], k["y"]], 1).astype(np.float32)
    rng = np.random.default_rng(0)
    extra = np.concatenate([rng.uniform(8, 1270, (300, 1)), rng.uniform(8, 710, (300, 1))], 1).astype(np.float32)
    pts = np.concatenate([pts, extra, np.array([[0.3, 0.2], [1279.4, 719.6], [6.5, 700.0]], np.float32)])
    po = oracle_mod.corner_subpix(img, pts)
    pg = bird.cornerSubPix(img, pts)
    assert pg.tobytes() == po.tobytes()
    assert (np.abs(pg - pts).sum(1) > 0).mean() > 0.5


def test_bird_compute_bit_exact(orbgpu_mod, oracle_mod, bird):
    img = _frame(1280, 720, 9)
    o = oracle_mod.OracleCvORB(2000)
    k = o.detect(img)
    kk = k.copy()[::-1]
    kk["x"][:40] += np.float32(0.37)
    kk["y"][40:80] -= np.float32(0.61)
    kk["x"][80] = 30.4
    ko, do = o.compute(img, kk)
    kg, dg = bird.compute(img, kk)
    assert kg.tobytes() == ko.tobytes()
    assert np.array_equal(dg, do)


@pytest.mark.parametrize("w,h,idx,masked", [(1280, 720, 10, True), (1280, 720, 11, False), (640, 480, 12, True),
                                             (643, 477, 15, True)])
def test_bird_extract_fused_bit_exact(orbgpu_mod, oracle_mod, bird, w, h, idx, masked):
    """Frame.cc:320-342 end to end: footprint, masked detect, cornerSubPix, border cull, descriptors."""
    img = _frame(w, h, idx)
    mask = _mask(w, h, idx) if masked else None
    ko, do = oracle_mod.OracleCvORB(2000).extract(img, mask)
    kg, dg = bird.extract(img, mask)
    assert len(kg) == len(ko) > 100
    assert kg.tobytes() == ko.tobytes()
    assert np.array_equal(dg, do)
    if mask is not None:   # the caller's mask is not modified (the footprint is drawn on the device copy)
        assert np.array_equal(mask, _mask(w, h, idx))


def test_bird_extract_device_resident(orbgpu_mod, oracle_mod, bird):
    import torch
    img, mask = _frame(1280, 720, 13), _mask(1280, 720, 13)
    di = torch.from_numpy(img).cuda()
    dm = torch.from_numpy(mask).cuda()
    torch.cuda.synchronize()
    kg, dg = bird.extract_device(di.data_ptr(), 1280, 720, dm.data_ptr())
    ko, do = oracle_mod.OracleCvORB(2000).extract(img, mask)
    assert kg.tobytes() == ko.tobytes()
    assert np.array_equal(dg, do)


def test_bird_empty_and_capacity(orbgpu_mod, bird):
    k = bird.detect(np.zeros((0, 0), np.uint8))
    assert len(k) == 0
    kk, d = bird.extract(np.full((300, 400), 77, np.uint8))
    assert len(kk) == 0 and d.shape == (0, 32)


def test_bird_stream_into_birdview_match(orbgpu_mod, oracle_mod, bird):
    """Birdview chain of Tracking (Tracking.cc:744 BirdviewMatch(LastFrame, CurrentFrame, ..., 15)): both
    frames' birdview features from the GPU stream, candidates from the birdview grid, the windowed
    matcher on the GPU — equal to the oracle chain."""
    w, h = 640, 480
    a = _frame(w, h, 20)
    rng = np.random.default_rng(20)
    b = np.clip(np.roll(a, (2, 3), axis=(0, 1)).astype(np.int16) + rng.integers(-2, 3, a.shape), 0, 255).astype(np.uint8)
    mask = _mask(w, h, 20)
    ka, da = bird.extract(a, mask)
    kb, db = bird.extract(b, mask)
    oka, oda = oracle_mod.OracleCvORB(2000).extract(a, mask)
    okb, odb = oracle_mod.OracleCvORB(2000).extract(b, mask)
    assert ka.tobytes() == oka.tobytes() and kb.tobytes() == okb.tobytes()
    assert np.array_equal(da, oda) and np.array_equal(db, odb)
    offs, idxs = [0], []
    for k in ka:   # Frame::GetFeaturesInAreaBirdview over the birdview grid (the whole image)
        c = orbgpu_mod.features_in_area(kb, 0, w, 0, h, float(k["x"]), float(k["y"]), 15, -1, -1)
        idxs.extend(c.tolist())
        offs.append(len(idxs))
    off = np.array(offs, np.int32)
    cand = np.array(idxs, np.int32)
    m = orbgpu_mod.ORBmatcher(0.9, True)
    n, mm = m.BirdviewMatch(da, ka, db, kb, off, cand)
    on, om = oracle_mod.window_match(0.9, True, False, da, ka, db, kb, off, cand)
    assert n == on and np.array_equal(mm, om)
    assert n > 200

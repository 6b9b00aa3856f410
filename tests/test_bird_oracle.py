"""Oracle checks of the birdview stream restatement (Frame.cc:318-342):
OpenCV-3.2 cv::ORB (HARRIS_SCORE) detect/compute and cv::cornerSubPix in oracle/cvorb_oracle.inc.

Parity against OpenCV itself is UNPINNED (OpenCV is absent, the reference holds no fixture for this
stream).  These tests pin what is derivable: the footprint rectangle from Frame.cc's constants, the
cv::ORB geometry / per-level budgets, the retainBest selection as a set, and cornerSubPix converging on
analytically rendered corners.  Also checks the product's host-only footprint helper against it."""
import numpy as np
import pytest


def _scene(w, h, idx):
    from orbgpu.synth import synth_frame
    return synth_frame(w, h, idx)


def test_footprint_rectangle_kat(oracle_mod):
    # Frame.cc:320-327 with pixel2meter = 0.03984*1.7, vehicle 1.901 x 4.63 m, 15 px boundary:
    # x = 640 - 14.03 - 15 = 610.97 -> 610, w = 28.07 + 30 -> 58; y = 360 - 34.18 - 15 -> 310, h -> 98
    m = oracle_mod.bird_footprint_mask(np.full((720, 1280), 255, np.uint8))
    ys, xs = np.nonzero(m == 0)
    assert (ys.min(), ys.max() + 1, xs.min(), xs.max() + 1) == (310, 408, 610, 668)
    assert (m == 0).sum() == 98 * 58


def test_footprint_product_helper_matches_oracle(orbgpu_mod, oracle_mod):
    # host-only C-ABI helper (no GPU call): orb_bird_footprint_mask
    for w, h in ((1280, 720), (640, 480), (50, 40), (400, 900)):
        base = np.random.default_rng(w).integers(0, 256, (h, w)).astype(np.uint8)
        assert np.array_equal(orbgpu_mod.bird_footprint_mask(base), oracle_mod.bird_footprint_mask(base))


def test_cvorb_level_geometry_and_budgets(oracle_mod):
    o = oracle_mod.OracleCvORB(2000)
    img = _scene(1280, 720, 3)
    k = o.detect(img)
    sizes = [o.level(l).shape[::-1] for l in range(8)]
    # cvRound(cols / (float)pow(1.2f, l))
    assert sizes == [(1280, 720), (1067, 600), (889, 500), (741, 417), (617, 347), (514, 289), (429, 241),
                     (357, 201)]
    # nfeaturesPerLevel for 2000 features: a scene frame fills every budget exactly (Harris ties are rare)
    assert np.bincount(k["octave"], minlength=8).tolist() == [434, 362, 302, 251, 209, 175, 145, 122]
    scale = np.float32(1.2) ** np.arange(8, dtype=np.float32)
    assert np.all(k["size"] == (np.float32(31) * np.array([np.float32(np.power(np.float64(np.float32(1.2)), l))
                                                            for l in range(8)], np.float32))[k["octave"]])
    assert np.all(k["class_id"] == -1)
    assert np.all((k["angle"] >= 0) & (k["angle"] < 360))
    del scale


@pytest.mark.parametrize("idx", [0, 5])
def test_cvorb_selection_is_retain_best(oracle_mod, idx):
    """Per level: KeyPointsFilter::retainBest(2N) on the FAST score, then retainBest(N) on Harris
    (orb.cpp computeKeyPoints).  Which of the tied elements at a boundary survive is nth_element's
    arrangement (libstdc++), so the check is on the bounds every implementation satisfies: the kept set F
    has >= N members, all with FAST >= t (the 2N-th best score), and every candidate strictly above t that
    was dropped has a Harris response <= min Harris of F."""
    o = oracle_mod.OracleCvORB(2000)
    k = o.detect(_scene(1280, 720, idx))
    nper = [434, 362, 302, 251, 209, 175, 145, 122]
    for l in range(8):
        c = o.candidates(l)
        kl = k[k["octave"] == l]
        s = np.float32(np.power(np.float64(np.float32(1.2)), l))
        key = {(float(np.float32(x) * s), float(np.float32(y) * s)): i for i, (x, y) in enumerate(zip(c["x"], c["y"]))}
        sel = np.array([key[(float(x), float(y))] for x, y in zip(kl["x"], kl["y"])], np.int64)
        assert len(set(sel.tolist())) == len(sel)
        assert np.array_equal(kl["response"], c["response"][sel])      # Harris carried through
        fast = c["class_id"].astype(np.int64)
        assert len(sel) >= min(nper[l], len(c))
        t = np.sort(fast)[::-1][2 * nper[l] - 1] if len(c) > 2 * nper[l] else -1
        assert np.all(fast[sel] >= t)
        dropped = np.setdiff1d(np.nonzero(fast > t)[0], sel)
        if len(dropped) and len(sel):
            assert c["response"][dropped].max() <= c["response"][sel].min()


def test_cvorb_detect_border_and_mask(oracle_mod):
    from orbgpu.synth import synth_bird_mask
    img = _scene(1280, 720, 9)
    mask = oracle_mod.bird_footprint_mask(synth_bird_mask(1280, 720, 9))
    o = oracle_mod.OracleCvORB(2000)
    k = o.detect(img, mask)
    assert len(k) > 1500
    for l in range(8):
        c = o.candidates(l)
        lv = o.level(l)
        h, w = lv.shape
        assert np.all((c["x"] >= 31) & (c["x"] < w - 31) & (c["y"] >= 31) & (c["y"] < h - 31))
    # level-0 keypoints never sit on a masked pixel
    k0 = k[k["octave"] == 0]
    assert np.all(mask[k0["y"].astype(int), k0["x"].astype(int)] != 0)
    # an all-zero mask leaves nothing; an empty image gives nothing
    assert len(o.detect(img, np.zeros_like(mask))) == 0
    assert len(o.detect(np.full((720, 1280), 128, np.uint8))) == 0


def _render_corner(w, h, cx, cy, lo=40, hi=200, ss=16):
    """Saddle (checkerboard) corner at (cx, cy), area-sampled with ss x ss supersampling."""
    ys = (np.arange(h * ss) + 0.5) / ss - 0.5
    xs = (np.arange(w * ss) + 0.5) / ss - 0.5
    q = ((xs[None, :] >= cx) ^ (ys[:, None] >= cy)).astype(np.float64)
    img = q.reshape(h, ss, w, ss).mean(axis=(1, 3))
    return np.round(lo + (hi - lo) * img).astype(np.uint8)


@pytest.mark.parametrize("cx,cy", [(40.3, 30.7), (41.5, 33.25), (38.9, 29.1)])
def test_corner_subpix_converges_on_rendered_corner(oracle_mod, cx, cy):
    img = _render_corner(80, 64, cx, cy)
    p = oracle_mod.corner_subpix(img, np.array([[round(cx), round(cy)]], np.float32))
    assert abs(p[0, 0] - cx) < 0.12 and abs(p[0, 1] - cy) < 0.12, p   # u8 quantisation bias


def test_corner_subpix_resets_far_moves(oracle_mod):
    # a flat image: det == 0 on the first iteration -> the point is returned unchanged
    img = np.full((64, 64), 90, np.uint8)
    p = oracle_mod.corner_subpix(img, np.array([[30.0, 31.0], [20.5, 40.25]], np.float32))
    assert np.array_equal(p, np.array([[30.0, 31.0], [20.5, 40.25]], np.float32))


def test_cvorb_compute_culls_and_sorts(oracle_mod):
    img = _scene(640, 480, 2)
    o = oracle_mod.OracleCvORB(500)
    k = o.detect(img)
    kk = k.copy()[::-1]                       # unsorted by level
    kk[0]["x"] = 30.4                         # cvRound -> 30 < 31: culled
    kk[1]["x"] = 30.6                         # cvRound -> 31: kept
    out, desc = o.compute(img, kk)
    assert len(out) == len(kk) - 1
    assert np.all(np.diff(out["octave"]) >= 0)
    assert desc.shape == (len(out), 32)
    # stable bucket sort: within a level the input order is kept
    for l in range(8):
        a = kk[(kk["octave"] == l)]
        a = a[~((a["x"] == np.float32(30.4)))]
        assert np.array_equal(out[out["octave"] == l], a)

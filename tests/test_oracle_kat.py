"""CPU: pin the oracle restatement against every known-answer constant derivable from the reference
 and against the committed golden fixtures (tests/golden, made by tools/gen_golden.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

# ORBextractor.cc:454-469, computed in the survey session and re-derived here
UMAX = [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
# mnFeaturesPerLevel (ORBextractor.cc:435-446), SURVEY §8a a1
NPL = {1000: [217, 181, 151, 126, 105, 87, 73, 60],
       2000: [434, 362, 302, 251, 209, 175, 145, 122],
       4000: [869, 724, 603, 503, 419, 349, 291, 242]}
# ComputePyramid level sizes (ORBextractor.cc:1112), SURVEY Appendix B
PYR = {(640, 480): [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)],
       (1280, 720): [(1280, 720), (1067, 600), (889, 500), (741, 417), (617, 347), (514, 289), (429, 241),
                     (357, 201)]}


@pytest.mark.parametrize("nf", sorted(NPL))
def test_features_per_level(oracle_mod, nf):
    t = oracle_mod.OracleExtractor(nf).tables()
    assert t["n_per_level"].tolist() == NPL[nf]
    assert t["umax"].tolist() == UMAX


def test_scale_tables(oracle_mod):
    t = oracle_mod.OracleExtractor(1000).tables()
    # float * double products rounded to float (ORBextractor.cc:421, h:98)
    s = [np.float32(1.0)]
    for i in range(1, 8):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(1.2))))
    assert np.array_equal(t["scale"], np.array(s, np.float32))
    assert np.array_equal(t["sigma2"], (np.array(s, np.float32) * np.array(s, np.float32)).astype(np.float32))
    assert np.array_equal(t["inv_scale"], (np.float32(1) / np.array(s, np.float32)).astype(np.float32))


@pytest.mark.parametrize("size", sorted(PYR))
def test_pyramid_sizes(oracle_mod, size):
    from orbgpu.synth import synth_frame
    w, h = size
    e = oracle_mod.OracleExtractor(1000)
    e.run(synth_frame(w, h, 0))
    assert [e.level(l).shape[::-1] for l in range(8)] == PYR[size]


def _cells(w, h):
    mx, my = w - 16, h - 16
    W, H = np.float32(mx - 16), np.float32(my - 16)
    nc, nr = int(W / np.float32(30)), int(H / np.float32(30))
    return nc * nr


def test_cell_counts():
    # FAST cells total 815 (640x480) and 2656 (1280x720)
    assert sum(_cells(w, h) for w, h in PYR[(640, 480)]) == 815
    assert sum(_cells(w, h) for w, h in PYR[(1280, 720)]) == 2656


def test_pattern_checksum(oracle_mod):
    p = oracle_mod.pattern()
    assert p.sum() == -406 and p.min() == -13 and p.max() == 12
    # |rotated offset| <= 18 < 19-px keypoint margin
    pts = p.reshape(-1, 2).astype(np.float64)
    assert np.hypot(pts[:, 0], pts[:, 1]).max() < 18.5


def test_pattern_tables_identical():
    # the oracle's and the product's transcriptions of bit_pattern_31_ must agree
    root = os.path.dirname(GOLDEN)
    a = open(os.path.join(root, "..", "oracle", "pattern31_data.inc")).read().split("\\\n", 1)[1]
    b = open(os.path.join(root, "..", "orb-slam-birdview_amd", "csrc", "pattern31_data.inc")).read().split("\\\n", 1)[1]
    assert a == b


def test_descriptor_distance_kat(oracle_mod):
    z = np.zeros(32, np.uint8)
    o = np.full(32, 255, np.uint8)
    assert oracle_mod.descriptor_distance(z, o) == 256
    assert oracle_mod.descriptor_distance(z, z) == 0
    one = z.copy()
    one[17] = 8
    assert oracle_mod.descriptor_distance(z, one) == 1
    rng = np.random.default_rng(1)
    for _ in range(50):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert oracle_mod.descriptor_distance(a, b) == int(np.unpackbits(a ^ b).sum())


def test_fast_atan2_kat(oracle_mod):
    f = oracle_mod.fast_atan2
    assert f(0.0, 0.0) == 0.0
    assert f(0.0, 1.0) == 0.0
    assert abs(f(1.0, 0.0) - 90.0) < 1e-4
    assert abs(f(0.0, -1.0) - 180.0) < 1e-4
    assert abs(f(-1.0, 0.0) - 270.0) < 1e-4
    assert abs(f(1.0, 1.0) - 45.0) < 0.01
    for y, x in [(3.0, 4.0), (-5.0, 2.0), (7.0, -1.0), (-2.0, -9.0)]:
        ref = np.degrees(np.arctan2(y, x)) % 360
        assert abs(f(y, x) - ref) < 0.02   # OpenCV's documented ~0.3 deg accuracy


def _corner_patch(delta, bright=True, arc=9, v=100):
    img = np.full((7, 7), v, np.uint8)
    circle = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
              (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    for k in range(arc):
        x, y = circle[k]
        img[3 + y, 3 + x] = v + delta if bright else v - delta
    return img


def test_fast_score_kat(oracle_mod):
    # 9-arc of +delta: corner at th < delta with score delta-1
    for d in (10, 21, 40):
        out = oracle_mod.fast_roi(_corner_patch(d), 20)
        if d > 20:
            assert out.tolist() == [[3, 3, d - 1]]
        else:
            assert len(out) == 0
    # a pixel exactly at threshold is not a corner (strict >)
    assert len(oracle_mod.fast_roi(_corner_patch(20), 20)) == 0
    assert len(oracle_mod.fast_roi(_corner_patch(21, bright=False), 20)) == 1
    # an 8-arc is not a corner
    assert len(oracle_mod.fast_roi(_corner_patch(50, arc=8), 20)) == 0


def test_three_maxima_kat(oracle_mod):
    tm = oracle_mod.three_maxima
    assert tm([0] * 30) == (-1, -1, -1)
    h = [0] * 30
    h[4], h[7], h[9] = 10, 5, 3
    assert tm(h) == (4, 7, 9)
    h[9] = 0
    h[7] = 0
    h[3] = 1   # 1 < 0.1*10 is false: kept
    assert tm(h) == (4, 3, -1)
    h[4] = 20  # 1 < 0.1*20: second dropped
    assert tm(h) == (4, -1, -1)
    h = [0] * 30
    h[1], h[2], h[3] = 20, 2, 1
    assert tm(h) == (1, 2, -1)
    h = [0] * 30
    h[5], h[6] = 3, 3   # ties keep the first (strict >)
    assert tm(h)[0] == 5


def test_rotation_bin_quirk(oracle_mod):
    # bin = round(rot * (1/30)): only bins 0..12 are used (upstream ORB-SLAM2 behaviour)
    assert oracle_mod.rot_bin(45.0, 0.0) == 2
    assert oracle_mod.rot_bin(0.0, 1.0) == 12
    assert oracle_mod.rot_bin(10.0, 10.0) == 0
    assert max(oracle_mod.rot_bin(a, 0.0) for a in np.linspace(0, 359.9, 500)) == 12


def test_blur_kernel_sum_257(oracle_mod):
    # The 8-bit 7x7 sigma-2 kernel is [18,34,49,55,49,34,18] (sum 257): a flat 100 blurs to 101
    img = np.full((20, 24), 100, np.uint8)
    assert (oracle_mod.blur(img) == 101).all()
    img[:] = 255
    assert (oracle_mod.blur(img) == 255).all()


def test_blur_tail_rounding(oracle_mod):
    # the SSE2 column body (x < W & ~3) rounds half-to-even, the scalar tail half-up:
    # a half-way sum shows up only where the column parity differs.
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (40, 43), dtype=np.uint8)
    a = oracle_mod.blur(img)
    b = oracle_mod.blur(img, oracle_mod.BLUR_ALL_HALFUP)
    assert np.array_equal(a[:, 40:], b[:, 40:])
    assert (a[:, :40] <= b[:, :40]).all()


def test_resize_identity_and_constant(oracle_mod):
    img = np.full((48, 64), 77, np.uint8)
    assert (oracle_mod.resize(img, 53, 40) == 77).all()
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (48, 64), dtype=np.uint8)
    assert np.array_equal(oracle_mod.resize(img, 64, 48), img)


def test_empty_and_flat(oracle_mod):
    e = oracle_mod.OracleExtractor(1000)
    assert e.run(np.zeros((0, 0), np.uint8)) == -1
    n = e.run(np.full((480, 640), 128, np.uint8))
    assert n == 0


def test_degenerate_geometry(oracle_mod):
    e = oracle_mod.OracleExtractor(1000)
    assert e.run(np.full((120, 160), 128, np.uint8)) == -2   # level 7 narrower than 62 px


def test_synth_deterministic():
    from orbgpu.synth import synth_frame, SplitMix64
    a = synth_frame(320, 240, 3)
    b = synth_frame(320, 240, 3)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, synth_frame(320, 240, 4))
    # counter-based draws equal the sequential splitmix64 stream
    r = SplitMix64(0x5EED0000)
    seq = []
    state = 0x5EED0000
    for _ in range(4):
        state = (state + 0x9E3779B97F4A7C15) & (2 ** 64 - 1)
        z = state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2 ** 64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2 ** 64 - 1)
        seq.append(z ^ (z >> 31))
    assert r.draw(4).tolist() == seq


def _golden(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} missing (run tools/gen_golden.py)")
    return np.load(path, allow_pickle=False)


@pytest.mark.parametrize("name", ["extract_320x240_500.npz", "extract_640x480_1000.npz", "extract_noise_640x480.npz"])
def test_oracle_matches_golden(oracle_mod, name):
    from orbgpu.synth import synth_frame
    g = _golden(name)
    w, h, nf, idx = [int(v) for v in g["cfg"]]
    kind = str(g["kind"])
    img = synth_frame(w, h, idx, kind)
    import hashlib
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["img_sha256"])
    k, d = oracle_mod.OracleExtractor(nf)(img)
    assert k.tobytes() == g["kps"].tobytes()
    assert np.array_equal(d, g["desc"])


def test_oracle_stereo_golden(oracle_mod):
    """Frame::ComputeStereoMatches restatement (Frame.cc:662-836) against its committed vectors."""
    import hashlib
    from orbgpu.synth import synth_frame, synth_stereo_right
    g = _golden("stereo_640x480.npz")
    w, h, nf, idx = [int(v) for v in g["cfg"]]
    left = synth_frame(w, h, idx)
    right = synth_stereo_right(left, idx)
    assert hashlib.sha256(left.tobytes()).hexdigest() == str(g["left_sha256"])
    assert hashlib.sha256(right.tobytes()).hexdigest() == str(g["right_sha256"])
    ol, orr = oracle_mod.OracleExtractor(nf), oracle_mod.OracleExtractor(nf)
    kl, dl = ol(left)
    kr, dr = orr(right)
    u, d, n = oracle_mod.stereo_matches(ol, orr, kl, dl, kr, dr, float(g["mb"]), float(g["mbf"]))
    assert n == int(g["n"]) and u.tobytes() == g["uright"].tobytes() and d.tobytes() == g["depth"].tobytes()


def test_oracle_stereo_kat(oracle_mod):
    """Identical views: every window distance is 0, the median is 0 and the 1.5*1.4*median cut
    (Frame.cc:822-835) rejects every match; accepted depths satisfy depth = mbf / (uL - uR)."""
    from orbgpu.synth import synth_frame, synth_stereo_right
    left = synth_frame(320, 240, 4)
    ol, orr = oracle_mod.OracleExtractor(500), oracle_mod.OracleExtractor(500)
    kl, dl = ol(left)
    kr, dr = orr(left.copy())
    u, d, n = oracle_mod.stereo_matches(ol, orr, kl, dl, kr, dr, 0.1, 50.0)
    assert n == 0 and (u == -1).all() and (d == -1).all()
    right = synth_stereo_right(left, 4)
    kr, dr = orr(right)
    u, d, n = oracle_mod.stereo_matches(ol, orr, kl, dl, kr, dr, 0.1, 50.0)
    ok = u >= 0
    assert n == ok.sum() > 0
    disp = kl["x"][ok] - u[ok]
    assert np.all(disp >= 0) and np.all(disp < 500.0)
    assert np.array_equal(d[ok], (np.float32(50.0) / disp.astype(np.float32)).astype(np.float32))


def test_oracle_vocab_loader_and_descent_kat(oracle_mod, tmp_path):
    """TemplatedVocabulary::loadFromBinaryFile (TemplatedVocabulary.h:1466-1510): nb_nodes - 1
    records plus the while(!eof) duplicate of the last one (one extra node and word); a feature equal
    to a leaf's stored descriptor whose path is unambiguous descends to that leaf; the L1-normalised
    TF-IDF BowVector sums to 1."""
    import struct
    from orbgpu.synth import write_synth_vocab
    path = str(tmp_path / "v.bin")
    nb, nw = write_synth_vocab(path, 4, 3, seed=7, stop_frac=0.0)
    v = oracle_mod.OracleVocabulary(path)
    assert (v.k, v.L) == (4, 3) and v.nnodes == nb + 1 and v.nwords == nw + 1
    raw = open(path, "rb").read()
    recs = [raw[24 + 41 * i:24 + 41 * (i + 1)] for i in range(nb - 1)]
    leaves = [(i + 1, np.frombuffer(r[4:36], np.uint8)) for i, r in enumerate(recs) if r[40]]
    wid, wt, nid = v.transform_each(np.stack([d for _, d in leaves]), 0)
    # leaves are numbered breadth-first after the internal nodes: word id = leaf order
    ok = wid == np.arange(len(leaves))
    assert ok.mean() > 0.9
    # levelsup 0 -> nid_level = L: the FeatureVector node is the leaf itself
    assert np.array_equal(nid[ok], np.array([i for i, _ in leaves])[ok])
    _, _, nid_root = v.transform_each(np.stack([d for _, d in leaves]), 3)   # nid_level <= 0 -> root
    assert (nid_root == 0).all()
    bow, fv = v.transform(np.stack([d for _, d in leaves]), 1)
    assert abs(sum(bow.values()) - 1.0) < 1e-12
    assert sum(len(x) for x in fv.values()) == len(leaves)
    assert struct.unpack("<6i", raw[:24])[1] == 41


def test_oracle_distinctive_descriptor_kat(oracle_mod):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307): median index (int)(0.5*(N-1));
    N = 1, 2 -> 0 (median 0 for every row); three descriptors a, a', b with a' one bit from a -> a."""
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, 32, dtype=np.uint8)
    b = ~a
    a2 = a.copy()
    a2[0] ^= 1
    assert oracle_mod.distinctive_descriptor(np.zeros((0, 32), np.uint8)) == -1
    assert oracle_mod.distinctive_descriptor(a[None]) == 0
    assert oracle_mod.distinctive_descriptor(np.stack([b, a])) == 0
    assert oracle_mod.distinctive_descriptor(np.stack([b, a2, a])) == 1   # rows: b->[0,255,256] a2->[0,1,255] a->[0,1,256]

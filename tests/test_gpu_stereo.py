"""GPU parity: Frame::ComputeStereoMatches (Frame.cc:662-836) through liborbgpu's
stereo kernels vs the oracle restatement — mvuRight / mvDepth bit-identical (float32 bytes), on the
host-image path (two extractor contexts) and the device-resident batched path (frame pairs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MB = 0.12           # baseline (m)
FX = 500.0


def _pair(w, h, idx, kind="shifted"):
    from orbgpu.synth import synth_frame, synth_stereo_right
    left = synth_frame(w, h, idx)
    if kind == "same":        # identical views: every window distance is 0, so the median cut (:822-835)
        return left, left.copy()   # rejects all of them (the reference's own behaviour)
    if kind == "near":        # zero disparity plus noise: disparities around 0 (the <= 0 -> 0.01 branch, :811-815)
        rng = np.random.default_rng(idx)
        return left, np.clip(left.astype(np.int16) + rng.integers(-2, 3, left.shape), 0, 255).astype(np.uint8)
    return left, synth_stereo_right(left, idx)


def _oracle(oracle_mod, left, right, nf):
    ol, orr = oracle_mod.OracleExtractor(nf), oracle_mod.OracleExtractor(nf)
    kl, dl = ol(left)
    kr, dr = orr(right)
    u, d, n = oracle_mod.stereo_matches(ol, orr, kl, dl, kr, dr, MB, MB * FX)
    return kl, dl, kr, dr, u, d, n


@pytest.mark.parametrize("w,h,nf,idx,kind", [
    (640, 480, 1000, 3, "shifted"),
    (640, 480, 1000, 8, "shifted"),
    (1280, 720, 2000, 1, "shifted"),
    (1280, 720, 4000, 2, "shifted"),
    (640, 480, 1000, 5, "same"),
    (640, 480, 1000, 6, "near"),
])
def test_stereo_matches_bit_exact(orbgpu_mod, oracle_mod, w, h, nf, idx, kind):
    left, right = _pair(w, h, idx, kind)
    kl, dl, kr, dr, ou, od, on = _oracle(oracle_mod, left, right, nf)
    gl = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7)
    gr = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7)
    gkl, gdl = gl(left)
    gkr, gdr = gr(right)
    assert gkl.tobytes() == kl.tobytes() and gkr.tobytes() == kr.tobytes()
    u, d, n = orbgpu_mod.compute_stereo_matches(gl, gr, gkl, gdl, gkr, gdr, MB, MB * FX)
    assert n == on, (n, on)
    assert n > 20 if kind != "same" else n == 0
    assert u.tobytes() == ou.tobytes(), np.flatnonzero(u != ou)[:10]
    assert d.tobytes() == od.tobytes()


def test_stereo_batch_device_matches_host_path(orbgpu_mod, oracle_mod):
    w, h, nf, npairs = 640, 480, 1000, 3
    pairs = [_pair(w, h, 20 + p) for p in range(npairs)]
    frames = np.stack([f for pr in pairs for f in pr])
    bx = orbgpu_mod.BatchExtractor(nf, w, h, 2 * npairs)
    bx.upload(frames)
    bx.launch()
    L = orbgpu_mod._lib.lib()
    cap = bx.kp_cap
    du, dd, dn = bx._alloc(npairs * cap * 4), bx._alloc(npairs * cap * 4), bx._alloc(npairs * 4)
    bx.stereo(npairs, MB, MB * FX, du, dd, dn)
    bx.sync()
    u = np.zeros(npairs * cap, np.float32)
    d = np.zeros(npairs * cap, np.float32)
    n = np.zeros(npairs, np.int32)
    for dst, src in ((u, du), (d, dd), (n, dn)):
        orbgpu_mod._lib.check(L.orb_memcpy_d2h(bx.h, dst.ctypes.data, src, dst.nbytes))
    for p, (left, right) in enumerate(pairs):
        kl, dl, kr, dr, ou, od, on = _oracle(oracle_mod, left, right, nf)
        k = len(kl)
        assert n[p] == on
        assert u[p * cap:p * cap + k].tobytes() == ou.tobytes()
        assert d[p * cap:p * cap + k].tobytes() == od.tobytes()
    for ptr in (du, dd, dn):
        L.orb_device_free(bx.h, ptr)
    bx.close()


def test_stereo_rejects_mismatched_contexts(orbgpu_mod):
    from orbgpu.synth import synth_frame
    a = orbgpu_mod.ORBextractor(500, 1.2, 8, 20, 7)
    b = orbgpu_mod.ORBextractor(500, 1.2, 8, 20, 7)
    ka, da = a(synth_frame(640, 480, 1))
    kb, db = b(synth_frame(320, 240, 1))
    with pytest.raises(orbgpu_mod.OrbError):
        orbgpu_mod.compute_stereo_matches(a, b, ka, da, kb, db, MB, MB * FX)


def test_stereo_no_left_keypoints(orbgpu_mod):
    from orbgpu.synth import synth_frame
    a = orbgpu_mod.ORBextractor(500, 1.2, 8, 20, 7)
    b = orbgpu_mod.ORBextractor(500, 1.2, 8, 20, 7)
    ka, da = a(np.full((480, 640), 128, np.uint8))
    kb, db = b(synth_frame(640, 480, 1))
    u, d, n = orbgpu_mod.compute_stereo_matches(a, b, ka, da, kb, db, MB, MB * FX)
    assert len(u) == 0 and n == 0


@pytest.mark.parametrize("mode", ["staged_one_device", "two_devices"])
def test_stereo_right_extractor_on_another_device(orbgpu_mod, oracle_mod, monkeypatch, mode):
    """C4 places each camera stream on its own GPU: the right image and pyramid then move to the left
    device (hipMemcpyPeerAsync) before the window search.  On a one-GPU box the same staging is forced
    with ORBGPU_STEREO_STAGE=1; with two GPUs the right extractor runs on device 1."""
    ndev = orbgpu_mod.device_count()
    if mode == "two_devices" and ndev < 2:
        pytest.skip("one GPU visible")
    if mode == "staged_one_device":
        monkeypatch.setenv("ORBGPU_STEREO_STAGE", "1")
    left, right = _pair(1280, 720, 4)
    kl, dl, kr, dr, ou, od, on = _oracle(oracle_mod, left, right, 2000)
    gl = orbgpu_mod.ORBextractor(2000, 1.2, 8, 20, 7, device=0)
    gr = orbgpu_mod.ORBextractor(2000, 1.2, 8, 20, 7, device=1 if mode == "two_devices" else 0)
    gkl, gdl = gl(left)
    gkr, gdr = gr(right)
    assert gkr.tobytes() == kr.tobytes() and np.array_equal(gdr, dr)
    u, d, n = orbgpu_mod.compute_stereo_matches(gl, gr, gkl, gdl, gkr, gdr, MB, MB * FX)
    assert n == on > 20
    assert u.tobytes() == ou.tobytes() and d.tobytes() == od.tobytes()

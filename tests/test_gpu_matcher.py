"""GPU parity: ORBmatcher searches through liborbgpu's Hamming kernels vs the oracle restatement of
ORBmatcher.cc — match indices bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _diff(got, want, best=None):
    """First mismatches of two distance arrays (for assertion messages)."""
    got, want = np.asarray(got), np.asarray(want)
    bad = np.flatnonzero(got != want)[:8]
    return {"n_bad": int((got != want).sum()), "at": bad.tolist(), "got": got[bad].tolist(), "want": want[bad].tolist(),
            "best_there": None if best is None else np.asarray(best)[bad].tolist()}


@pytest.fixture(scope="module")
def frames(orbgpu_mod):
    """Two extracted views (second shifted by a few px) -> realistic descriptor sets with matches."""
    from orbgpu.synth import synth_frame
    a = synth_frame(640, 480, 40)
    b = np.roll(a, (3, 5), axis=(0, 1))
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    ka, da = g(a)
    kb, db = g(b)
    return ka, da, kb, db


def _featvec(desc, nodes=16, seed=0):
    """Synthetic vocabulary: node = high nibble of descriptor byte 0 (similar descriptors share nodes)."""
    fv = {}
    for i, d in enumerate(desc):
        fv.setdefault(int(d[0] >> 4) % nodes, []).append(i)
    return fv


def _oracle_fv(oracle_mod, fv):
    ids = sorted(fv)
    return oracle_mod.make_featvec(ids, [fv[i] for i in ids])


def test_hamming_topk_vs_numpy(orbgpu_mod):
    rng = np.random.default_rng(0)
    q = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    t[::7] = t[0]   # many exact ties
    m = orbgpu_mod.ORBmatcher()
    D = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(2)
    for k in (1, 2, 5, 8):
        dist, idx, nv = m.hamming_topk(q, t, k)
        order = np.lexsort((np.broadcast_to(np.arange(700), D.shape), D), axis=1)[:, :k]
        assert np.array_equal(idx, order)
        assert np.array_equal(dist, np.take_along_axis(D, order, 1))
        assert (nv == 700).all()


def test_hamming_topk_csr_and_thresholds(orbgpu_mod):
    rng = np.random.default_rng(1)
    q = rng.integers(0, 256, (64, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    lens = rng.integers(0, 30, 64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    cand = rng.integers(0, 200, off[-1]).astype(np.int32)
    thr = np.where(rng.random(200) < 0.3, -1, 2 ** 31 - 1).astype(np.int32)
    thr[::11] = 120
    m = orbgpu_mod.ORBmatcher()
    dist, idx, nv = m.hamming_topk(q, t, 4, off, cand, thr)
    for i in range(64):
        c = cand[off[i]:off[i + 1]]
        d = np.unpackbits(q[i][None] ^ t[c], axis=1).sum(1)
        keep = thr[c] > d
        pos = np.nonzero(keep)[0]
        order = pos[np.lexsort((pos, d[pos]))][:4]
        assert nv[i] == keep.sum()
        exp_i = np.full(4, -1)
        exp_d = np.full(4, -1)
        exp_i[:len(order)] = c[order]
        exp_d[:len(order)] = d[order]
        assert idx[i].tolist() == exp_i.tolist() and dist[i].tolist() == exp_d.tolist(), i


def test_top2_device_vs_numpy(orbgpu_mod):
    from orbgpu import _lib
    rng = np.random.default_rng(2)
    nq, nt = 1000, 2300
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    t[1500] = q[3]
    t[2200] = q[3]
    b = orbgpu_mod.BatchExtractor(1000, 640, 480, 1)
    L = _lib.lib()
    dq, dt = b._alloc(q.nbytes), b._alloc(t.nbytes)
    out = [b._alloc(nq * 4) for _ in range(3)]
    L.orb_memcpy_h2d(b.h, dq, q.ctypes.data, q.nbytes)
    L.orb_memcpy_h2d(b.h, dt, t.ctypes.data, t.nbytes)
    b.hamming_top2(dq, nq, dt, nt, *out)
    b.sync()
    res = [np.zeros(nq, np.int32) for _ in range(3)]
    for r, d in zip(res, out):
        L.orb_memcpy_d2h(b.h, r.ctypes.data, d, nq * 4)
    D = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(2)
    srt = np.sort(D, 1)
    assert np.array_equal(res[0], srt[:, 0])
    assert np.array_equal(res[1], D.argmin(1))   # first index on ties
    assert np.array_equal(res[2], srt[:, 1]), _diff(res[2], srt[:, 1], res[0])
    assert res[1][3] == 1500
    for p in [dq, dt] + out:
        L.orb_device_free(b.h, p)
    b.close()


@pytest.mark.parametrize("ratio,check_ori", [(0.7, True), (0.75, True), (0.6, False), (0.99, True)])
def test_search_by_bow_kf_f(orbgpu_mod, oracle_mod, frames, ratio, check_ori):
    ka, da, kb, db = frames
    rng = np.random.default_rng(3)
    mp = (rng.random(len(da)) < 0.8).astype(np.uint8)
    fva, fvb = _featvec(da), _featvec(db)
    n, m = orbgpu_mod.ORBmatcher(ratio, check_ori).SearchByBoW_KF_F(da, ka["angle"], mp, fva, db, kb["angle"], fvb)
    oa, _ka = _oracle_fv(oracle_mod, fva)
    ob, _kb = _oracle_fv(oracle_mod, fvb)
    on, om = oracle_mod.search_by_bow_kf_f(ratio, check_ori, da, ka["angle"], mp, oa, db, kb["angle"], ob)
    assert n == on and np.array_equal(m, om)
    assert n > 50


def test_search_by_bow_single_node_bruteforce(orbgpu_mod, oracle_mod, frames):
    # C4 semantics: one FeatureVector node with every index, all MapPoints valid, ratio 0.7, checkOri
    ka, da, kb, db = frames
    fva, fvb = {0: list(range(len(da)))}, {0: list(range(len(db)))}
    mp = np.ones(len(da), np.uint8)
    n, m = orbgpu_mod.ORBmatcher(0.7, True).SearchByBoW_KF_F(da, ka["angle"], mp, fva, db, kb["angle"], fvb)
    oa, _ka = _oracle_fv(oracle_mod, fva)
    ob, _kb = _oracle_fv(oracle_mod, fvb)
    on, om = oracle_mod.search_by_bow_kf_f(0.7, True, da, ka["angle"], mp, oa, db, kb["angle"], ob)
    assert n == on and np.array_equal(m, om)


@pytest.mark.parametrize("ratio,check_ori", [(0.75, True), (0.9, False)])
def test_search_by_bow_kf_kf(orbgpu_mod, oracle_mod, frames, ratio, check_ori):
    ka, da, kb, db = frames
    rng = np.random.default_rng(4)
    mp1 = (rng.random(len(da)) < 0.85).astype(np.uint8)
    mp2 = (rng.random(len(db)) < 0.85).astype(np.uint8)
    fva, fvb = _featvec(da), _featvec(db)
    n, m = orbgpu_mod.ORBmatcher(ratio, check_ori).SearchByBoW_KF_KF(da, ka["angle"], mp1, fva, db, kb["angle"],
                                                                      mp2, fvb)
    oa, _ka = _oracle_fv(oracle_mod, fva)
    ob, _kb = _oracle_fv(oracle_mod, fvb)
    on, om = oracle_mod.search_by_bow_kf_kf(ratio, check_ori, da, ka["angle"], mp1, oa, db, kb["angle"], mp2, ob)
    assert n == on and np.array_equal(m, om)


@pytest.mark.parametrize("ratio,check_ori", [(0.75, True), (0.7, False)])
def test_search_by_bow_batches(orbgpu_mod, oracle_mod, frames, ratio, check_ori):
    """The BoW searches over several keyframes in one call (Tracking.cc:1931-1938's relocalisation candidates against
    one Frame; LoopClosing.cc:252-265's loop candidates against one KF1): each entry equals the single call and the
    oracle.  Keyframes: both frames with different map-point masks and FeatureVector granularities, one without
    features, one without a common node."""
    ka, da, kb, db = frames
    rng = np.random.default_rng(41)
    kfs = []
    for p, (d, k, nodes) in enumerate([(da, ka, 16), (db, kb, 8), (da, ka, 24), (db, kb, 16)]):
        kfs.append(dict(desc=d, angle=k["angle"], mp=(rng.random(len(d)) < 0.6 + 0.1 * p).astype(np.uint8),
                        featvec=_featvec(d, nodes)))
    kfs.append(dict(desc=np.zeros((0, 32), np.uint8), angle=np.zeros(0, np.float32), mp=np.zeros(0, np.uint8),
                    featvec={}))
    kfs.append(dict(kfs[1], featvec={k + 5000: v for k, v in kfs[1]["featvec"].items()}))
    m = orbgpu_mod.ORBmatcher(ratio, check_ori)
    # (KF, F): every keyframe against the Frame db
    fvf = _featvec(db, 16)
    ob_f, _kf = _oracle_fv(oracle_mod, fvf)
    got = m.SearchByBoW_KF_F_batch(kfs, db, kb["angle"], fvf)
    for k, (n, mt) in zip(kfs, got):
        sn, sm = m.SearchByBoW_KF_F(k["desc"], k["angle"], k["mp"], k["featvec"], db, kb["angle"], fvf)
        oa, _ka = _oracle_fv(oracle_mod, k["featvec"])
        on, om = oracle_mod.search_by_bow_kf_f(ratio, check_ori, k["desc"], k["angle"], k["mp"], oa, db, kb["angle"],
                                               ob_f)
        assert n == sn == on and np.array_equal(mt, sm) and np.array_equal(mt, om)
    assert got[0][0] > 50 and got[4][0] == 0 and got[5][0] == 0
    # (KF, KF): KF1 = da against every keyframe
    mp1 = (rng.random(len(da)) < 0.85).astype(np.uint8)
    fv1 = _featvec(da, 16)
    o1, _k1 = _oracle_fv(oracle_mod, fv1)
    got = m.SearchByBoW_KF_KF_batch(da, ka["angle"], mp1, fv1, kfs)
    for k, (n, mt) in zip(kfs, got):
        sn, sm = m.SearchByBoW_KF_KF(da, ka["angle"], mp1, fv1, k["desc"], k["angle"], k["mp"], k["featvec"])
        ob, _kb = _oracle_fv(oracle_mod, k["featvec"])
        on, om = oracle_mod.search_by_bow_kf_kf(ratio, check_ori, da, ka["angle"], mp1, o1, k["desc"], k["angle"],
                                                k["mp"], ob)
        assert n == sn == on and np.array_equal(mt, sm) and np.array_equal(mt, om)
    assert got[1][0] > 50 and got[4][0] == 0 and got[5][0] == 0


def test_search_by_bow_batches_rerank_and_errors(orbgpu_mod, oracle_mod):
    """The re-rank path inside a batch (identical queries against trains at distances 0..39 exhaust the 8-entry lists,
    so items are re-ranked on the GPU with the taken set: only the keyframe's own items, between other keyframes'),
    an empty batch, and a malformed entry refused before anything runs."""
    import ctypes
    from orbgpu import _lib
    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    bits = np.unpackbits(base)
    trains = []
    for d in range(40):
        b = bits.copy()
        b[:d] ^= 1
        trains.append(np.packbits(b))
    t = np.array(trains, np.uint8)
    q = np.repeat(base[None], 40, 0)
    ang = np.zeros(40, np.float32)
    fv = {0: list(range(40))}
    oq, _kq = _oracle_fv(oracle_mod, fv)
    m = orbgpu_mod.ORBmatcher(0.99, False)
    mps = [np.ones(40, np.uint8), (np.arange(40) % 3 != 0).astype(np.uint8), np.ones(40, np.uint8)]
    kfs = [dict(desc=q, angle=ang, mp=mps[0], featvec=fv), dict(desc=q, angle=ang, mp=mps[1], featvec=fv),
           dict(desc=t, angle=ang, mp=mps[2], featvec=fv)]
    got = m.SearchByBoW_KF_F_batch(kfs, t, ang, fv)
    for k, (n, mt) in zip(kfs, got):
        on, om = oracle_mod.search_by_bow_kf_f(0.99, False, k["desc"], ang, k["mp"], oq, t, ang, oq)
        assert n == on and np.array_equal(mt, om)
    assert got[0][0] > 30
    got = m.SearchByBoW_KF_KF_batch(q, ang, np.ones(40, np.uint8), fv, kfs[::-1])
    for k, (n, mt) in zip(kfs[::-1], got):
        on, om = oracle_mod.search_by_bow_kf_kf(0.99, False, q, ang, np.ones(40, np.uint8), oq, k["desc"], ang,
                                                k["mp"], oq)
        assert n == on and np.array_equal(mt, om)
    L = _lib.lib()
    f, _kf = orbgpu_mod._featvec(fv)
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    assert _lib.STATUS.get(L.orb_search_by_bow_kf_f_batch(m._ctx.h, 0.7, 1, 40, p(t), p(ang), f, 0, None)) == "ORB_OK"
    ids, off, idx = np.array([0, 1], np.uint32), np.array([0, 30, 20], np.int32), np.arange(40, dtype=np.int32)
    bad = orbgpu_mod.OrbFeatVec(2, ids.ctypes.data, off.ctypes.data, idx.ctypes.data)
    out = np.full(40, -7, np.int32)
    n = ctypes.c_int(-5)
    arr = (_lib.OrbBowKf * 1)()
    arr[0] = _lib.OrbBowKf(40, p(q), p(ang), p(mps[0]), bad, p(out), ctypes.pointer(n))
    for st in (L.orb_search_by_bow_kf_f_batch(m._ctx.h, 0.7, 1, 40, p(t), p(ang), f, 1, ctypes.cast(arr, ctypes.c_void_p)),
               L.orb_search_by_bow_kf_kf_batch(m._ctx.h, 0.7, 1, 40, p(q), p(ang), p(mps[0]), f, 1,
                                               ctypes.cast(arr, ctypes.c_void_p))):
        assert _lib.STATUS.get(st) == "ORB_ERR_ARG"
    assert n.value == -5 and (out == -7).all()


def test_exhaustion_rerank_path(orbgpu_mod, oracle_mod):
    # identical queries against trains at distances 0..39: each query takes the next train, so the
    # 8-entry GPU lists run out and the remaining queries are re-ranked on the GPU.
    rng = np.random.default_rng(5)
    base = rng.integers(0, 256, 32, dtype=np.uint8)
    bits = np.unpackbits(base)
    trains = []
    for d in range(40):
        b = bits.copy()
        b[:d] ^= 1
        trains.append(np.packbits(b))
    t = np.array(trains, np.uint8)
    q = np.repeat(base[None], 40, 0)
    ang = np.zeros(40, np.float32)
    fv = {0: list(range(40))}
    n, m = orbgpu_mod.ORBmatcher(0.99, False).SearchByBoW_KF_F(q, ang, np.ones(40, np.uint8), fv, t, ang, fv)
    oa, _k = _oracle_fv(oracle_mod, fv)
    on, om = oracle_mod.search_by_bow_kf_f(0.99, False, q, ang, np.ones(40, np.uint8), oa, t, ang, oa)
    assert n == on and np.array_equal(m, om) and n > 30
    # the window matcher's vMatchedDistance stealing over the same data
    k = np.zeros(40, orbgpu_mod.KP_DTYPE)
    off = np.arange(0, 41 * 40, 40, dtype=np.int32)
    cand = np.tile(np.arange(40, dtype=np.int32), 40)
    n2, m2 = orbgpu_mod.ORBmatcher(0.99, True).SearchForInitialization(q, k, t, k, off, cand)
    on2, om2 = oracle_mod.window_match(0.99, True, True, q, k, t, k, off, cand)
    assert n2 == on2 and np.array_equal(m2, om2)


@pytest.mark.parametrize("only_stereo,check_ori,far_epipole", [(False, False, True), (False, True, False),
                                                               (True, False, True)])
def test_search_for_triangulation(orbgpu_mod, oracle_mod, frames, only_stereo, check_ori, far_epipole):
    ka, da, kb, db = frames
    rng = np.random.default_rng(6)
    mp1 = (rng.random(len(da)) < 0.3).astype(np.uint8)
    mp2 = (rng.random(len(db)) < 0.3).astype(np.uint8)
    ur1 = np.where(rng.random(len(da)) < 0.5, 10.0, -1.0).astype(np.float32)
    ur2 = np.where(rng.random(len(db)) < 0.5, 10.0, -1.0).astype(np.float32)
    F = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)   # horizontal epipolar lines: y2 = y1
    F += rng.normal(0, 1e-4, (3, 3)).astype(np.float32)
    ex, ey = (1e5, 1e5) if far_epipole else (320.0, 240.0)
    t = oracle_mod.OracleExtractor(1000).tables()
    fva, fvb = _featvec(da, 8), _featvec(db, 8)
    m = orbgpu_mod.ORBmatcher(0.6, check_ori)
    pairs = m.SearchForTriangulation(da, ka, mp1, ur1, fva, db, kb, mp2, ur2, fvb, F, ex, ey, t["scale"],
                                     t["sigma2"], only_stereo)
    oa, _ka = _oracle_fv(oracle_mod, fva)
    ob, _kb = _oracle_fv(oracle_mod, fvb)
    op = oracle_mod.search_for_triangulation(check_ori, only_stereo, da, ka, mp1, ur1, oa, db, kb, mp2, ur2, ob, F,
                                             ex, ey, t["scale"], t["sigma2"])
    assert np.array_equal(pairs, op)
    assert len(op) > 0


@pytest.mark.parametrize("shape", ["one_node", "disjoint", "trains_all_mapped", "empty_fv1", "repeated_ids",
                                   "200_nodes", "300_nodes"])
def test_search_for_triangulation_node_shapes(orbgpu_mod, oracle_mod, frames, shape):
    """The staging shapes of orb_search_for_triangulation (one item record per query, the candidates' train records
    in node order, queries of a node without candidates not staged): one node holding every feature
    (candidate ranges far longer than a wave), FeatureVectors without a common node, every train carrying a map
    point, an empty FeatureVector, a train index listed in two nodes, and 200 / 300 common nodes.  Pair for pair
    against the oracle."""
    ka, da, kb, db = frames
    rng = np.random.default_rng(21)
    mp1 = (rng.random(len(da)) < 0.3).astype(np.uint8)
    mp2 = (rng.random(len(db)) < 0.3).astype(np.uint8)
    ur1 = np.where(rng.random(len(da)) < 0.5, 10.0, -1.0).astype(np.float32)
    ur2 = np.where(rng.random(len(db)) < 0.5, 10.0, -1.0).astype(np.float32)
    F = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32) + rng.normal(0, 1e-4, (3, 3)).astype(np.float32)
    fva, fvb = _featvec(da, 8), _featvec(db, 8)
    if shape == "one_node":
        fva, fvb = {3: list(range(len(da)))}, {3: list(range(len(db)))}
    elif shape == "disjoint":
        fvb = {k + 100: v for k, v in fvb.items()}
    elif shape == "trains_all_mapped":
        mp2[:] = 1
    elif shape == "empty_fv1":
        fva = {}
    elif shape in ("200_nodes", "300_nodes"):
        k = int(shape.split("_")[0])
        fva, fvb = {}, {}
        for i in range(len(da)):
            fva.setdefault(i % k, []).append(i)
        for i in range(len(db)):
            fvb.setdefault(i % k, []).append(i)
    else:   # the reference's FeatureVector lists each feature once; a repeated index is staged once per listing
        k0, k1 = sorted(fvb)[:2]
        fvb[k1] = fvb[k1] + fvb[k0][:5]
    t = oracle_mod.OracleExtractor(1000).tables()
    m = orbgpu_mod.ORBmatcher(0.6, True)
    pairs = m.SearchForTriangulation(da, ka, mp1, ur1, fva, db, kb, mp2, ur2, fvb, F, 320.0, 240.0, t["scale"],
                                     t["sigma2"], False)
    oa, _keep_a = _oracle_fv(oracle_mod, fva)
    ob, _keep_b = _oracle_fv(oracle_mod, fvb)
    op = oracle_mod.search_for_triangulation(True, False, da, ka, mp1, ur1, oa, db, kb, mp2, ur2, ob, F, 320.0, 240.0,
                                             t["scale"], t["sigma2"])
    assert np.array_equal(pairs, op)
    if shape in ("one_node", "200_nodes", "300_nodes"):
        assert len(op) > 0
    if shape in ("disjoint", "trains_all_mapped", "empty_fv1"):
        assert len(op) == 0


def test_search_for_triangulation_rejects_malformed_featvec(orbgpu_mod, oracle_mod, frames):
    """A FeatureVector CSR whose offsets decrease or do not start at 0, whose feature indices leave [0, n), or whose
    node ids do not ascend strictly is refused (ORB_ERR_ARG) before anything is staged or walked, by
    SearchForTriangulation and both SearchByBoW forms: the calls size their pinned records from offsets[nnodes],
    index descriptors / keypoints / map-point flags with the indices, and merge the two node lists as std::map
    keys (matcher.hip featvec_ok)."""
    import ctypes
    from orbgpu import _lib
    ka, da, kb, db = frames
    n1 = len(da)
    t = oracle_mod.OracleExtractor(1000).tables()
    m = orbgpu_mod.ORBmatcher(0.6, True)
    fva, fvb = _featvec(da, 8), _featvec(db, 8)
    fb, _keep_b = orbgpu_mod._featvec(fvb)
    q = n1 // 3
    idx_ok = np.arange(n1, dtype=np.int32)
    idx_hi = idx_ok.copy()
    idx_hi[5] = n1          # one past the last feature
    idx_neg = idx_ok.copy()
    idx_neg[7] = -1
    cases = {   # (node ids, offsets, indices)
        "offsets_decrease": ([0, 1, 2], [0, 5, 3, n1], idx_ok),
        "offsets_not_zero": ([0, 1, 2], [2, 5, 9, n1], idx_ok),
        "index_past_n": ([0, 1, 2], [0, q, 2 * q, n1], idx_hi),
        "index_negative": ([0, 1, 2], [0, q, 2 * q, n1], idx_neg),
        "ids_repeated": ([0, 2, 2], [0, q, 2 * q, n1], idx_ok),
        "ids_descending": ([5, 3, 1], [0, q, 2 * q, n1], idx_ok),
    }
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    L = _lib.lib()
    for name, (ids_l, off_l, idx) in cases.items():
        off = np.asarray(off_l, np.int32)
        ids = np.asarray(ids_l, np.uint32)
        fa = orbgpu_mod.OrbFeatVec(len(ids), ids.ctypes.data, off.ctypes.data, idx.ctypes.data)
        a = [np.ascontiguousarray(x) for x in (da, np.asarray(ka, orbgpu_mod.KP_DTYPE), np.zeros(n1, np.uint8),
                                                np.full(n1, -1, np.float32), db,
                                                np.asarray(kb, orbgpu_mod.KP_DTYPE), np.zeros(len(db), np.uint8),
                                                np.full(len(db), -1, np.float32), np.eye(3, dtype=np.float32).reshape(9),
                                                np.asarray(t["scale"], np.float32), np.asarray(t["sigma2"], np.float32))]
        pairs = np.zeros((n1 + 1, 2), np.int32)
        n = ctypes.c_int()
        st = L.orb_search_for_triangulation(m._ctx.h, 1, 0, n1, p(a[0]), p(a[1]), p(a[2]), p(a[3]), fa,
                                            len(db), p(a[4]), p(a[5]), p(a[6]), p(a[7]), fb, p(a[8]), 320.0,
                                            240.0, p(a[9]), p(a[10]), len(a[9]), p(pairs), len(pairs), ctypes.byref(n))
        assert _lib.STATUS.get(st) == "ORB_ERR_ARG", (name, st)
        ang1, ang2 = np.zeros(n1, np.float32), np.zeros(len(db), np.float32)
        mp1, mp2 = np.ones(n1, np.uint8), np.ones(len(db), np.uint8)
        match = np.full(max(n1, len(db)), -7, np.int32)
        st = L.orb_search_by_bow_kf_f(m._ctx.h, 0.7, 1, n1, p(a[0]), p(ang1), p(mp1), fa, len(db), p(a[4]), p(ang2),
                                      fb, p(match), ctypes.byref(n))
        assert _lib.STATUS.get(st) == "ORB_ERR_ARG", (name, "kf_f", st)
        st = L.orb_search_by_bow_kf_kf(m._ctx.h, 0.75, 1, n1, p(a[0]), p(ang1), p(mp1), fa, len(db), p(a[4]),
                                       p(ang2), p(mp2), fb, p(match), ctypes.byref(n))
        assert _lib.STATUS.get(st) == "ORB_ERR_ARG", (name, "kf_kf", st)
        assert (match == -7).all(), name   # nothing written
    # the context stays usable
    ok = m.SearchForTriangulation(da, ka, np.zeros(n1, np.uint8), np.full(n1, -1, np.float32), fva, db, kb,
                                  np.zeros(len(db), np.uint8), np.full(len(db), -1, np.float32), fvb,
                                  np.eye(3, dtype=np.float32), 320.0, 240.0, t["scale"], t["sigma2"])
    assert ok.ndim == 2


def test_search_for_triangulation_capacity(orbgpu_mod, oracle_mod, frames):
    """pairs_out smaller than the pair count: ORB_ERR_CAPACITY with *npairs = the count and the first cap pairs
    written (include/orbgpu.h)."""
    import ctypes
    from orbgpu import _lib
    ka, da, kb, db = frames
    t = oracle_mod.OracleExtractor(1000).tables()
    F = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)
    fva, fvb = _featvec(da, 8), _featvec(db, 8)
    m = orbgpu_mod.ORBmatcher(0.6, False)
    mp1, mp2 = np.zeros(len(da), np.uint8), np.zeros(len(db), np.uint8)
    ur1, ur2 = np.full(len(da), -1, np.float32), np.full(len(db), -1, np.float32)
    full = m.SearchForTriangulation(da, ka, mp1, ur1, fva, db, kb, mp2, ur2, fvb, F, 1e5, 1e5, t["scale"], t["sigma2"])
    assert len(full) > 3
    fa, _keep_a = orbgpu_mod._featvec(fva)
    fb, _keep_b = orbgpu_mod._featvec(fvb)
    a = [np.ascontiguousarray(x) for x in (da, np.asarray(ka, orbgpu_mod.KP_DTYPE), mp1, ur1, db,
                                            np.asarray(kb, orbgpu_mod.KP_DTYPE), mp2, ur2, F.reshape(9),
                                            np.asarray(t["scale"], np.float32), np.asarray(t["sigma2"], np.float32))]
    cap = 3
    pairs = np.full((cap, 2), -9, np.int32)
    n = ctypes.c_int(-1)
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    st = _lib.lib().orb_search_for_triangulation(m._ctx.h, 0, 0, len(da), p(a[0]), p(a[1]), p(a[2]), p(a[3]), fa,
                                                 len(db), p(a[4]), p(a[5]), p(a[6]), p(a[7]), fb, p(a[8]), 1e5, 1e5,
                                                 p(a[9]), p(a[10]), len(a[9]), p(pairs), cap, ctypes.byref(n))
    assert _lib.STATUS.get(st) == "ORB_ERR_CAPACITY", st
    assert n.value == len(full)
    assert np.array_equal(pairs, full[:cap])


@pytest.mark.parametrize("case", ["F_nan", "F_inf", "F_zero", "epipole_nan"])
def test_search_for_triangulation_nonfinite(orbgpu_mod, oracle_mod, frames, case):
    """Degenerate geometry keeps the reference's IEEE semantics (ORBmatcher.cc:140-157, :725-733): a NaN or
    infinite F12 entry, an all-zero F12 (den == 0) and a NaN epipole.  A NaN epipolar distance never passes
    `dsqr < 3.84 sigma2`, a NaN epipole distance never trips the `< 100 scale` rejection; the GPU kernel is built
    without -fno-honor-nans and must agree with the oracle pair for pair."""
    ka, da, kb, db = frames
    rng = np.random.default_rng(16)
    mp1 = (rng.random(len(da)) < 0.3).astype(np.uint8)
    mp2 = (rng.random(len(db)) < 0.3).astype(np.uint8)
    ur1 = np.where(rng.random(len(da)) < 0.5, 10.0, -1.0).astype(np.float32)
    ur2 = np.where(rng.random(len(db)) < 0.5, 10.0, -1.0).astype(np.float32)
    F = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32) + rng.normal(0, 1e-4, (3, 3)).astype(np.float32)
    ex, ey = 320.0, 240.0
    if case == "F_nan":
        F[2, 2] = np.nan
    elif case == "F_inf":
        F[0, 0] = np.inf   # a = x1 * inf: inf, or NaN where x1 == 0; den = inf
    elif case == "F_zero":
        F[:] = 0
    else:
        ex = float("nan")
    t = oracle_mod.OracleExtractor(1000).tables()
    fva, fvb = _featvec(da, 8), _featvec(db, 8)
    m = orbgpu_mod.ORBmatcher(0.6, True)
    pairs = m.SearchForTriangulation(da, ka, mp1, ur1, fva, db, kb, mp2, ur2, fvb, F, ex, ey, t["scale"],
                                     t["sigma2"], False)
    oa, _keep_a = _oracle_fv(oracle_mod, fva)   # (the second element keeps the CSR arrays alive)
    ob, _keep_b = _oracle_fv(oracle_mod, fvb)
    op = oracle_mod.search_for_triangulation(True, False, da, ka, mp1, ur1, oa, db, kb, mp2, ur2, ob, F, ex, ey,
                                             t["scale"], t["sigma2"])
    assert np.array_equal(pairs, op)
    if case == "epipole_nan":
        assert len(op) > 0


def _tri_batch_pairs(frames, oracle_mod, seed):
    """Six KF2s for one KF1 (LocalMapping's neighbour loop): both frames as KF2, different F12 (epipolar lines
    near y2 = y1, rotated), epipoles near, far and NaN, different map-point and stereo masks, and KF2 FeatureVectors
    of different node granularity."""
    ka, da, kb, db = frames
    rng = np.random.default_rng(seed)
    t = oracle_mod.OracleExtractor(1000).tables()
    base = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32)
    out = []
    for p in range(6):
        k2, d2 = (kb, db) if p % 3 != 2 else (ka, da)
        F = base + rng.normal(0, 1e-4 * (1 + p), (3, 3)).astype(np.float32)
        ex, ey = [(320.0, 240.0), (1e5, 1e5), (float("nan"), 100.0), (50.0, 400.0), (320.0, 240.0), (1e5, -1e5)][p]
        out.append(dict(desc2=d2, kps2=k2, has_mp2=(rng.random(len(d2)) < 0.2 + 0.1 * p).astype(np.uint8),
                        uright2=np.where(rng.random(len(d2)) < 0.5, 10.0, -1.0).astype(np.float32),
                        featvec2=_featvec(d2, [8, 6, 10, 8, 4, 8][p]), F12=F, ex=ex, ey=ey,
                        scale_factors2=t["scale"], level_sigma2_2=t["sigma2"]))
    return out


@pytest.mark.parametrize("check_ori,only_stereo", [(False, False), (True, False), (False, True)])
def test_search_for_triangulation_batch(orbgpu_mod, oracle_mod, frames, check_ori, only_stereo):
    """orb_search_for_triangulation_batch: KF1 against six KF2s in one call gives, pair for pair, the single call's
    result and the oracle's (ORBmatcher.cc:657-823 per pair)."""
    ka, da, kb, db = frames
    rng = np.random.default_rng(31)
    mp1 = (rng.random(len(da)) < 0.3).astype(np.uint8)
    ur1 = np.where(rng.random(len(da)) < 0.5, 10.0, -1.0).astype(np.float32)
    fva = _featvec(da, 8)
    others = _tri_batch_pairs(frames, oracle_mod, 32)
    m = orbgpu_mod.ORBmatcher(0.6, check_ori)
    got = m.SearchForTriangulationBatch(da, ka, mp1, ur1, fva, others, only_stereo)
    assert len(got) == len(others)
    oa, _keep_a = _oracle_fv(oracle_mod, fva)
    total = 0
    for o, g in zip(others, got):
        single = m.SearchForTriangulation(da, ka, mp1, ur1, fva, o["desc2"], o["kps2"], o["has_mp2"], o["uright2"],
                                          o["featvec2"], o["F12"], o["ex"], o["ey"], o["scale_factors2"],
                                          o["level_sigma2_2"], only_stereo)
        ob, _keep_b = _oracle_fv(oracle_mod, o["featvec2"])
        op = oracle_mod.search_for_triangulation(check_ori, only_stereo, da, ka, mp1, ur1, oa, o["desc2"], o["kps2"],
                                                 o["has_mp2"], o["uright2"], ob, o["F12"], o["ex"], o["ey"],
                                                 o["scale_factors2"], o["level_sigma2_2"])
        assert np.array_equal(g, single) and np.array_equal(g, op)
        total += len(op)
    assert total > 0


def test_search_for_triangulation_batch_local_mapping_order(orbgpu_mod, oracle_mod, frames):
    """The documented use in LocalMapping::CreateNewMapPoints (LocalMapping.cc:247-278, 449): the reference calls
    SearchForTriangulation per neighbour and gives KF1 features new map points between the calls.  With
    check_ori = 0, the batch computed once plus dropping, pair by pair, the matches whose idx1 received a map point
    from an earlier pair equals the sequential loop of single calls with the map-point mask updated as it goes
    (here every other accepted match "triangulates")."""
    ka, da, kb, db = frames
    rng = np.random.default_rng(33)
    mp1 = (rng.random(len(da)) < 0.2).astype(np.uint8)
    ur1 = np.full(len(da), -1.0, np.float32)
    fva = _featvec(da, 8)
    others = _tri_batch_pairs(frames, oracle_mod, 34)
    m = orbgpu_mod.ORBmatcher(0.6, False)
    # the reference order: single calls, the KF1 mask growing between them
    seq, mask = [], mp1.copy()
    for o in others:
        r = m.SearchForTriangulation(da, ka, mask, ur1, fva, o["desc2"], o["kps2"], o["has_mp2"], o["uright2"],
                                     o["featvec2"], o["F12"], o["ex"], o["ey"], o["scale_factors2"],
                                     o["level_sigma2_2"])
        seq.append(r)
        mask[r[::2, 0]] = 1
    # the batch, then the caller's filter
    got = m.SearchForTriangulationBatch(da, ka, mp1, ur1, fva, others)
    mask = mp1.copy()
    n_dropped = 0
    for r, g in zip(seq, got):
        keep = mask[g[:, 0]] == 0
        n_dropped += int((~keep).sum())
        assert np.array_equal(g[keep], r)
        mask[r[::2, 0]] = 1
    assert sum(len(r) for r in seq) > 0 and n_dropped > 0


def test_search_for_triangulation_batch_edges(orbgpu_mod, oracle_mod, frames):
    """An empty pair list, a KF2 without features or without a common node, a malformed KF2 FeatureVector (the whole
    call refused with ORB_ERR_ARG before anything runs or is written), and one pair's list overflowing (ORB_ERR_CAPACITY,
    every pair's count and lists still filled)."""
    import ctypes
    from orbgpu import _lib
    ka, da, kb, db = frames
    L = _lib.lib()
    m = orbgpu_mod.ORBmatcher(0.6, False)
    n1 = len(da)
    fva = _featvec(da, 8)
    fa, _keep_a = orbgpu_mod._featvec(fva)
    a = [np.ascontiguousarray(x) for x in (da, np.asarray(ka, orbgpu_mod.KP_DTYPE), np.zeros(n1, np.uint8),
                                            np.full(n1, -1, np.float32))]
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    st = L.orb_search_for_triangulation_batch(m._ctx.h, 0, 0, n1, p(a[0]), p(a[1]), p(a[2]), p(a[3]), fa, 0, None)
    assert _lib.STATUS.get(st) == "ORB_OK"
    others = _tri_batch_pairs(frames, oracle_mod, 35)[:3]
    others[0] = dict(others[0], desc2=np.zeros((0, 32), np.uint8), kps2=np.zeros(0, orbgpu_mod.KP_DTYPE),
                     has_mp2=np.zeros(0, np.uint8), uright2=np.zeros(0, np.float32), featvec2={})
    others[1] = dict(others[1], featvec2={k + 1000: v for k, v in others[1]["featvec2"].items()})
    got = m.SearchForTriangulationBatch(da, ka, a[2], a[3], fva, others)
    assert len(got[0]) == 0 and len(got[1]) == 0 and len(got[2]) > 3
    single = m.SearchForTriangulation(da, ka, a[2], a[3], fva, others[2]["desc2"], others[2]["kps2"],
                                      others[2]["has_mp2"], others[2]["uright2"], others[2]["featvec2"],
                                      others[2]["F12"], others[2]["ex"], others[2]["ey"],
                                      others[2]["scale_factors2"], others[2]["level_sigma2_2"])
    assert np.array_equal(got[2], single)
    # one malformed KF2 CSR: refused, nothing written
    o = others[2]
    b = [np.ascontiguousarray(x) for x in (o["desc2"], np.asarray(o["kps2"], orbgpu_mod.KP_DTYPE), o["has_mp2"],
                                            o["uright2"], np.asarray(o["F12"], np.float32).reshape(9),
                                            np.asarray(o["scale_factors2"], np.float32),
                                            np.asarray(o["level_sigma2_2"], np.float32))]
    fb, _keep_b = orbgpu_mod._featvec(o["featvec2"])
    ids, off, idx8 = np.array([0, 1], np.uint32), np.array([0, 5, 3], np.int32), np.arange(8, dtype=np.int32)
    bad = orbgpu_mod.OrbFeatVec(2, ids.ctypes.data, off.ctypes.data, idx8.ctypes.data)
    outs = [np.full((n1 + 1, 2), -7, np.int32) for _ in range(2)]
    cnt = [ctypes.c_int(-5) for _ in range(2)]
    arr = (_lib.OrbTriPair * 2)()
    for i, fv in enumerate((fb, bad)):
        arr[i] = _lib.OrbTriPair(len(b[0]), p(b[0]), p(b[1]), p(b[2]), p(b[3]), fv, p(b[4]), o["ex"], o["ey"], p(b[5]),
                                 p(b[6]), len(b[5]), p(outs[i]), n1 + 1, ctypes.pointer(cnt[i]))
    st = L.orb_search_for_triangulation_batch(m._ctx.h, 0, 0, n1, p(a[0]), p(a[1]), p(a[2]), p(a[3]), fa, 2,
                                              ctypes.cast(arr, ctypes.c_void_p))
    assert _lib.STATUS.get(st) == "ORB_ERR_ARG"
    assert all(c.value == -5 for c in cnt) and all((x == -7).all() for x in outs)
    # the second pair's list too small: every count reported, the first pair complete, the second cut at cap
    arr[1] = _lib.OrbTriPair(len(b[0]), p(b[0]), p(b[1]), p(b[2]), p(b[3]), fb, p(b[4]), o["ex"], o["ey"], p(b[5]),
                             p(b[6]), len(b[5]), p(outs[1]), 2, ctypes.pointer(cnt[1]))
    st = L.orb_search_for_triangulation_batch(m._ctx.h, 0, 0, n1, p(a[0]), p(a[1]), p(a[2]), p(a[3]), fa, 2,
                                              ctypes.cast(arr, ctypes.c_void_p))
    assert _lib.STATUS.get(st) == "ORB_ERR_CAPACITY"
    assert cnt[0].value == len(single) and cnt[1].value == len(single)
    assert np.array_equal(outs[0][:len(single)], single) and np.array_equal(outs[1][:2], single[:2])


@pytest.mark.parametrize("level0_only,window", [(True, 100), (False, 15), (True, 40)])
def test_window_match(orbgpu_mod, oracle_mod, frames, level0_only, window):
    ka, da, kb, db = frames
    offs, idxs = [0], []
    for k in ka:
        c = orbgpu_mod.features_in_area(kb, 0, 640, 0, 480, float(k["x"]), float(k["y"]), window,
                                        int(k["octave"]) if level0_only else -1,
                                        int(k["octave"]) if level0_only else -1)
        idxs.extend(c.tolist())
        offs.append(len(idxs))
    off = np.array(offs, np.int32)
    cand = np.array(idxs, np.int32)
    for ratio in (0.9, 0.99):
        m = orbgpu_mod.ORBmatcher(ratio, True)
        fn = m.SearchForInitialization if level0_only else m.BirdviewMatch
        n, mm = fn(da, ka, db, kb, off, cand)
        on, om = oracle_mod.window_match(ratio, True, level0_only, da, ka, db, kb, off, cand)
        assert n == on and np.array_equal(mm, om)
        assert n > 20


@pytest.mark.parametrize("level0_only,window,centred", [(True, 100, True), (True, 15, False), (False, 15, False),
                                                         (False, 40, True)])
def test_window_match_grid(orbgpu_mod, oracle_mod, frames, level0_only, window, centred):
    """orb_window_match_grid (GetFeaturesInArea on the device over F2's grid) against the oracle with
    candidates from the oracle's own GetFeaturesInArea restatement, around moved centres (vbPrevMatched)
    or each query's own keypoint; the frame's grid bounds are not the image's (mnMinX > 0)."""
    ka, da, kb, db = frames
    bounds = (3.5, 636.0, 1.0, 470.5)
    rng = np.random.default_rng(7)
    cen = np.stack([ka["x"], ka["y"]], 1).astype(np.float32)
    if centred:
        cen = (cen + rng.uniform(-6, 6, cen.shape)).astype(np.float32)
    offs, idxs = [0], []
    for i, k in enumerate(ka):
        if not (level0_only and k["octave"] > 0):
            lv = int(k["octave"])
            c = oracle_mod.features_in_area(kb, *bounds, float(cen[i, 0]), float(cen[i, 1]), float(window), lv, lv)
            idxs.extend(c.tolist())
        offs.append(len(idxs))
    off = np.array(offs, np.int32)
    cand = np.array(idxs or [0], np.int32)
    grid = orbgpu_mod.frame_grid(kb, *bounds)
    for ratio in (0.9, 0.99):
        m = orbgpu_mod.ORBmatcher(ratio, True)
        n, mm = m.window_match_grid(level0_only, da, ka, db, kb, grid, window, cen if centred else None,
                                    (bounds[0], bounds[2]))
        on, om = oracle_mod.window_match(ratio, True, level0_only, da, ka, db, kb, off, cand)
        assert n == on and np.array_equal(mm, om)
        assert n > 20


def test_frame_grid_matches_oracle_lookup(orbgpu_mod, oracle_mod, frames):
    """frame_grid's CSR is the reference grid: a lookup over it equals oracle_features_in_area."""
    ka, da, kb, db = frames
    inv_w, inv_h, off, idx = orbgpu_mod.frame_grid(kb, 0, 640, 0, 480)
    assert off[-1] == len(kb) and sorted(idx.tolist()) == list(range(len(kb)))
    for k in kb[::37]:
        px = int(np.floor(float(np.float32(k["x"]) * np.float32(inv_w)) + 0.5))
        py = int(np.floor(float(np.float32(k["y"]) * np.float32(inv_h)) + 0.5))
        cell = idx[off[px * 48 + py]:off[px * 48 + py + 1]]
        assert np.all(np.diff(cell) > 0)


@pytest.mark.parametrize("nt", [0, 1, 40, 700])
def test_top2_device_small_train_sets(orbgpu_mod, nt):
    """Edge sizes of the batched kernel: one train, a single slice, and a query count that is not a
    multiple of 64 (partial last wavefront)."""
    from orbgpu import _lib
    rng = np.random.default_rng(nt)
    nq = 77
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    b = orbgpu_mod.BatchExtractor(1000, 640, 480, 1)
    L = _lib.lib()
    dq, dt = b._alloc(q.nbytes), b._alloc(t.nbytes)
    out = [b._alloc(nq * 4) for _ in range(3)]
    L.orb_memcpy_h2d(b.h, dq, q.ctypes.data, q.nbytes)
    L.orb_memcpy_h2d(b.h, dt, t.ctypes.data, t.nbytes)
    b.hamming_top2(dq, nq, dt, nt, *out)
    b.sync()
    res = [np.zeros(nq, np.int32) for _ in range(3)]
    for r, d in zip(res, out):
        L.orb_memcpy_d2h(b.h, r.ctypes.data, d, nq * 4)
    if nt == 0:   # an empty train set (a previous frame without keypoints): the no-match sentinels
        assert (res[0] == 257).all() and (res[1] == -1).all() and (res[2] == 257).all()
    else:
        D = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(2)
        srt = np.sort(D, 1)
        assert np.array_equal(res[0], srt[:, 0]) and np.array_equal(res[1], D.argmin(1))
        assert np.array_equal(res[2], srt[:, 1] if nt > 1 else np.full(nq, 257))
    for p in [dq, dt] + out:
        L.orb_device_free(b.h, p)


def test_top2_device_extreme_distances_and_ties(orbgpu_mod):
    """Distances 0 and 256 (the ends of the MFMA kernel's tile-local key range) and long runs of equal
    distances across 32-train tiles: the first index wins, the second is the second-smallest distance."""
    from orbgpu import _lib
    rng = np.random.default_rng(7)
    nq = 70
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    q[1] = 0
    q[2] = 255
    t = np.concatenate([np.repeat(q[:1], 50, 0), np.repeat(~q[:1], 47, 0), np.zeros((5, 32), np.uint8),
                        np.full((3, 32), 255, np.uint8)])
    nt = len(t)
    b = orbgpu_mod.BatchExtractor(1000, 640, 480, 1)
    L = _lib.lib()
    dq, dt = b._alloc(q.nbytes), b._alloc(t.nbytes)
    out = [b._alloc(nq * 4) for _ in range(3)]
    L.orb_memcpy_h2d(b.h, dq, q.ctypes.data, q.nbytes)
    L.orb_memcpy_h2d(b.h, dt, t.ctypes.data, t.nbytes)
    b.hamming_top2(dq, nq, dt, nt, *out)
    b.sync()
    res = [np.zeros(nq, np.int32) for _ in range(3)]
    for r, d in zip(res, out):
        L.orb_memcpy_d2h(b.h, r.ctypes.data, d, nq * 4)
    D = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(2)
    srt = np.sort(D, 1)
    assert np.array_equal(res[0], srt[:, 0]) and np.array_equal(res[1], D.argmin(1))
    assert np.array_equal(res[2], srt[:, 1]), _diff(res[2], srt[:, 1], res[0])
    assert (res[0][0], res[1][0], res[2][0]) == (0, 0, 0)
    assert res[0][1] == 0 and res[1][1] == 97 and res[0][2] == 0 and res[1][2] == 102
    for p in [dq, dt] + out:
        L.orb_device_free(b.h, p)
    b.close()


def test_top2_frames_batch_vs_numpy(orbgpu_mod):
    """orb_hamming_top2_frames_device: many frame pairs of an extraction batch in one launch, counts
    read on the device — vs numpy on the downloaded descriptors."""
    from orbgpu import _lib
    from orbgpu.synth import synth_batch
    B = 6
    bx = orbgpu_mod.BatchExtractor(1000, 640, 480, B)
    bx.upload(synth_batch(640, 480, B, first=30))
    bx.launch()
    bx.sync()
    cap = bx.kp_cap
    qf, tf = [0, 1, 2, 3, 4, 5, 2], [1, 2, 3, 4, 5, 0, 2]
    L = _lib.lib()
    out = [bx._alloc(len(qf) * cap * 4) for _ in range(3)]
    bx.hamming_top2_frames(qf, tf, *out)
    bx.sync()
    res = [np.zeros(len(qf) * cap, np.int32) for _ in range(3)]
    for r, d in zip(res, out):
        L.orb_memcpy_d2h(bx.h, r.ctypes.data, d, r.nbytes)
    for p, (a, b) in enumerate(zip(qf, tf)):
        _, da = bx.results(a)
        _, db = bx.results(b)
        D = np.unpackbits(da[:, None, :] ^ db[None, :, :], axis=2).sum(2)
        srt = np.sort(D, 1)
        n = len(da)
        sl = slice(p * cap, p * cap + n)
        assert np.array_equal(res[0][sl], srt[:, 0])
        assert np.array_equal(res[1][sl], D.argmin(1))
        assert np.array_equal(res[2][sl], srt[:, 1])
    for d in out:
        L.orb_device_free(bx.h, d)
    bx.close()


def test_top2_frames_pair_list_changes(orbgpu_mod):
    """The pair list stays on the device between calls and is re-sent only when it changes
    (orb_hamming_top2_frames_device): alternate lists of different lengths on one context, each call checked
    against numpy, including a repeat of the first list after the others."""
    from orbgpu import _lib
    from orbgpu.synth import synth_batch
    B = 5
    bx = orbgpu_mod.BatchExtractor(800, 640, 480, B)
    bx.upload(synth_batch(640, 480, B, first=70))
    bx.launch()
    bx.sync()
    cap = bx.kp_cap
    L = _lib.lib()
    lists = [([0, 1, 2], [1, 2, 3]), ([3, 4], [4, 0]), ([0, 1, 2], [1, 2, 3]), ([4, 2, 1, 0, 3], [0, 0, 4, 2, 3]),
             ([4, 2, 1, 0, 3], [0, 0, 4, 2, 3]), ([1], [1])]
    out = [bx._alloc(5 * cap * 4) for _ in range(3)]
    for qf, tf in lists:
        bx.hamming_top2_frames(qf, tf, *out)
        bx.sync()
        res = [np.zeros(len(qf) * cap, np.int32) for _ in range(3)]
        for r, d in zip(res, out):
            L.orb_memcpy_d2h(bx.h, r.ctypes.data, d, r.nbytes)
        for p, (a, b) in enumerate(zip(qf, tf)):
            best, idx, second = _top2_numpy(bx.results(a)[1], bx.results(b)[1])
            sl = slice(p * cap, p * cap + len(best))
            assert np.array_equal(res[0][sl], best) and np.array_equal(res[1][sl], idx), (qf, tf, p)
            assert np.array_equal(res[2][sl], second), (qf, tf, p)
    for d in out:
        L.orb_device_free(bx.h, d)
    bx.close()


def _top2_numpy(dq, dt):
    """(best, first argmin, second) of the 256-bit Hamming distances, DescriptorDistance
    (ORBmatcher.cc:1647-1663) as a popcount of the XOR of four u64 words."""
    a = np.ascontiguousarray(dq).view(np.uint64)
    b = np.ascontiguousarray(dt).view(np.uint64)
    D = np.zeros((len(a), len(b)), np.int32)
    for w in range(4):
        D += np.bitwise_count(a[:, w, None] ^ b[None, :, w]).astype(np.int32)
    srt = np.partition(D, 1, axis=1) if D.shape[1] > 1 else D
    return D.min(1), D.argmin(1), srt[:, 1] if D.shape[1] > 1 else np.full(len(a), 257)


def test_top2_frames_bench_shape(orbgpu_mod):
    """The Hamming half of the headline metric exactly as bench.py times it: B = 256 C3 frames
    (1280x720, 2000 features, bench_frames), the 255 consecutive pairs f -> f+1 in ONE
    orb_hamming_top2_frames_device launch.  At this shape top2_batch_slices gives one train slice, so
    k_top2_mfma writes best / index / second directly (hamming_kernels.hip, gridDim.y == 1 branch; no
    k_top2b_merge).  Pairs 0, 127 and 254 against numpy on the downloaded descriptors: best distance,
    first index on ties (SearchByBoW's strict '<', ORBmatcher.cc:216-225) and the second distance."""
    from orbgpu import _lib
    from orbgpu.synth import bench_frames
    B = 256
    bx = orbgpu_mod.BatchExtractor(2000, 1280, 720, B)
    bx.upload(bench_frames(1280, 720, B))
    bx.launch()
    bx.sync()
    cap = bx.kp_cap
    counts = bx.counts()
    assert counts.min() > 1900
    L = _lib.lib()
    assert L.orb_hamming_top2_slices(B - 1, cap, cap) == 1   # the direct-write branch
    qf, tf = list(range(B - 1)), list(range(1, B))
    out = [bx._alloc((B - 1) * cap * 4) for _ in range(3)]
    bx.hamming_top2_frames(qf, tf, *out)
    bx.sync()
    for p in (0, 127, 254):
        res = [np.zeros(cap, np.int32) for _ in range(3)]
        for r, d in zip(res, out):
            L.orb_memcpy_d2h(bx.h, r.ctypes.data, d + p * cap * 4, r.nbytes)
        _, dq = bx.results(p)
        _, dt = bx.results(p + 1)
        best, idx, second = _top2_numpy(dq, dt)
        n = len(dq)
        assert np.array_equal(res[0][:n], best), p
        assert np.array_equal(res[1][:n], idx), p
        assert np.array_equal(res[2][:n], second), (p, _diff(res[2][:n], second, best))
    # every pair: the whole launch's outputs against exact distances from a float32 GEMM of the unpacked bits
    # (popcount(q ^ t) = |q| + |t| - 2 q.t, exact integers in float32), and a second launch bit-identical
    allr = [np.zeros((B - 1) * cap, np.int32) for _ in range(3)]
    for r, d in zip(allr, out):
        L.orb_memcpy_d2h(bx.h, r.ctypes.data, d, r.nbytes)
    bits = [np.unpackbits(bx.results(f)[1], axis=1).astype(np.float32) for f in range(B)]
    for p in range(B - 1):
        Q, T = bits[p], bits[p + 1]
        D = (Q.sum(1)[:, None] + T.sum(1)[None, :] - 2 * (Q @ T.T)).astype(np.int32)
        n = len(Q)
        sl = slice(p * cap, p * cap + n)
        assert np.array_equal(allr[0][sl], D.min(1)), p
        assert np.array_equal(allr[1][sl], D.argmin(1)), p
        sec = np.partition(D, 1, axis=1)[:, 1]
        assert np.array_equal(allr[2][sl], sec), (p, _diff(allr[2][sl], sec, D.min(1)))
    bx.hamming_top2_frames(qf, tf, *out)
    bx.sync()
    for r, d in zip(allr, out):
        again = np.zeros_like(r)
        L.orb_memcpy_d2h(bx.h, again.ctypes.data, d, again.nbytes)
        assert np.array_equal(again, r)
    for d in out:
        L.orb_device_free(bx.h, d)
    bx.close()


def test_distinctive_descriptors_vs_oracle(orbgpu_mod, oracle_mod):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307), batched over map points with
    1..300 observations (noisy copies of a prototype: realistic ties in the medians), plus empty."""
    rng = np.random.default_rng(11)
    sets = [np.zeros((0, 32), np.uint8)]
    for n in [1, 2, 3, 4, 7, 31, 64, 65, 130, 300] + list(rng.integers(1, 40, 40)):
        proto = rng.integers(0, 256, 32, dtype=np.uint8)
        flips = rng.random((n, 256)) < rng.uniform(0.02, 0.3)
        sets.append(np.packbits(np.unpackbits(proto)[None, :] ^ flips.astype(np.uint8), axis=1))
    m = orbgpu_mod.ORBmatcher()
    got = m.ComputeDistinctiveDescriptors(sets)
    exp = [oracle_mod.distinctive_descriptor(s) for s in sets]
    assert got.tolist() == exp

"""The vocabulary-gated matchers fed by the GPU vocabulary transform, as the reference chains them:
Frame::ComputeBoW / KeyFrame::ComputeBoW (Frame.cc:562-569, KeyFrame.cc:74-83: transform with levelsup 4,
TemplatedVocabulary.h:1139-1210) produce the FeatureVectors that SearchByBoW (ORBmatcher.cc:159-288,
:522-655) and SearchForTriangulation (:657-823) walk node by node.  An ORBvoc.bin-sized synthetic vocabulary
(k = 10, L = 6, 10^6 words; the real blob is absent, .MISSING_LARGE_BLOBS:1), C3 (1280x720, 2000 features)
and C5 (4000 features) frame pairs extracted on the GPU; every link compared with the oracle's chain."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vocabs(orbgpu_mod, oracle_mod, tmp_path_factory):
    from orbgpu.synth import write_synth_vocab_large
    path = str(tmp_path_factory.mktemp("voc") / "voc_k10_L6.bin")
    write_synth_vocab_large(path, 10, 6, seed=4)
    gv = orbgpu_mod.ORBVocabulary()
    gv.loadFromBinaryFile(path)
    ov = oracle_mod.OracleVocabulary(path)
    # 10^6 leaves, + 1: the loader replays the reference's while(!f.eof()) read, which stores the last record
    # twice (TemplatedVocabulary.h loadFromBinaryFile)
    assert (gv.k, gv.L, gv.nwords) == (10, 6, 10 ** 6 + 1) and (ov.k, ov.L) == (10, 6)
    yield gv, ov
    gv.close()


def _pair(orbgpu_mod, nf, seed):
    """Two views of one synthetic scene (the second shifted by (2, 3) px), extracted on the GPU."""
    from orbgpu.synth import synth_frame
    a = synth_frame(1280, 720, seed)
    b = np.roll(a, (3, 2), axis=(0, 1))
    ex = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7)
    ka, da = ex(a)
    kb, db = ex(b)
    return ka, da, kb, db


def _ofv(oracle_mod, fv):
    ids = sorted(fv)
    return oracle_mod.make_featvec(ids, [fv[i] for i in ids])


@pytest.mark.parametrize("nf,seed", [(2000, 21), (4000, 22)])   # C3, C5
def test_vocab_featvec_into_bow_matchers(orbgpu_mod, oracle_mod, vocabs, nf, seed):
    gv, ov = vocabs
    ka, da, kb, db = _pair(orbgpu_mod, nf, seed)
    assert len(da) > 0.95 * nf and len(db) > 0.95 * nf
    # link 1: ComputeBoW on the GPU = the oracle's transform (BowVector values and FeatureVector lists)
    bow_a, fva = gv.transform(da, 4)
    bow_b, fvb = gv.transform(db, 4)
    obow_a, ofva = ov.transform(da, 4)
    obow_b, ofvb = ov.transform(db, 4)
    assert fva == ofva and fvb == ofvb
    assert bow_a == obow_a and bow_b == obow_b   # exact doubles (the BowVector the scores read)
    assert len(fva) > 50   # levelsup 4 on a 6-level tree: nodes of level 2 (<= 100)
    oa, _ka = _ofv(oracle_mod, fva)
    ob, _kb = _ofv(oracle_mod, fvb)
    rng = np.random.default_rng(seed)
    # link 2: SearchByBoW(KF, F) as TrackReferenceKeyFrame calls it (Tracking.cc:1029-1032, ORBmatcher(0.7, true)),
    # map points on ~70 % of the keyframe's features
    mp = (rng.random(len(da)) < 0.7).astype(np.uint8)
    n, m = orbgpu_mod.ORBmatcher(0.7, True).SearchByBoW_KF_F(da, ka["angle"], mp, fva, db, kb["angle"], fvb)
    on, om = oracle_mod.search_by_bow_kf_f(0.7, True, da, ka["angle"], mp, oa, db, kb["angle"], ob)
    assert n == on and np.array_equal(m, om) and n > 0.2 * nf
    # SearchByBoW(KF, KF) as LoopClosing::ComputeSim3 calls it (LoopClosing.cc:265, ORBmatcher(0.75, true))
    mp2 = (rng.random(len(db)) < 0.7).astype(np.uint8)
    n2, m2 = orbgpu_mod.ORBmatcher(0.75, True).SearchByBoW_KF_KF(da, ka["angle"], mp, fva, db, kb["angle"], mp2, fvb)
    on2, om2 = oracle_mod.search_by_bow_kf_kf(0.75, True, da, ka["angle"], mp, oa, db, kb["angle"], mp2, ob)
    assert n2 == on2 and np.array_equal(m2, om2) and n2 > 0
    # link 3: SearchForTriangulation as LocalMapping::CreateNewMapPoints calls it (LocalMapping.cc:225, 278:
    # ORBmatcher(0.6, false)) on the features without a map point, mono pair, epipole far outside the image;
    # F12 of a pure horizontal translation (epipolar lines y2 = y1) with a little noise
    mp_t1 = (rng.random(len(da)) < 0.3).astype(np.uint8)
    mp_t2 = (rng.random(len(db)) < 0.3).astype(np.uint8)
    ur = np.full(len(da), -1.0, np.float32), np.full(len(db), -1.0, np.float32)
    F = np.array([[0, 0, 0], [0, 0, -1], [0, 1, 0]], np.float32) + rng.normal(0, 1e-4, (3, 3)).astype(np.float32)
    t = oracle_mod.OracleExtractor(nf).tables()
    pairs = orbgpu_mod.ORBmatcher(0.6, False).SearchForTriangulation(da, ka, mp_t1, ur[0], fva, db, kb, mp_t2, ur[1],
                                                                     fvb, F, 1e5, 1e5, t["scale"], t["sigma2"], False)
    op = oracle_mod.search_for_triangulation(False, False, da, ka, mp_t1, ur[0], oa, db, kb, mp_t2, ur[1], ob, F,
                                             1e5, 1e5, t["scale"], t["sigma2"])
    assert np.array_equal(pairs, op) and len(op) > 0

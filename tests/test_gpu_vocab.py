"""GPU parity: DBoW2 vocabulary transform (TemplatedVocabulary.h:1139-1277 via Frame::ComputeBoW,
Frame.cc:562-569) through liborbgpu's descent kernel vs the oracle restatement —
word ids, weights, FeatureVector nodes and the assembled BowVector / FeatureVector identical.
ORBvoc.bin is absent from the container, so the vocabularies are synthetic files in its format."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (k, L, scoring, weighting): ORB-SLAM's own TF_IDF + L1_NORM first, then the other normalisations
VOCABS = [(10, 3, 0, 0), (6, 4, 1, 2), (8, 3, 5, 1), (5, 4, 3, 3)]


@pytest.fixture(scope="module")
def descs(orbgpu_mod):
    from orbgpu.synth import synth_frame
    g = orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)
    _, d1 = g(synth_frame(640, 480, 12))
    rnd = np.random.default_rng(5).integers(0, 256, (300, 32), dtype=np.uint8)
    return np.concatenate([d1, rnd])


@pytest.mark.parametrize("k,L,scoring,weighting", VOCABS)
@pytest.mark.parametrize("levelsup", [0, 1, 2, 4])
def test_vocab_transform_bit_exact(orbgpu_mod, oracle_mod, tmp_path, descs, k, L, scoring, weighting, levelsup):
    from orbgpu.synth import write_synth_vocab
    path = str(tmp_path / f"voc_{k}_{L}_{scoring}_{weighting}.bin")
    write_synth_vocab(path, k, L, seed=k * 10 + L, scoring=scoring, weighting=weighting)
    ov = oracle_mod.OracleVocabulary(path)
    gv = orbgpu_mod.ORBVocabulary()
    gv.loadFromBinaryFile(path)
    assert (gv.k, gv.L, gv.scoring, gv.weighting, gv.nnodes, gv.nwords) == \
        (ov.k, ov.L, ov.scoring, ov.weighting, ov.nnodes, ov.nwords)
    ow, owt, ond = ov.transform_each(descs, levelsup)
    gw, gwt, gnd = gv.transform_each(descs, levelsup)
    assert np.array_equal(gw, ow) and np.array_equal(gnd, ond)
    assert np.array_equal(gwt.astype(np.float64), owt)
    obow, ofv = ov.transform(descs, levelsup)
    gbow, gfv = gv.transform(descs, levelsup)
    assert gbow == obow and gfv == ofv     # exact doubles, same key order / index lists
    gv.close()


def test_vocab_batch_device_matches_host(orbgpu_mod, oracle_mod, tmp_path):
    from orbgpu import _lib
    from orbgpu.synth import synth_batch, write_synth_vocab
    path = str(tmp_path / "voc.bin")
    write_synth_vocab(path, 10, 3, seed=3)
    gv = orbgpu_mod.ORBVocabulary()
    gv.loadFromBinaryFile(path)
    ov = oracle_mod.OracleVocabulary(path)
    B = 4
    bx = orbgpu_mod.BatchExtractor(1000, 640, 480, B)
    bx.upload(synth_batch(640, 480, B, first=50))
    bx.launch()
    cap = bx.kp_cap
    L = _lib.lib()
    dw, dwt, dnd = (bx._alloc(B * cap * 4) for _ in range(3))
    _lib.check(L.orb_vocab_transform_batch_device(bx.h, gv.v, B, 1, dw, dwt, dnd))
    bx.sync()
    w = np.zeros(B * cap, np.int32)
    wt = np.zeros(B * cap, np.float32)
    nd = np.zeros(B * cap, np.uint32)
    for dst, src in ((w, dw), (wt, dwt), (nd, dnd)):
        _lib.check(L.orb_memcpy_d2h(bx.h, dst.ctypes.data, src, dst.nbytes))
    for f in range(B):
        _, desc = bx.results(f)
        ow, owt, ond = ov.transform_each(desc, 1)
        n = len(desc)
        assert np.array_equal(w[f * cap:f * cap + n], ow)
        assert np.array_equal(nd[f * cap:f * cap + n], ond)
        assert np.array_equal(wt[f * cap:f * cap + n].astype(np.float64), owt)
    for p in (dw, dwt, dnd):
        L.orb_device_free(bx.h, p)
    bx.close()
    gv.close()


def test_vocab_bad_file_is_an_error(orbgpu_mod, tmp_path):
    p = tmp_path / "bad.bin"
    p.write_bytes(b"\x01\x00\x00\x00" * 3)
    gv = orbgpu_mod.ORBVocabulary()
    with pytest.raises(orbgpu_mod.OrbError):
        gv.loadFromBinaryFile(str(p))

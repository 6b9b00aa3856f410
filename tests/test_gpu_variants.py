"""GPU parity of the swappable OpenCV arithmetic (orb_params.variant, include/orbgpu.h ORB_VARIANT_*).

The reference links whichever OpenCV 2.4.3-3.4 the build machine has (CMakeLists.txt:31-37) and calls its
resize (ORBextractor.cc:1120) and GaussianBlur (:1085-1086); the octree sort (:684) breaks size ties by
heap address.  Each variant of the product kernels is compared byte for byte with the oracle run under
the matching ORACLE_* flag (the bit values are equal), at C2 and C3 sizes, through the single-frame
host path, the batched bench configuration (B = 256, two contexts, graph replay) and the birdview
stream (cv::ORB's own pyramid resize and descriptor blur).  Each variant is also checked to CHANGE the
oracle's output on these frames, so the test would notice a kernel that ignores its variant bit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TIE, RESIZE, BLUR, NOFMA = 1, 2, 4, 8

VARIANTS = [TIE, RESIZE, BLUR, NOFMA, RESIZE | BLUR, TIE | RESIZE | BLUR | NOFMA]


def _same(a, b):
    (ka, da), (kb, db) = a, b
    return len(ka) == len(kb) and ka.tobytes() == kb.tobytes() and np.array_equal(da, db)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("w,h,nf,idx,kind", [
    (640, 480, 1000, 0, "scene"),      # C2
    (1280, 720, 2000, 7, "scene"),     # C3
    (1280, 720, 2000, 9, "noise"),     # maximum candidates: phase-2 ties everywhere
    (641, 479, 1000, 2, "scene"),      # odd width: blur tail columns (x >= w & ~3), resize edges
])
def test_variant_single_frame_bit_exact(orbgpu_mod, oracle_mod, variant, w, h, nf, idx, kind):
    from orbgpu.synth import synth_frame
    img = synth_frame(w, h, idx, kind)
    o = oracle_mod.OracleExtractor(nf, flags=variant)
    ref = o(img)
    g = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7, variant=variant)
    got = g(img)
    assert _same(got, ref), (variant, len(got[0]), len(ref[0]))
    pyr = g.mvImagePyramid
    for l in range(8):   # the resize variant shows in every level above 0
        assert np.array_equal(pyr[l], o.level(l)), (variant, l)


@pytest.mark.parametrize("variant,w,h,nf,idx", [
    (TIE, 1280, 720, 2000, 7), (RESIZE, 1280, 720, 2000, 7), (RESIZE, 640, 480, 1000, 0),
    (TIE, 640, 480, 1000, 0), (BLUR, 1280, 720, 2000, 0),   # (blur moves ~half of the C3 frames: frame 0 does)
])
def test_variant_changes_the_reference_output(orbgpu_mod, oracle_mod, variant, w, h, nf, idx):
    """The variants are not no-ops on these frames (DESIGN.md §3.3 blast radius): the oracle's default and
    variant outputs differ, and the GPU follows each."""
    from orbgpu.synth import synth_frame
    img = synth_frame(w, h, idx)
    d = oracle_mod.OracleExtractor(nf)(img)
    v = oracle_mod.OracleExtractor(nf, flags=variant)(img)
    assert not _same(d, v), variant
    g0 = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7)(img)
    gv = orbgpu_mod.ORBextractor(nf, 1.2, 8, 20, 7, variant=variant)(img)
    assert _same(g0, d) and _same(gv, v)


@pytest.mark.parametrize("w,h,nf,variant", [
    (1280, 720, 2000, RESIZE | BLUR | TIE),   # C3 bench configuration under the 3.x-generic / tie-reversed build
    (1280, 720, 2000, NOFMA),
    (640, 480, 1000, RESIZE | BLUR | TIE),    # C2
])
def test_variant_bench_configuration_bit_exact(orbgpu_mod, oracle_mod, w, h, nf, variant):
    from orbgpu.synth import bench_frames
    B = 256
    frames = bench_frames(w, h, B, first=0)
    exs = [orbgpu_mod.BatchExtractor(nf, w, h, B, variant=variant) for _ in range(2)]
    for e in exs:
        e.upload(frames)
    for step in range(4):
        exs[step % 2].launch()
    for e in exs:
        e.sync()
    o = oracle_mod.OracleExtractor(nf, flags=variant)
    ref = {f: o(frames[f]) for f in (0, 64, 255)}
    for e in exs:
        for f, r in ref.items():
            assert _same(e.results(f), r), (variant, f)
    for e in exs:
        e.close()


def test_variant_small_batch_shapes(orbgpu_mod, oracle_mod):
    """C5's 8-frame batch (1024-thread octree blocks, one keypoint per describe wave for B = 1)."""
    from orbgpu.synth import bench_frames
    frames = bench_frames(1280, 720, 8, first=3)
    for B in (8, 1):
        e = orbgpu_mod.BatchExtractor(4000, 1280, 720, B, variant=TIE | RESIZE | BLUR | NOFMA)
        e.upload(frames[:B])
        e.launch()
        e.sync()
        o = oracle_mod.OracleExtractor(4000, flags=TIE | RESIZE | BLUR | NOFMA)
        for f in range(B):
            assert _same(e.results(f), o(frames[f])), (B, f)
        e.close()


def test_unknown_variant_bits_rejected(orbgpu_mod):
    with pytest.raises(orbgpu_mod.OrbError):
        orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7, variant=16)   # ORACLE_TRIG_CR: not a product variant
    with pytest.raises(orbgpu_mod.OrbError):
        orbgpu_mod.BirdORB(2000, variant=TIE)                        # cv::ORB has no octree


@pytest.mark.parametrize("variant", [RESIZE, BLUR, RESIZE | BLUR])
@pytest.mark.parametrize("w,h,idx,masked", [(1280, 720, 1, True), (641, 479, 14, False)])
def test_bird_variant_bit_exact(orbgpu_mod, oracle_mod, variant, w, h, idx, masked):
    """cv::ORB's pyramid (resize + mask resize, orb.cpp) and descriptor blur follow the same OpenCV build."""
    from orbgpu.synth import synth_bird_mask, synth_frame
    img = synth_frame(w, h, idx)
    mask = synth_bird_mask(w, h, idx) if masked else None
    o = oracle_mod.OracleCvORB(2000, flags=variant)
    ko, do = o.extract(img, mask)
    b = orbgpu_mod.BirdORB(2000, variant=variant)
    kg, dg = b.extract(img, mask)
    assert kg.tobytes() == ko.tobytes() and np.array_equal(dg, do), variant
    if variant & RESIZE:
        k0, _ = oracle_mod.OracleCvORB(2000).extract(img, mask)
        assert k0.tobytes() != ko.tobytes()   # the resize variant moves the cv::ORB keypoints too
    b.close()

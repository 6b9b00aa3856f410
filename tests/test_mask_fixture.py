"""The reference's only image as test input: Examples/Monocular/mask_new_front.png (1920x1208), which
mono_fisheye.cc:56 reads and :102-116 applies (applyMask, crop 1900x800, 1/2 resize) before every frame
goes to ORBextractor / the birdview cv::ORB.  tests/golden/mask_new_front.npz (tools/gen_mask_fixture.py)
holds the mask as bits, the oracle's outputs on the driver's 950x400 frame built from it (two seeds), and
the PNG converted to gray (the low-texture edge frame of SURVEY 8(d)) with its oracle extraction.

CPU: the oracle reproduces the fixture.  GPU: ORBextractor (fisheye.yaml's 2000 / 1.2 / 8 / 15 / 5), the
birdview stream with the frame's keep mask and the 1920x1208 gray frame, byte for byte."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN

SEEDS = (0, 5)


@pytest.fixture(scope="module")
def fx():
    p = os.path.join(GOLDEN, "mask_new_front.npz")
    if not os.path.exists(p):
        pytest.skip("mask_new_front.npz missing (run tools/gen_mask_fixture.py)")
    g = np.load(p)
    keep = np.unpackbits(g["keep_bits"], axis=1)[:, :int(g["shape"][1])].astype(bool)
    assert keep.shape == (1208, 1920)
    return g, keep


def _frame(g, keep, s):
    from orbgpu.synth import fisheye_driver_frame
    img, km = fisheye_driver_frame(keep, s)
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g[f"img_sha256_{s}"])
    return img, km


def test_fixture_mask_geometry(fx):
    """applyMask + crop + 1/2 resize (mono_fisheye.cc:102-116): 950x400, masked pixels are 0."""
    g, keep = fx
    assert 0 < (~keep).sum() < keep.size // 2
    img, km = _frame(g, keep, 0)
    assert img.shape == (400, 950) and km.shape == (400, 950)
    assert (img[km == 0] < 128).mean() > 0.9   # mostly zero where the driver masked the camera image


@pytest.mark.parametrize("s", SEEDS)
def test_oracle_matches_mask_fixture(fx, oracle_mod, s):
    g, keep = fx
    img, km = _frame(g, keep, s)
    k, d = oracle_mod.OracleExtractor(2000, 1.2, 8, 15, 5)(img)
    assert k.tobytes() == g[f"kps_{s}"].tobytes() and np.array_equal(d, g[f"desc_{s}"])
    bk, bd = oracle_mod.OracleCvORB(2000).extract(img, km)
    assert bk.tobytes() == g[f"bird_kps_{s}"].tobytes() and np.array_equal(bd, g[f"bird_desc_{s}"])


def test_oracle_matches_gray_mask_frame(fx, oracle_mod):
    g, _ = fx
    k, d = oracle_mod.OracleExtractor(2000, 1.2, 8, 20, 7)(g["gray"])
    assert len(k) == len(g["kps_gray"]) and k.tobytes() == g["kps_gray"].tobytes()
    assert np.array_equal(d, g["desc_gray"])


@pytest.mark.gpu
@pytest.mark.parametrize("s", SEEDS)
def test_gpu_extractor_on_mask_frame(fx, orbgpu_mod, s):
    """ORBextractor::operator() on the fisheye driver's masked 950x400 frame (Frame.cc:414-420)."""
    g, keep = fx
    img, _ = _frame(g, keep, s)
    k, d = orbgpu_mod.ORBextractor(2000, 1.2, 8, 15, 5)(img)
    assert len(k) == len(g[f"kps_{s}"]) > 1900
    assert k.tobytes() == g[f"kps_{s}"].tobytes() and np.array_equal(d, g[f"desc_{s}"])


@pytest.mark.gpu
@pytest.mark.parametrize("s", SEEDS)
def test_gpu_birdview_on_mask_frame(fx, orbgpu_mod, s):
    """The birdview stream (Frame.cc:320-342: masked cv::ORB detect, cornerSubPix, compute) with the
    driver's keep mask as the detection mask."""
    g, keep = fx
    img, km = _frame(g, keep, s)
    bk, bd = orbgpu_mod.BirdORB(2000).extract(img, km)
    assert len(bk) == len(g[f"bird_kps_{s}"]) > 1900
    assert bk.tobytes() == g[f"bird_kps_{s}"].tobytes() and np.array_equal(bd, g[f"bird_desc_{s}"])


@pytest.mark.gpu
def test_gpu_extractor_on_gray_mask_frame(fx, orbgpu_mod):
    """The PNG as a 1920x1208 gray frame: almost no texture, so nearly every cell takes the minThFAST
    fallback (ORBextractor.cc:812-816) and the octree sees a handful of candidates per level."""
    g, _ = fx
    k, d = orbgpu_mod.ORBextractor(2000, 1.2, 8, 20, 7)(g["gray"])
    assert len(k) == len(g["kps_gray"]) > 0
    assert k.tobytes() == g["kps_gray"].tobytes() and np.array_equal(d, g["desc_gray"])

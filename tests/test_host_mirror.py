"""The C++ host mirror (orb-slam-birdview_amd/host/: ORB_SLAM2::ORBextractor / ORBmatcher over the
C-ABI).  GPU: tests/cpp/test_host_mirror drives the mirror the way Frame/Tracking/LocalMapping drive
the reference classes and checks every result against the oracle, bit-exact.  CPU: the mirror
builds, links liborbgpu and fails loudly (OrbGpuError, no CPU fallback) without a device."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "orb-slam-birdview_amd")
CPP = os.path.join(ROOT, "tests", "cpp")
BIN = os.path.join(CPP, "test_host_mirror")


@pytest.fixture(scope="module")
def mirror_bin():
    subprocess.check_call(["make", "-s", "-C", PKG, "liborbslam_host.so"])
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    subprocess.check_call(["make", "-s", "-C", CPP])
    return BIN


def _run(bin_path, frames, nf, tmp_path, vocab=None):
    n, h, w = frames.shape
    raw = tmp_path / f"frames_{w}x{h}.raw"
    raw.write_bytes(np.ascontiguousarray(frames, np.uint8).tobytes())
    argv = [bin_path, str(raw), str(w), str(h), str(n), str(nf)] + ([vocab] if vocab else [])
    p = subprocess.run(argv, capture_output=True, text=True, timeout=300)
    return p.returncode, p.stdout, p.stderr


def test_mirror_library_exports_reference_api(mirror_bin):
    import orbgpu
    orbgpu._lib.lib()   # torch's HIP runtime first: loading the mirror before it would pull in a second one
    lib = ctypes.CDLL(os.path.join(PKG, "liborbslam_host.so"))
    out = subprocess.run(["nm", "-DC", "--defined-only", os.path.join(PKG, "liborbslam_host.so")],
                         capture_output=True, text=True, check=True).stdout
    for sym in ["ORB_SLAM2::ORBextractor::ORBextractor(int, float, int, int, int)",
                "ORB_SLAM2::ORBextractor::operator()(ORB_SLAM2::ImageView const&, ORB_SLAM2::ImageView const&, "
                "std::vector<orb_keypoint, std::allocator<orb_keypoint> >&, ORB_SLAM2::DescriptorMat&)",
                "ORB_SLAM2::ORBmatcher::ORBmatcher(float, bool)",
                "ORB_SLAM2::ORBmatcher::DescriptorDistance(unsigned char const*, unsigned char const*)",
                "ORB_SLAM2::ORBmatcher::SearchByBoW(ORB_SLAM2::KeyFrameData const&, ORB_SLAM2::FrameData const&",
                "ORB_SLAM2::ORBmatcher::SearchByBoW(ORB_SLAM2::KeyFrameData const&, ORB_SLAM2::KeyFrameData const&",
                "ORB_SLAM2::ORBmatcher::SearchForTriangulation(",
                "ORB_SLAM2::ORBmatcher::SearchForInitialization(",
                "ORB_SLAM2::ORBmatcher::BirdviewMatch(",
                "ORB_SLAM2::FrameGrid::GetFeaturesInArea(",
                "ORB_SLAM2::ComputeStereoMatches(",
                "ORB_SLAM2::BirdviewORB::create(", "ORB_SLAM2::BirdviewORB::detect(", "ORB_SLAM2::BirdviewORB::compute(",
                "ORB_SLAM2::cornerSubPix(",
                "ORB_SLAM2::ORBVocabulary::transform("]:
        assert sym in out, sym
    del lib


def test_mirror_fails_loudly_without_gpu(mirror_bin, tmp_path):
    import orbgpu
    if orbgpu.device_count() > 0:
        pytest.skip("a GPU is present")
    rc, out, _ = _run(mirror_bin, np.zeros((1, 64, 64), np.uint8), 100, tmp_path)
    assert rc == 1
    assert "CHECK exception FAIL orb_create" in out and "no CPU fallback" in out


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,nf", [(640, 480, 1000), (1280, 720, 2000)])
def test_mirror_parity_on_gpu(mirror_bin, tmp_path, w, h, nf):
    from orbgpu.synth import synth_frame
    from orbgpu.synth import synth_stereo_right
    a = synth_frame(w, h, 21)
    # frame 1: a rectified right view of frame 0 (matchers and ComputeStereoMatches use the pair)
    frames = np.stack([a, synth_stereo_right(a, 21), synth_frame(w, h, 5, "noise")])
    from orbgpu.synth import write_synth_vocab
    voc = str(tmp_path / "voc.bin")
    write_synth_vocab(voc, 10, 4, seed=2)
    rc, out, err = _run(mirror_bin, frames, nf, tmp_path, voc)
    fails = [l for l in out.splitlines() if " FAIL" in l]
    assert rc == 0 and not fails, "\n".join(fails) + "\n" + err[-2000:]
    summary = [l for l in out.splitlines() if l.startswith("SUMMARY")][0].split()
    assert int(summary[1]) >= 20 and int(summary[2]) == 0


@pytest.fixture(scope="module")
def cv_overload_bin():
    # the mirror's -DORBGPU_WITH_OPENCV overloads, compiled over tests/cpp/cv_api (a model of the OpenCV
    # 3.2 types: OpenCV is absent in this image)
    subprocess.check_call(["make", "-s", "-C", CPP, "test_cv_overload"])
    return os.path.join(CPP, "test_cv_overload")


def test_cv_overload_builds_and_fails_loudly_without_gpu(cv_overload_bin, tmp_path):
    import orbgpu
    if orbgpu.device_count() > 0:
        pytest.skip("a GPU is present")
    rc, out, _ = _run(cv_overload_bin, np.zeros((1, 64, 64), np.uint8), 100, tmp_path)
    assert rc == 1 and "CHECK exception FAIL" in out


@pytest.mark.gpu
def test_cv_overload_matches_plain_overload(cv_overload_bin, tmp_path):
    # Frame.cc:414-420's call shape: (*extractor)(im, cv::Mat(), mvKeys, mDescriptors) on a padded cv::Mat,
    # then mvImagePyramid[l] as cv::Mat; bytes equal to the ImageView overload's (itself bit-exact vs the oracle)
    from orbgpu.synth import synth_frame
    frames = np.stack([synth_frame(1280, 720, 3), synth_frame(1280, 720, 6, "noise")])
    rc, out, err = _run(cv_overload_bin, frames, 2000, tmp_path)
    fails = [l for l in out.splitlines() if " FAIL" in l]
    assert rc == 0 and not fails, "\n".join(fails) + "\n" + err[-2000:]
    summary = [l for l in out.splitlines() if l.startswith("SUMMARY")][0].split()
    assert int(summary[1]) == 12 and int(summary[2]) == 0

"""Sanitizer runs of the host code.  GPU AddressSanitizer is not available on this pool, so
only host code is instrumented:

* CPU: the oracle under ASan + UBSan on every entry point (extraction under every flag, the literal
  std::list octree, cv::ORB + cornerSubPix, SearchByBoW, stereo, distinctive descriptors), and its
  threaded CPU-baseline paths under TSan (tests/cpp/oracle_sanitize.cc).
* GPU box: the C++ host mirror (orb-slam-birdview_amd/host/) compiled into the parity harness under
  ASan + UBSan, and under TSan, where its stereo section drives a left and a right extractor from a fresh
  std::thread per frame while a matcher runs on a third (Frame.cc:124-127's pattern).
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1:suppressions=" + os.path.join(CPP, "tsan.supp"))


def _no_aslr(kind):
    """TSan's shadow layout needs the executable at an address it expects; kernels with 32-bit mmap
    randomisation break that ("unexpected memory mapping"), so TSan runs start with ASLR off (setarch -R
    executes the test binary directly, before anything touches the GPU)."""
    if kind != "tsan":
        return []
    import platform
    import shutil
    return ["setarch", platform.machine(), "-R"] if shutil.which("setarch") else []


def _frames(tmp_path, w, h, n):
    from orbgpu.synth import synth_frame
    fr = np.stack([synth_frame(w, h, 70 + i) for i in range(n - 1)] + [synth_frame(w, h, 1, "noise")])
    p = tmp_path / f"fr_{w}x{h}.raw"
    p.write_bytes(fr.tobytes())
    return str(p)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_oracle_under_sanitizer(tmp_path, kind):
    target = f"oracle_sanitize_{kind}"
    subprocess.check_call(["make", "-s", "-C", CPP, target], timeout=600)
    raw = _frames(tmp_path, 640, 480, 3)
    args = _no_aslr(kind) + [os.path.join(CPP, target), raw, "640", "480", "3"] + (["threads"] if kind == "tsan" else [])
    p = subprocess.run(args, capture_output=True, text=True, timeout=900, env=ENV)
    assert p.returncode == 0 and "bad=0" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
    assert "WARNING: ThreadSanitizer" not in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_mirror_under_sanitizer(tmp_path, kind):
    binary = os.path.join(CPP, f"test_host_mirror_{kind}")
    if not os.path.exists(binary):   # built in-tree on the CPU side (__graft_entry__.build); never on the box
        pytest.skip(f"{binary} not built")
    from orbgpu.synth import synth_frame
    left = synth_frame(640, 480, 3)
    frames = np.stack([left, np.roll(left, 5, axis=1), synth_frame(640, 480, 4), synth_frame(640, 480, 5)])
    raw = tmp_path / "m.raw"
    raw.write_bytes(frames.tobytes())
    p = subprocess.run(_no_aslr(kind) + [binary, str(raw), "640", "480", "4", "1000"], capture_output=True, text=True,
                       timeout=600, env=ENV)
    assert p.returncode == 0 and "SUMMARY" in p.stdout, (p.stdout[-3000:], p.stderr[-4000:])
    assert "stereo_threads_fresh_thread_per_frame" in p.stdout
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr
    assert "WARNING: ThreadSanitizer" not in p.stderr, p.stderr[-4000:]

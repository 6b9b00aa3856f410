"""Pins of the float semantics the oracle and the kernels share, checked on the CPU:

* glibc sinf/cosf (ORBextractor.cc:113): oracle/glibc_sincosf.inc equals this machine's libm on every
  float in [0, 2*pi] (tools/trig_pin.cpp, ~20 s), and the device copy (csrc/glibc_trig.h) carries the
  same table;
* the FMA contractions of the reference's -O3 -march=native build: tools/ref_flags_probe.cpp, compiled
  with those flags, agrees with the explicit forms the oracle and the kernels use
  (tools/ref_flags_check.cpp).

The GPU side of the trig pin (orb_debug_sincosf vs the oracle) is tests/test_gpu_extract.py.
"""
import json
import os
import platform
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")


def _cpu_has_fma():
    try:
        flags = open("/proc/cpuinfo").read()
    except OSError:
        return False
    return re.search(r"^flags\s*:.*\bfma\b", flags, re.M) is not None and re.search(r"\bavx2\b", flags) is not None


def _toolchain():
    gcc = subprocess.run(["g++", "-dumpfullversion"], capture_output=True, text=True).stdout.strip()
    return f"glibc {platform.libc_ver()[1]}, g++ {gcc}"


# glibc (2.28+) selects its FMA build of sinf/cosf by ifunc on an AVX2+FMA host; the restatement is of
# that build, so on a host without FMA libm runs different code and the pin does not apply there.
needs_fma = pytest.mark.skipif(not _cpu_has_fma(), reason="host CPU lacks AVX2/FMA: glibc runs its non-FMA sinf/cosf")


def _build(tmp_path, name, cmds):
    for c in cmds:
        subprocess.check_call(c, cwd=tmp_path)
    return os.path.join(tmp_path, name)


@pytest.fixture(scope="module")
def trig_pin(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("trig"))
    return _build(d, "trig_pin", [["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", "trig_pin",
                                   os.path.join(TOOLS, "trig_pin.cpp"), "-lm"]])


@needs_fma
def test_glibc_sincosf_restatement_equals_libm_everywhere_on_0_2pi(trig_pin):
    print("pin scope:", _toolchain())
    out = json.loads(subprocess.check_output([trig_pin, "exhaustive"], timeout=600))
    assert out["floats"] > 1_000_000_000
    assert out["restatement_vs_libm_sinf"] == 0 and out["restatement_vs_libm_cosf"] == 0
    assert out["sincosf_vs_sinf_cosf"] == 0            # GCC's merged sincosf call computes the same pair
    # libm is NOT correctly rounded: round 1's double-then-round pin differed here
    assert out["libm_vs_correctly_rounded_sinf"] > 0 and out["libm_vs_correctly_rounded_cosf"] > 0


def test_device_trig_table_matches_oracle_table():
    """csrc/glibc_trig.h and oracle/glibc_sincosf.inc are independent restatements: same constants."""
    hexf = re.compile(r"-?0x1(?:\.[0-9A-Fa-f]+)?p[+-]?\d+")
    dev = open(os.path.join(ROOT, "orb-slam-birdview_amd", "csrc", "glibc_trig.h")).read()
    orc = open(os.path.join(ROOT, "oracle", "glibc_sincosf.inc")).read()
    to = lambda s: sorted({float.fromhex(h.lstrip("-")) for h in hexf.findall(s)})
    assert to(dev) == to(orc)


@needs_fma
def test_reference_flags_contraction_forms(tmp_path):
    # -march=x86-64-v3 stands for the reference's -march=native on an AVX2+FMA host (CMakeLists.txt:10-11)
    print("pin scope:", _toolchain())
    d = str(tmp_path)
    exe = _build(d, "chk", [
        ["g++", "-O3", "-march=x86-64-v3", "-std=c++11", "-c", os.path.join(TOOLS, "ref_flags_probe.cpp"), "-o", "probe.o"],
        ["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-c", os.path.join(TOOLS, "ref_flags_check.cpp"), "-o", "check.o"],
        ["g++", "-o", "chk", "check.o", "probe.o", "-lm"]])
    out = json.loads(subprocess.check_output([exe, "3001"], timeout=600))
    assert out["offsets_mismatch_vs_fused_form"] == 0 and out["descriptor_mismatch"] == 0
    assert out["epipolar_dsqr_mismatch"] == 0 and out["epipole_gate_mismatch"] == 0
    assert out["epipolar_uncontracted_differs"] > 0   # the contraction is real (dsqr's last bits)

"""CPU: the C-ABI library loads, exports every symbol include/orbgpu.h declares, and its host-only
helpers agree with the oracle.  No compute call needs a GPU here; without one orb_create must fail
loudly (no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "orbgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(orb_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from orbgpu import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    names = _declared_symbols()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the Python binding declares a signature for each of them
    assert set(names) <= set(_lib.SIGNATURES), set(names) - set(_lib.SIGNATURES)


def test_abi_version_and_keypoint_layout(orbgpu_mod):
    from orbgpu import _lib
    assert _lib.lib().orb_abi_version() == 2   # 2: orb_params / orb_bird_params gained `variant`
    assert orbgpu_mod.KP_DTYPE.itemsize == 28   # cv::KeyPoint
    # the ctypes structs match the header's field lists
    assert [f for f, _ in _lib.OrbParams._fields_][-1] == "variant"
    assert [f for f, _ in _lib.OrbBirdParams._fields_][-1] == "variant"


def test_variant_bits_match_header_and_oracle(orbgpu_mod):
    """ORB_VARIANT_* (include/orbgpu.h) == the Python constants == the oracle's ORACLE_* flags, so a parity
    test passes one value to both sides."""
    hdr = open(os.path.join(ROOT, "include", "orbgpu.h")).read()
    ora = open(os.path.join(ROOT, "oracle", "orb_oracle.h")).read()
    v = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define ORB_VARIANT_([A-Z_]+)\s+(\d+)", hdr)}
    o = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define ORACLE_([A-Z_]+)\s+(\d+)", ora)}
    assert v["TIE_REVERSE"] == o["TIE_REVERSE_SEQ"] == orbgpu_mod.VARIANT_TIE_REVERSE
    assert v["RESIZE_GENERIC"] == o["RESIZE_GENERIC"] == orbgpu_mod.VARIANT_RESIZE_GENERIC
    assert v["BLUR_HALFUP"] == o["BLUR_ALL_HALFUP"] == orbgpu_mod.VARIANT_BLUR_HALFUP
    assert v["NO_FMA"] == o["NO_FMA"] == orbgpu_mod.VARIANT_NO_FMA
    assert v["MASK"] == v["TIE_REVERSE"] | v["RESIZE_GENERIC"] | v["BLUR_HALFUP"] | v["NO_FMA"]


def test_no_cpu_fallback_without_gpu(orbgpu_mod):
    if orbgpu_mod.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(orbgpu_mod.OrbError):
        orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7)


def test_invalid_params_rejected(orbgpu_mod):
    with pytest.raises(orbgpu_mod.OrbError):
        orbgpu_mod.ORBextractor(1000, 1.0, 8, 20, 7)   # scaleFactor must be > 1
    with pytest.raises(orbgpu_mod.OrbError):
        orbgpu_mod.ORBextractor(1000, 1.2, 40, 20, 7)  # > ORBGPU_MAX_LEVELS
    with pytest.raises(orbgpu_mod.OrbError):
        orbgpu_mod.ORBextractor(1000, 1.2, 8, 20, 7, variant=32)   # unknown ORB_VARIANT_* bit


def test_descriptor_distance_host_helper(orbgpu_mod, oracle_mod):
    rng = np.random.default_rng(0)
    for _ in range(100):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert orbgpu_mod.ORBmatcher.DescriptorDistance(a, b) == oracle_mod.descriptor_distance(a, b)


def test_features_in_area_host_helper(orbgpu_mod, oracle_mod):
    rng = np.random.default_rng(7)
    n = 400
    k = np.zeros(n, orbgpu_mod.KP_DTYPE)
    k["x"] = rng.uniform(-5, 645, n)
    k["y"] = rng.uniform(-5, 485, n)
    k["octave"] = rng.integers(0, 8, n)
    for _ in range(30):
        x, y, r = rng.uniform(0, 640), rng.uniform(0, 480), rng.uniform(5, 120)
        lv = int(rng.integers(-1, 3))
        a = orbgpu_mod.features_in_area(k, 0, 640, 0, 480, x, y, r, lv, lv)
        b = oracle_mod.features_in_area(k, 0, 640, 0, 480, x, y, r, lv, lv)
        assert a.tolist() == b.tolist()


def test_window_match_grid_rejects_malformed_csr(orbgpu_mod):
    """orb_window_match_grid validates F2's grid CSR before it touches the context (k_window_topk reads
    cell_idx[cell_off[..]], so a malformed CSR would be an out-of-bounds device read): cell_off[0] != 0,
    a decreasing offset and an index past n2 are ORB_ERR_ARG, each with its own message.  The context
    is NULL here (no GPU), so a well-formed grid gets as far as the NULL-context error."""
    from orbgpu import _lib
    L = _lib.lib()
    n2 = 10
    desc = np.zeros((n2, 32), np.uint8)
    k = np.zeros(n2, orbgpu_mod.KP_DTYPE)
    match = np.zeros(n2, np.int32)
    nm = ctypes.c_int(0)

    def call(off, idx):
        g = _lib.OrbFrameGrid(0.0, 0.0, 0.1, 0.1, off.ctypes.data, idx.ctypes.data)
        st = L.orb_window_match_grid(None, 0.9, 1, 1, n2, desc.ctypes.data, k.ctypes.data, None, 100.0, n2,
                                     desc.ctypes.data, k.ctypes.data, g, match.ctypes.data, ctypes.byref(nm))
        return st, L.orb_last_error().decode()

    good = np.zeros(64 * 48 + 1, np.int32)
    good[5:] = n2   # cell 4 holds all ten keypoints
    idx = np.arange(n2, dtype=np.int32)
    assert call(good, idx) == (-1, "NULL context")
    bad = good.copy()
    bad[0] = 1
    assert call(bad, idx) == (-1, "orb_window_match_grid: grid cell_off[0] != 0")
    bad = good.copy()
    bad[100] = 3   # 10 -> 3 -> 10: a run that would start past its end
    assert call(bad, idx) == (-1, "orb_window_match_grid: grid cell_off decreases")
    bad_idx = idx.copy()
    bad_idx[7] = n2
    assert call(good, bad_idx) == (-1, "orb_window_match_grid: grid index out of range")

"""ctypes loader for liborbgpu.so (the in-tree gfx950 build) — the only compute path.

There is no CPU fallback: if the library is missing, or the HIP runtime has no device, the
calls raise.  torch (if importable) is imported first so that the process holds exactly one HIP
runtime (torch bundles its own libamdhip64.so.7; liborbgpu binds to whichever is loaded first).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
# ORBGPU_LIB_PATH: an alternative in-tree build of the same library (A/B of kernel variants)
LIB_PATH = os.environ.get("ORBGPU_LIB_PATH") or os.path.join(PKG_ROOT, "liborbgpu.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "orbgpu.h")

_LIB = None

# OpenCV arithmetic variant bits (include/orbgpu.h ORB_VARIANT_*; equal to the oracle's ORACLE_* flags)
VARIANT_DEFAULT, VARIANT_TIE_REVERSE, VARIANT_RESIZE_GENERIC, VARIANT_BLUR_HALFUP, VARIANT_NO_FMA = 0, 1, 2, 4, 8

vp, ci, cf, csz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t


class OrbParams(ctypes.Structure):
    _fields_ = [("nfeatures", ci), ("scaleFactor", cf), ("nlevels", ci), ("iniThFAST", ci),
                ("minThFAST", ci), ("device", ci), ("max_width", ci), ("max_height", ci),
                ("max_batch", ci), ("variant", ci)]


class OrbBirdParams(ctypes.Structure):
    _fields_ = [("nfeatures", ci), ("scaleFactor", cf), ("nlevels", ci), ("edgeThreshold", ci),
                ("fastThreshold", ci), ("device", ci), ("variant", ci)]


class OrbFeatVec(ctypes.Structure):
    _fields_ = [("nnodes", ci), ("node_ids", vp), ("offsets", vp), ("indices", vp)]


class OrbTriPair(ctypes.Structure):   # orb_tri_pair
    _fields_ = [("n2", ci), ("desc2", vp), ("kps2", vp), ("has_mp2", vp), ("uright2", vp), ("fv2", OrbFeatVec),
                ("F12", vp), ("ex", cf), ("ey", cf), ("scale2", vp), ("sigma2_2", vp), ("nlevels2", ci),
                ("pairs_out", vp), ("cap", ci), ("npairs", ctypes.POINTER(ci))]


class OrbBowKf(ctypes.Structure):   # orb_bow_kf
    _fields_ = [("n", ci), ("desc", vp), ("angle", vp), ("mp", vp), ("fv", OrbFeatVec), ("match", vp),
                ("nmatches", ctypes.POINTER(ci))]


class OrbFrameGrid(ctypes.Structure):
    _fields_ = [("min_x", cf), ("min_y", cf), ("inv_w", cf), ("inv_h", cf), ("cell_off", vp), ("cell_idx", vp)]


# name -> (restype, argtypes); mirrors include/orbgpu.h
SIGNATURES = {
    "orb_abi_version": (ci, []),
    "orb_last_error": (ctypes.c_char_p, []),
    "orb_device_count": (ci, []),
    "orb_create": (vp, [ctypes.POINTER(OrbParams), ctypes.POINTER(ci)]),
    "orb_destroy": (None, [vp]),
    "orb_scale_tables": (ci, [vp, vp, vp, vp, vp, vp, vp]),
    "orb_extract": (ci, [vp, vp, ci, ci, csz, vp, ci, ctypes.POINTER(ci), vp]),
    "orb_get_level": (ci, [vp, ci, ctypes.POINTER(vp), ctypes.POINTER(ci), ctypes.POINTER(ci),
                           ctypes.POINTER(csz)]),
    "orb_batch_kp_cap": (ci, [vp, ci, ci]),
    "orb_extract_batch_device": (ci, [vp, vp, ci, ci, ci, csz, csz, vp, vp, vp, ci]),
    "orb_sync": (ci, [vp]),
    "orb_device_alloc": (vp, [vp, csz]),
    "orb_device_free": (ci, [vp, vp]),
    "orb_memcpy_h2d": (ci, [vp, vp, vp, csz]),
    "orb_memcpy_d2h": (ci, [vp, vp, vp, csz]),
    "orb_memset_device": (ci, [vp, vp, ci, csz]),
    "orb_profile_enable": (ci, [vp, ci]),
    "orb_profile_read": (ci, [vp, vp, vp]),
    "orb_debug_candidates": (ci, [vp, ci, ci, vp, ci]),
    "orb_debug_level_keypoints": (ci, [vp, ci, ci, vp, ci]),
    "orb_debug_level_image": (ci, [vp, ci, ci, vp, ctypes.POINTER(ci), ctypes.POINTER(ci)]),
    "orb_debug_fast_stamps": (ci, [vp, vp, ci]),
    "orb_debug_sincosf": (ci, [vp, vp, ci, vp, vp]),
    "orb_descriptor_distance": (ci, [vp, vp]),
    "orb_hamming_topk": (ci, [vp, vp, ci, vp, ci, vp, vp, vp, ci, vp, vp, vp]),
    "orb_hamming_top2_device": (ci, [vp, vp, ci, vp, ci, vp, vp, vp]),
    "orb_hamming_top2_frames_device": (ci, [vp, vp, vp, ci, ci, vp, vp, vp, vp, vp]),
    "orb_hamming_top2_slices": (ci, [ci, ci, ci]),
    "orb_hamming_top2_mfma_bits": (ci, []),
    "orb_search_by_bow_kf_f": (ci, [vp, cf, ci, ci, vp, vp, vp, OrbFeatVec, ci, vp, vp, OrbFeatVec, vp,
                                    ctypes.POINTER(ci)]),
    "orb_search_by_bow_kf_kf": (ci, [vp, cf, ci, ci, vp, vp, vp, OrbFeatVec, ci, vp, vp, vp, OrbFeatVec, vp,
                                     ctypes.POINTER(ci)]),
    "orb_search_for_triangulation": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, OrbFeatVec, ci, vp, vp, vp, vp,
                                          OrbFeatVec, vp, cf, cf, vp, vp, ci, vp, ci, ctypes.POINTER(ci)]),
    "orb_search_by_bow_kf_f_batch": (ci, [vp, cf, ci, ci, vp, vp, OrbFeatVec, ci, vp]),
    "orb_search_by_bow_kf_kf_batch": (ci, [vp, cf, ci, ci, vp, vp, vp, OrbFeatVec, ci, vp]),
    "orb_search_for_triangulation_batch": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, OrbFeatVec, ci, vp]),
    "orb_window_match": (ci, [vp, cf, ci, ci, ci, vp, vp, ci, vp, vp, vp, vp, vp, ctypes.POINTER(ci)]),
    "orb_window_match_grid": (ci, [vp, cf, ci, ci, ci, vp, vp, vp, cf, ci, vp, vp, OrbFrameGrid, vp,
                                   ctypes.POINTER(ci)]),
    "orb_features_in_area": (ci, [ci, vp, cf, cf, cf, cf, cf, cf, cf, ci, ci, vp, ci]),
    "orb_compute_stereo_matches": (ci, [vp, vp, ci, vp, vp, ci, vp, vp, cf, cf, vp, vp, ctypes.POINTER(ci)]),
    "orb_stereo_batch_device": (ci, [vp, ci, cf, cf, vp, vp, vp]),
    "orb_vocab_load": (ci, [vp, ctypes.c_char_p, ctypes.POINTER(vp)]),
    "orb_vocab_destroy": (None, [vp]),
    "orb_vocab_info": (ci, [vp, vp, vp, vp, vp, vp, vp]),
    "orb_vocab_transform": (ci, [vp, vp, vp, ci, ci, vp, vp, vp]),
    "orb_vocab_transform_batch_device": (ci, [vp, vp, ci, ci, vp, vp, vp]),
    "orb_vocab_bow": (ci, [vp, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "orb_distinctive_descriptors": (ci, [vp, ci, vp, vp, vp]),
    "orb_bird_create": (vp, [ctypes.POINTER(OrbBirdParams), ctypes.POINTER(ci)]),
    "orb_bird_destroy": (None, [vp]),
    "orb_bird_detect": (ci, [vp, vp, ci, ci, csz, vp, csz, vp, ci, ctypes.POINTER(ci)]),
    "orb_bird_compute": (ci, [vp, vp, ci, ci, csz, vp, ctypes.POINTER(ci), vp]),
    "orb_corner_subpix": (ci, [vp, vp, ci, ci, csz, vp, ci, ci, ci, ci, ctypes.c_double]),
    "orb_bird_extract": (ci, [vp, vp, ci, ci, csz, vp, csz, vp, ci, ctypes.POINTER(ci), vp]),
    "orb_bird_extract_device": (ci, [vp, vp, ci, ci, csz, vp, csz, vp, ci, ctypes.POINTER(ci), vp]),
    "orb_bird_footprint_mask": (ci, [vp, ci, ci, csz]),
    "orb_bird_debug_candidates": (ci, [vp, ci, vp, ci]),
    "orb_bird_debug_level": (ci, [vp, ci, vp, ctypes.POINTER(ci), ctypes.POINTER(ci)]),
}

STATUS = {0: "ORB_OK", -1: "ORB_ERR_ARG", -2: "ORB_ERR_HIP", -3: "ORB_ERR_CAPACITY",
          -4: "ORB_ERR_GEOMETRY", -5: "ORB_ERR_NOMEM", -6: "ORB_ERR_INTERNAL"}


class OrbError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        msg = lib().orb_last_error()
        super().__init__(f"{where}: {STATUS.get(status, status)} ({msg.decode() if msg else ''})")


def _preload_torch():
    try:
        import torch  # noqa: F401  (binds the process to torch's HIP runtime before liborbgpu loads)
    except Exception:
        pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built: run `make -C {PKG_ROOT}` (hipcc, gfx950)")
        _preload_torch()
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(status, where=""):
    if status != 0:
        raise OrbError(status, where)
    return status

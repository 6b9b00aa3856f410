"""orbgpu — MI355X-native ORB front-end (Python mirror of the reference C++ interface).

ORBextractor / ORBmatcher keep the names, argument meaning and return conventions of
donglinb/ORB-SLAM-BIRDVIEW include/ORBextractor.h:45-111 and include/ORBmatcher.h:37-119, with
OpenCV containers replaced by numpy: keypoints are a structured array with cv::KeyPoint's 28-byte
layout (KP_DTYPE), descriptors an (n, 32) uint8 array, FeatureVectors a dict {node_id: [indices]}.
Every call runs on the GPU through liborbgpu.so (include/orbgpu.h); there is no CPU fallback.
"""
import ctypes

import numpy as np

from ._lib import (VARIANT_BLUR_HALFUP, VARIANT_DEFAULT, VARIANT_NO_FMA, VARIANT_RESIZE_GENERIC,
                   VARIANT_TIE_REVERSE, OrbBirdParams, OrbError, OrbFeatVec, OrbFrameGrid, OrbParams, check, lib)

__all__ = ["ORBextractor", "ORBmatcher", "BatchExtractor", "KP_DTYPE", "OrbError", "device_count",
           "features_in_area", "compute_stereo_matches", "ORBVocabulary", "BirdORB", "cornerSubPix",
           "bird_footprint_mask", "VARIANT_DEFAULT", "VARIANT_TIE_REVERSE", "VARIANT_RESIZE_GENERIC",
           "VARIANT_BLUR_HALFUP", "VARIANT_NO_FMA"]

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28

TH_LOW, TH_HIGH, HISTO_LENGTH = 50, 100, 30   # ORBmatcher.cc:37-39


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def device_count():
    return lib().orb_device_count()


class _Ctx:
    def __init__(self, nfeatures, scale_factor, nlevels, ini_th, min_th, device=0, max_width=0,
                 max_height=0, max_batch=1, variant=0):
        self.params = OrbParams(nfeatures, scale_factor, nlevels, ini_th, min_th, device, max_width,
                                max_height, max_batch, variant)
        st = ctypes.c_int()
        self.h = lib().orb_create(ctypes.byref(self.params), ctypes.byref(st))
        if not self.h:
            raise OrbError(st.value, "orb_create")
        self.nlevels = nlevels

    def close(self):
        if getattr(self, "h", None):
            lib().orb_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # debug views (parity tests pinpoint the failing stage)
    def debug_candidates(self, level, frame=0):
        cap = 1 << 16
        while True:
            out = np.zeros((cap, 3), np.int32)
            n = lib().orb_debug_candidates(self.h, frame, level, _p(out), cap)
            if n >= 0:
                return out[:n]
            if n == -1:
                raise OrbError(n, "orb_debug_candidates")
            cap = -n

    def debug_level_image(self, level, frame=0):
        """Pyramid level `level` of frame `frame` of the last extraction (orb_debug_level_image)."""
        w, h = ctypes.c_int(), ctypes.c_int()
        check(lib().orb_debug_level_image(self.h, frame, level, None, ctypes.byref(w), ctypes.byref(h)),
              "orb_debug_level_image")
        out = np.zeros((h.value, w.value), np.uint8)
        check(lib().orb_debug_level_image(self.h, frame, level, _p(out), ctypes.byref(w), ctypes.byref(h)),
              "orb_debug_level_image")
        return out

    def debug_level_keypoints(self, level, frame=0):
        out = np.zeros((1 << 15, 3), np.int32)
        n = lib().orb_debug_level_keypoints(self.h, frame, level, _p(out), len(out))
        if n < 0:
            raise OrbError(n, "orb_debug_level_keypoints")
        return out[:n]


class ORBextractor(_Ctx):
    """ORB_SLAM2::ORBextractor (ORBextractor.cc:410-470, 1043-1132) on one MI355X.  `variant` selects the
    OpenCV arithmetic the reference build links (VARIANT_* bits; 0 = the pinned OpenCV 3.2 default)."""

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device=0, variant=0):
        super().__init__(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device, variant=variant)
        n = nlevels
        self._t = [np.zeros(n, np.float32) for _ in range(4)]
        self._npl = np.zeros(n, np.int32)
        self._umax = np.zeros(16, np.int32)
        check(lib().orb_scale_tables(self.h, *[_p(a) for a in self._t], _p(self._npl), _p(self._umax)),
              "orb_scale_tables")
        self._last_shape = None

    # getters (ORBextractor.h:63-83)
    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return float(self.params.scaleFactor)

    def GetScaleFactors(self):
        return self._t[0].copy()

    def GetInverseScaleFactors(self):
        return self._t[1].copy()

    def GetScaleSigmaSquares(self):
        return self._t[2].copy()

    def GetInverseScaleSigmaSquares(self):
        return self._t[3].copy()

    @property
    def mnFeaturesPerLevel(self):
        return self._npl.copy()

    @property
    def umax(self):
        return self._umax.copy()

    def __call__(self, image, mask=None, keypoints=None, descriptors=None):
        """operator()(image, mask, keypoints, descriptors): returns (keypoints, descriptors).

        An empty image returns the given outputs untouched (ORBextractor.cc:1046-1047); mask is
        ignored as in the reference (ORBextractor.h:58)."""
        img = np.asarray(image)
        if img.size == 0:
            return keypoints, descriptors
        assert img.dtype == np.uint8 and img.ndim == 2, "CV_8UC1 expected (ORBextractor.cc:1050)"
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = 4 * max(self.params.nfeatures, 1) + 256
        while True:
            kps = np.zeros(cap, KP_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = ctypes.c_int(0)
            st = lib().orb_extract(self.h, _p(img), w, h, img.strides[0], _p(kps), cap, ctypes.byref(n),
                                   _p(desc))
            if st == -3:
                cap = n.value
                continue
            check(st, "orb_extract")
            break
        self._last_shape = (h, w)
        return kps[:n.value].copy(), desc[:n.value].copy()

    @property
    def mvImagePyramid(self):
        """Host views of the last frame's pyramid levels (ORBextractor.h:85)."""
        out = []
        for l in range(self.nlevels):
            ptr, w, h, stride = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int(), ctypes.c_size_t()
            check(lib().orb_get_level(self.h, l, ctypes.byref(ptr), ctypes.byref(w), ctypes.byref(h),
                                      ctypes.byref(stride)), "orb_get_level")
            buf = (ctypes.c_uint8 * (stride.value * h.value)).from_address(ptr.value)
            out.append(np.ctypeslib.as_array(buf).reshape(h.value, stride.value)[:, :w.value].copy())
        return out

class BatchExtractor(_Ctx):
    """Device-resident batched extraction (orb_extract_batch_device): frames already in HBM."""

    def __init__(self, nfeatures, width, height, batch, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7,
                 device=0, variant=0):
        super().__init__(nfeatures, scale_factor, nlevels, ini_th, min_th, device, width, height, batch, variant)
        self.w, self.hgt, self.batch = width, height, batch
        self.kp_cap = lib().orb_batch_kp_cap(self.h, width, height)
        if self.kp_cap < 0:
            raise OrbError(self.kp_cap, "orb_batch_kp_cap")
        self.pitch = width
        self.d_frames = self._alloc(batch * width * height)
        self.d_kps = self._alloc(batch * self.kp_cap * 28)
        self.d_desc = self._alloc(batch * self.kp_cap * 32)
        self.d_counts = self._alloc(batch * 4)

    def _alloc(self, nbytes):
        p = lib().orb_device_alloc(self.h, nbytes)
        if not p:
            raise OrbError(-5, "orb_device_alloc")
        return p

    def upload(self, frames):
        frames = np.ascontiguousarray(frames, np.uint8)
        assert frames.shape == (self.batch, self.hgt, self.w)
        check(lib().orb_memcpy_h2d(self.h, self.d_frames, _p(frames), frames.nbytes), "h2d")

    def launch(self, nframes=None):
        n = self.batch if nframes is None else nframes
        check(lib().orb_extract_batch_device(self.h, self.d_frames, n, self.w, self.hgt, self.w * self.hgt,
                                             self.w, self.d_kps, self.d_desc, self.d_counts, self.kp_cap),
              "orb_extract_batch_device")

    def sync(self):
        check(lib().orb_sync(self.h), "orb_sync")

    def counts(self):
        out = np.zeros(self.batch, np.int32)
        check(lib().orb_memcpy_d2h(self.h, _p(out), self.d_counts, out.nbytes), "d2h")
        return out

    def results(self, frame):
        n = int(self.counts()[frame])
        kps = np.zeros(self.kp_cap, KP_DTYPE)
        desc = np.zeros((self.kp_cap, 32), np.uint8)
        check(lib().orb_memcpy_d2h(self.h, _p(kps), self.d_kps + frame * self.kp_cap * 28, kps.nbytes), "d2h")
        check(lib().orb_memcpy_d2h(self.h, _p(desc), self.d_desc + frame * self.kp_cap * 32, desc.nbytes), "d2h")
        return kps[:n], desc[:n]

    def profile(self, on=True):
        check(lib().orb_profile_enable(self.h, int(on)), "orb_profile_enable")

    def profile_read(self):
        ms = np.zeros(7, np.float64)   # ORB_K_COUNT
        n = np.zeros(7, np.int32)
        check(lib().orb_profile_read(self.h, _p(ms), _p(n)), "orb_profile_read")
        return ms, n

    def stereo(self, npairs, mb, mbf, d_uright, d_depth, d_nmatched):
        """Frame::ComputeStereoMatches for frame pairs (2p, 2p+1) of the last launch, on the device."""
        check(lib().orb_stereo_batch_device(self.h, npairs, mb, mbf, d_uright, d_depth, d_nmatched),
              "orb_stereo_batch_device")

    def hamming_top2_frames(self, q_frames, t_frames, d_best, d_idx, d_second):
        """All-pairs top-2 between frames q_frames[p] and t_frames[p] of the last launch, one launch."""
        qf = np.ascontiguousarray(q_frames, np.int32)
        tf = np.ascontiguousarray(t_frames, np.int32)
        check(lib().orb_hamming_top2_frames_device(self.h, self.d_desc, self.d_counts, self.kp_cap, len(qf), _p(qf),
                                                   _p(tf), d_best, d_idx, d_second), "orb_hamming_top2_frames_device")

    def hamming_top2(self, d_q, nq, d_t, nt, d_best, d_idx, d_second):
        check(lib().orb_hamming_top2_device(self.h, d_q, nq, d_t, nt, d_best, d_idx, d_second),
              "orb_hamming_top2_device")

    def close(self):
        if getattr(self, "h", None):
            for p in ("d_frames", "d_kps", "d_desc", "d_counts"):
                if getattr(self, p, None):
                    lib().orb_device_free(self.h, getattr(self, p))
                    setattr(self, p, None)
        super().close()


def _featvec(fv):
    """dict {node_id: [indices]} (DBoW2::FeatureVector) -> (OrbFeatVec, keepalive)."""
    ids = np.array(sorted(fv.keys()), np.uint32)
    groups = [np.asarray(fv[int(k)], np.int32) for k in ids]
    off = np.zeros(len(groups) + 1, np.int32)
    if groups:
        off[1:] = np.cumsum([len(g) for g in groups])
    idx = np.ascontiguousarray(np.concatenate(groups) if groups else np.zeros(1, np.int32), np.int32)
    s = OrbFeatVec(len(ids), ids.ctypes.data if len(ids) else None, off.ctypes.data, idx.ctypes.data)
    return s, (ids, off, idx)


def compute_stereo_matches(left, right, kpsL, descL, kpsR, descR, mb, mbf):
    """Frame::ComputeStereoMatches (Frame.cc:662-836): left / right are the ORBextractors that
    extracted the rectified left / right images last.  Returns (mvuRight, mvDepth, n_with_depth)."""
    kl = np.ascontiguousarray(kpsL, KP_DTYPE)
    kr = np.ascontiguousarray(kpsR, KP_DTYPE)
    dl = np.ascontiguousarray(descL, np.uint8)
    dr = np.ascontiguousarray(descR, np.uint8)
    u = np.zeros(max(len(kl), 1), np.float32)
    d = np.zeros(max(len(kl), 1), np.float32)
    n = ctypes.c_int(0)
    check(lib().orb_compute_stereo_matches(left.h, right.h, len(kl), _p(kl), _p(dl), len(kr), _p(kr), _p(dr), mb, mbf,
                                           _p(u), _p(d), ctypes.byref(n)), "orb_compute_stereo_matches")
    return u[:len(kl)], d[:len(kl)], n.value


def features_in_area(kps_un, min_x, max_x, min_y, max_y, x, y, r, min_level=-1, max_level=-1):
    """Frame::GetFeaturesInArea (Frame.cc:494-547) over the 64x48 grid."""
    k = np.ascontiguousarray(kps_un, KP_DTYPE)
    out = np.zeros(max(1, len(k)), np.int32)
    n = lib().orb_features_in_area(len(k), _p(k), min_x, max_x, min_y, max_y, x, y, r, min_level, max_level,
                                   _p(out), len(out))
    return out[:n]


def frame_grid(kps_un, min_x, max_x, min_y, max_y):
    """Frame::AssignFeaturesToGrid (Frame.cc:378-393, PosInGrid :549-559) as the C-ABI's orb_frame_grid
    CSR: cell (ix, iy) holds its keypoint indices in order at cell_idx[cell_off[ix*48+iy] ..].  Returns
    (inv_w, inv_h, cell_off, cell_idx) with the float32 arithmetic of the reference."""
    k = np.asarray(kps_un, KP_DTYPE)
    f32 = np.float32
    inv_w = f32(64) / (f32(max_x) - f32(min_x))
    inv_h = f32(48) / (f32(max_y) - f32(min_y))
    vx = ((k["x"].astype(f32) - f32(min_x)) * inv_w).astype(np.float64)
    vy = ((k["y"].astype(f32) - f32(min_y)) * inv_h).astype(np.float64)
    px = (np.sign(vx) * np.floor(np.abs(vx) + 0.5)).astype(np.int64)   # std::round: half away from zero
    py = (np.sign(vy) * np.floor(np.abs(vy) + 0.5)).astype(np.int64)
    ok = (px >= 0) & (px < 64) & (py >= 0) & (py < 48)
    cell = np.where(ok, px * 48 + py, -1)
    order = np.argsort(np.where(ok, cell, 1 << 30), kind="stable")[: int(ok.sum())]
    off = np.zeros(64 * 48 + 1, np.int32)
    np.add.at(off, cell[ok] + 1, 1)
    return float(inv_w), float(inv_h), np.cumsum(off).astype(np.int32), order.astype(np.int32)


class ORBmatcher:
    """ORB_SLAM2::ORBmatcher's descriptor matchers (ORBmatcher.cc) on the GPU."""

    _shared_ctx = {}

    def __init__(self, nnratio=0.6, checkOri=True, device=0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        key = device
        if key not in ORBmatcher._shared_ctx:   # matchers are stack objects in the reference: share a context
            ORBmatcher._shared_ctx[key] = _Ctx(1000, 1.2, 8, 20, 7, device)
        self._ctx = ORBmatcher._shared_ctx[key]

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return lib().orb_descriptor_distance(_p(a), _p(b))

    def hamming_topk(self, q, t, k=2, cand_off=None, cand_idx=None, train_thr=None):
        q = np.ascontiguousarray(q, np.uint8)
        t = np.ascontiguousarray(t, np.uint8)
        nq = len(q)
        dist = np.zeros((nq, k), np.int32)
        idx = np.zeros((nq, k), np.int32)
        nv = np.zeros(nq, np.int32)
        co = None if cand_off is None else np.ascontiguousarray(cand_off, np.int32)
        cx = None if cand_idx is None else np.ascontiguousarray(cand_idx, np.int32)
        th = None if train_thr is None else np.ascontiguousarray(train_thr, np.int32)
        check(lib().orb_hamming_topk(self._ctx.h, _p(q), nq, _p(t), len(t), _p(co), _p(cx), _p(th), k,
                                     _p(dist), _p(idx), _p(nv)), "orb_hamming_topk")
        return dist, idx, nv

    def SearchByBoW_KF_F(self, desc_kf, angle_kf, mp_kf, featvec_kf, desc_f, angle_f, featvec_f):
        """SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (ORBmatcher.cc:159-288).
        Returns (nmatches, match_f) with match_f[iF] = KF feature index or -1."""
        fa, ka = _featvec(featvec_kf)
        fb, kb = _featvec(featvec_f)
        a = [np.ascontiguousarray(x) for x in (desc_kf, np.asarray(angle_kf, np.float32),
                                                np.asarray(mp_kf, np.uint8), desc_f,
                                                np.asarray(angle_f, np.float32))]
        out = np.full(len(a[3]), -1, np.int32)
        nm = ctypes.c_int()
        check(lib().orb_search_by_bow_kf_f(self._ctx.h, self.mfNNratio, int(self.mbCheckOrientation), len(a[0]),
                                           _p(a[0]), _p(a[1]), _p(a[2]), fa, len(a[3]), _p(a[3]), _p(a[4]), fb,
                                           _p(out), ctypes.byref(nm)), "SearchByBoW(KF,F)")
        return nm.value, out

    def SearchByBoW_KF_KF(self, desc1, angle1, mp1, featvec1, desc2, angle2, mp2, featvec2):
        """SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (ORBmatcher.cc:522-655)."""
        fa, ka = _featvec(featvec1)
        fb, kb = _featvec(featvec2)
        a = [np.ascontiguousarray(x) for x in (desc1, np.asarray(angle1, np.float32), np.asarray(mp1, np.uint8),
                                                desc2, np.asarray(angle2, np.float32), np.asarray(mp2, np.uint8))]
        out = np.full(len(a[0]), -1, np.int32)
        nm = ctypes.c_int()
        check(lib().orb_search_by_bow_kf_kf(self._ctx.h, self.mfNNratio, int(self.mbCheckOrientation), len(a[0]),
                                            _p(a[0]), _p(a[1]), _p(a[2]), fa, len(a[3]), _p(a[3]), _p(a[4]),
                                            _p(a[5]), fb, _p(out), ctypes.byref(nm)), "SearchByBoW(KF,KF)")
        return nm.value, out

    def _bow_entries(self, kfs, nout):
        """(ctypes array of orb_bow_kf, outputs, counts, keepalive) for dicts {desc, angle, mp, featvec}."""
        from ._lib import OrbBowKf
        arr, outs, counts, keep = (OrbBowKf * max(len(kfs), 1))(), [], [], []
        for p, k in enumerate(kfs):
            f, kf = _featvec(k["featvec"])
            a = [np.ascontiguousarray(x) for x in (k["desc"], np.asarray(k["angle"], np.float32),
                                                    np.asarray(k["mp"], np.uint8))]
            out = np.full(max(nout, 1), -1, np.int32)
            n = ctypes.c_int()
            keep += [kf, a, out, n]
            outs.append(out[:nout])
            counts.append(n)
            arr[p] = OrbBowKf(len(a[0]), _p(a[0]), _p(a[1]), _p(a[2]), f, _p(out), ctypes.pointer(n))
        return arr, outs, counts, keep

    def SearchByBoW_KF_F_batch(self, kfs, desc_f, angle_f, featvec_f):
        """orb_search_by_bow_kf_f_batch: SearchByBoW(pKF, F) for every keyframe of kfs (dicts with desc, angle, mp,
        featvec) in one call (Tracking::Relocalization's candidate loop, Tracking.cc:1931-1938).  Returns a list of
        (nmatches, match_f), each equal to SearchByBoW_KF_F's."""
        fb, kb = _featvec(featvec_f)
        d = np.ascontiguousarray(desc_f)
        ang = np.ascontiguousarray(angle_f, np.float32)
        arr, outs, counts, keep = self._bow_entries(kfs, len(d))
        check(lib().orb_search_by_bow_kf_f_batch(self._ctx.h, self.mfNNratio, int(self.mbCheckOrientation), len(d),
                                                 _p(d), _p(ang), fb, len(kfs), ctypes.cast(arr, ctypes.c_void_p)),
              "SearchByBoW(KF,F) batch")
        return [(n.value, o) for n, o in zip(counts, outs)]

    def SearchByBoW_KF_KF_batch(self, desc1, angle1, mp1, featvec1, kf2s):
        """orb_search_by_bow_kf_kf_batch: SearchByBoW(KF1, pKF2) for every KF2 of kf2s (dicts with desc, angle, mp,
        featvec) in one call (LoopClosing::ComputeSim3's candidate loop, LoopClosing.cc:252-265).  Returns a list
        of (nmatches, match12), each equal to SearchByBoW_KF_KF's."""
        fa, ka = _featvec(featvec1)
        a = [np.ascontiguousarray(x) for x in (desc1, np.asarray(angle1, np.float32), np.asarray(mp1, np.uint8))]
        arr, outs, counts, keep = self._bow_entries(kf2s, len(a[0]))
        check(lib().orb_search_by_bow_kf_kf_batch(self._ctx.h, self.mfNNratio, int(self.mbCheckOrientation),
                                                  len(a[0]), _p(a[0]), _p(a[1]), _p(a[2]), fa, len(kf2s),
                                                  ctypes.cast(arr, ctypes.c_void_p)), "SearchByBoW(KF,KF) batch")
        return [(n.value, o) for n, o in zip(counts, outs)]

    def SearchForTriangulation(self, desc1, kps1, has_mp1, uright1, featvec1, desc2, kps2, has_mp2, uright2,
                               featvec2, F12, ex, ey, scale_factors2, level_sigma2_2, bOnlyStereo=False):
        """SearchForTriangulation (ORBmatcher.cc:657-823). Returns an (n, 2) array of (idx1, idx2)."""
        fa, ka = _featvec(featvec1)
        fb, kb = _featvec(featvec2)
        a = [np.ascontiguousarray(x) for x in (desc1, np.asarray(kps1, KP_DTYPE), np.asarray(has_mp1, np.uint8),
                                                np.asarray(uright1, np.float32), desc2, np.asarray(kps2, KP_DTYPE),
                                                np.asarray(has_mp2, np.uint8), np.asarray(uright2, np.float32),
                                                np.asarray(F12, np.float32).reshape(9),
                                                np.asarray(scale_factors2, np.float32),
                                                np.asarray(level_sigma2_2, np.float32))]
        cap = len(a[0]) + 1
        pairs = np.zeros((cap, 2), np.int32)
        n = ctypes.c_int()
        check(lib().orb_search_for_triangulation(self._ctx.h, int(self.mbCheckOrientation), int(bOnlyStereo),
                                                 len(a[0]), _p(a[0]), _p(a[1]), _p(a[2]), _p(a[3]), fa, len(a[4]),
                                                 _p(a[4]), _p(a[5]), _p(a[6]), _p(a[7]), fb, _p(a[8]), ex, ey,
                                                 _p(a[9]), _p(a[10]), len(a[9]), _p(pairs), cap, ctypes.byref(n)),
              "SearchForTriangulation")
        return pairs[:n.value]

    def SearchForTriangulationBatch(self, desc1, kps1, has_mp1, uright1, featvec1, others, bOnlyStereo=False):
        """orb_search_for_triangulation_batch: KF1 against several KF2s in one call (LocalMapping.cc:247-278's
        loop).  others: a list of dicts with the single call's KF2 arguments (desc2, kps2, has_mp2, uright2,
        featvec2, F12, ex, ey, scale_factors2, level_sigma2_2).  Returns one (n, 2) array per KF2, each equal to
        SearchForTriangulation's for the same inputs."""
        from ._lib import OrbTriPair
        fa, ka = _featvec(featvec1)
        a = [np.ascontiguousarray(x) for x in (desc1, np.asarray(kps1, KP_DTYPE), np.asarray(has_mp1, np.uint8),
                                                np.asarray(uright1, np.float32))]
        keep, arr, outs, counts = [ka, a], (OrbTriPair * max(len(others), 1))(), [], []
        for p, o in enumerate(others):
            fb, kb = _featvec(o["featvec2"])
            b = [np.ascontiguousarray(x) for x in (o["desc2"], np.asarray(o["kps2"], KP_DTYPE),
                                                    np.asarray(o["has_mp2"], np.uint8), np.asarray(o["uright2"], np.float32),
                                                    np.asarray(o["F12"], np.float32).reshape(9),
                                                    np.asarray(o["scale_factors2"], np.float32),
                                                    np.asarray(o["level_sigma2_2"], np.float32))]
            cap = len(a[0]) + 1
            out = np.zeros((cap, 2), np.int32)
            n = ctypes.c_int()
            keep += [kb, b, out, n]
            outs.append(out)
            counts.append(n)
            arr[p] = OrbTriPair(len(b[0]), _p(b[0]), _p(b[1]), _p(b[2]), _p(b[3]), fb, _p(b[4]), float(o["ex"]),
                                float(o["ey"]), _p(b[5]), _p(b[6]), len(b[5]), _p(out), cap, ctypes.pointer(n))
        check(lib().orb_search_for_triangulation_batch(self._ctx.h, int(self.mbCheckOrientation), int(bOnlyStereo),
                                                       len(a[0]), _p(a[0]), _p(a[1]), _p(a[2]), _p(a[3]), fa,
                                                       len(others), ctypes.cast(arr, ctypes.c_void_p)),
              "SearchForTriangulationBatch")
        return [out[:n.value] for out, n in zip(outs, counts)]

    def _window(self, level0_only, desc1, kps1, desc2, kps2, cand_off, cand_idx):
        a = [np.ascontiguousarray(x) for x in (desc1, np.asarray(kps1, KP_DTYPE), desc2, np.asarray(kps2, KP_DTYPE),
                                                np.asarray(cand_off, np.int32), np.asarray(cand_idx, np.int32))]
        if len(a[5]) == 0:
            a[5] = np.zeros(1, np.int32)
        out = np.full(len(a[0]), -1, np.int32)
        nm = ctypes.c_int()
        check(lib().orb_window_match(self._ctx.h, self.mfNNratio, int(self.mbCheckOrientation), int(level0_only),
                                     len(a[0]), _p(a[0]), _p(a[1]), len(a[2]), _p(a[2]), _p(a[3]), _p(a[4]),
                                     _p(a[5]), _p(out), ctypes.byref(nm)), "window match")
        return nm.value, out

    def window_match_grid(self, level0_only, desc1, kps1, desc2, kps2, grid, window, centres=None, min_xy=(0.0, 0.0)):
        """orb_window_match_grid: the window searches with GetFeaturesInArea on the device over F2's grid
        (frame_grid(...)); centres: (n1, 2) float32 window centres or None = kps1 positions."""
        inv_w, inv_h, off, idx = grid
        a = [np.ascontiguousarray(x) for x in (desc1, np.asarray(kps1, KP_DTYPE), desc2, np.asarray(kps2, KP_DTYPE))]
        cen = None if centres is None else np.ascontiguousarray(centres, np.float32).reshape(-1, 2)
        idx = idx if len(idx) else np.zeros(1, np.int32)
        g = OrbFrameGrid(float(min_xy[0]), float(min_xy[1]), inv_w, inv_h, off.ctypes.data, idx.ctypes.data)
        out = np.full(max(len(a[0]), 1), -1, np.int32)
        nm = ctypes.c_int()
        check(lib().orb_window_match_grid(self._ctx.h, self.mfNNratio, int(self.mbCheckOrientation), int(level0_only),
                                          len(a[0]), _p(a[0]), _p(a[1]), _p(cen), float(window), len(a[2]), _p(a[2]),
                                          _p(a[3]), g, _p(out), ctypes.byref(nm)), "window match (grid)")
        return nm.value, out[:len(a[0])]

    def SearchForInitialization(self, desc1, kps1, desc2, kps2, cand_off, cand_idx):
        """SearchForInitialization (ORBmatcher.cc:405-520); candidates = F2.GetFeaturesInArea per query.
        Returns (nmatches, vnMatches12)."""
        return self._window(True, desc1, kps1, desc2, kps2, cand_off, cand_idx)

    def ComputeDistinctiveDescriptors(self, descriptor_sets):
        """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:242-307) for a batch of map points:
        descriptor_sets[m] = (n_m, 32) descriptors of point m's observations.  Returns the index of the
        chosen descriptor per point (-1 for an empty set)."""
        sets = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in descriptor_sets]
        off = np.zeros(len(sets) + 1, np.int32)
        off[1:] = np.cumsum([len(d) for d in sets])
        allv = np.ascontiguousarray(np.concatenate(sets) if off[-1] else np.zeros((1, 32), np.uint8))
        out = np.zeros(max(len(sets), 1), np.int32)
        check(lib().orb_distinctive_descriptors(self._ctx.h, len(sets), _p(off), _p(allv), _p(out)),
              "orb_distinctive_descriptors")
        return out[:len(sets)]

    def BirdviewMatch(self, desc1, kps1, desc2, kps2, cand_off, cand_idx):
        """BirdviewMatch(const Frame&, const Frame&, vector<int>&, int) (ORBmatcher.cc:1790-1899)."""
        return self._window(False, desc1, kps1, desc2, kps2, cand_off, cand_idx)


class ORBVocabulary:
    """DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (include/ORBVocabulary.h:32) on the GPU:
    loadFromBinaryFile (TemplatedVocabulary.h:1466-1510) and transform(features, BowVector&,
    FeatureVector&, levelsup) (:1139-1210).  BowVector -> {word: value}, FeatureVector -> {node: [i]}."""

    def __init__(self, device=0):
        self._ctx = _Ctx(1000, 1.2, 8, 20, 7, device)
        self.v = None

    def loadFromBinaryFile(self, path):
        if self.v:
            lib().orb_vocab_destroy(self.v)
            self.v = None
        out = ctypes.c_void_p()
        check(lib().orb_vocab_load(self._ctx.h, path.encode(), ctypes.byref(out)), "orb_vocab_load")
        self.v = out
        vals = [ctypes.c_int() for _ in range(6)]
        check(lib().orb_vocab_info(self.v, *[ctypes.byref(x) for x in vals]), "orb_vocab_info")
        self.k, self.L, self.scoring, self.weighting, self.nnodes, self.nwords = [x.value for x in vals]
        return True

    def transform_each(self, desc, levelsup=4):
        """Per-feature (word id, weight, node id levelsup above the leaf)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        w = np.zeros(max(n, 1), np.int32)
        wt = np.zeros(max(n, 1), np.float32)
        nd = np.zeros(max(n, 1), np.uint32)
        check(lib().orb_vocab_transform(self._ctx.h, self.v, _p(d), n, levelsup, _p(w), _p(wt), _p(nd)),
              "orb_vocab_transform")
        return w[:n], wt[:n], nd[:n]

    def bow(self, word, weight, node):
        n = len(word)
        bw = np.zeros(max(n, 1), np.int32)
        bv = np.zeros(max(n, 1), np.float64)
        fn = np.zeros(max(n, 1), np.uint32)
        fo = np.zeros(n + 1, np.int32)
        fi = np.zeros(max(n, 1), np.int32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        args = [np.ascontiguousarray(word, np.int32), np.ascontiguousarray(weight, np.float32),
                np.ascontiguousarray(node, np.uint32)]
        check(lib().orb_vocab_bow(self.v, n, *[_p(a) for a in args], _p(bw), _p(bv), ctypes.byref(nb), _p(fn),
                                  _p(fo), _p(fi), ctypes.byref(nf)), "orb_vocab_bow")
        bowv = {int(bw[i]): float(bv[i]) for i in range(nb.value)}
        fv = {int(fn[j]): fi[fo[j]:fo[j + 1]].tolist() for j in range(nf.value)}
        return bowv, fv

    def transform(self, desc, levelsup=4):
        """transform(features, BowVector&, FeatureVector&, levelsup) -> (bow, featvec)."""
        return self.bow(*self.transform_each(desc, levelsup))

    def close(self):
        if getattr(self, "v", None):
            lib().orb_vocab_destroy(self.v)
            self.v = None

    def __del__(self):
        self.close()


class BirdORB:
    """cv::ORB as the birdview stream uses it (Frame.cc:329: ORB::create(2000) -> nfeatures 2000,
    scaleFactor 1.2, nlevels 8, edgeThreshold 31, HARRIS_SCORE, patchSize 31, fastThreshold 20),
    plus cornerSubPix and the fused Frame.cc:320-342 sequence, on one MI355X (orb_bird_* C-ABI)."""

    def __init__(self, nfeatures=2000, scaleFactor=1.2, nlevels=8, edgeThreshold=31, fastThreshold=20, device=0,
                 variant=0):
        self.params = OrbBirdParams(nfeatures, scaleFactor, nlevels, edgeThreshold, fastThreshold, device, variant)
        st = ctypes.c_int()
        self.h = lib().orb_bird_create(ctypes.byref(self.params), ctypes.byref(st))
        if not self.h:
            raise OrbError(st.value, "orb_bird_create")
        self.nlevels = nlevels

    def close(self):
        if getattr(self, "h", None):
            lib().orb_bird_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    @staticmethod
    def _img(image):
        img = np.asarray(image)
        assert img.dtype == np.uint8 and img.ndim == 2, "CV_8UC1 expected"
        return np.ascontiguousarray(img)

    def detect(self, image, mask=None):
        """cv::ORB::detect(image, keypoints, mask) -> keypoints (KP_DTYPE)."""
        img = self._img(image)
        if img.size == 0:
            return np.zeros(0, KP_DTYPE)
        h, w = img.shape
        m = None if mask is None else self._img(mask)
        cap = 2 * max(self.params.nfeatures, 1) + 256
        while True:
            kps = np.zeros(cap, KP_DTYPE)
            n = ctypes.c_int(0)
            st = lib().orb_bird_detect(self.h, _p(img), w, h, img.strides[0], _p(m), w if m is None else m.strides[0],
                                       _p(kps), cap, ctypes.byref(n))
            if st == -3:
                cap = n.value
                continue
            check(st, "orb_bird_detect")
            return kps[:n.value].copy()

    def compute(self, image, keypoints):
        """cv::ORB::compute(image, keypoints, descriptors) -> (keypoints, descriptors); keypoints are
        border-culled and level-sorted as the reference does in place."""
        img = self._img(image)
        k = np.ascontiguousarray(keypoints, KP_DTYPE).copy()
        if img.size == 0:
            return k, np.zeros((0, 32), np.uint8)
        h, w = img.shape
        desc = np.zeros((max(len(k), 1), 32), np.uint8)
        n = ctypes.c_int(len(k))
        check(lib().orb_bird_compute(self.h, _p(img), w, h, img.strides[0], _p(k) if len(k) else None,
                                     ctypes.byref(n), _p(desc)), "orb_bird_compute")
        return k[:n.value].copy(), desc[:n.value].copy()

    def cornerSubPix(self, image, corners, winSize=(5, 5), maxCount=40, epsilon=0.001):
        img = self._img(image)
        h, w = img.shape
        p = np.ascontiguousarray(corners, np.float32).reshape(-1, 2).copy()
        check(lib().orb_corner_subpix(self.h, _p(img), w, h, img.strides[0], _p(p), len(p), winSize[0], winSize[1],
                                      maxCount, epsilon), "orb_corner_subpix")
        return p

    def extract(self, image, mask=None):
        """Frame.cc:320-342 fused: footprint-masked detect, cornerSubPix(5x5, 40, 0.001), compute."""
        img = self._img(image)
        if img.size == 0:
            return np.zeros(0, KP_DTYPE), np.zeros((0, 32), np.uint8)
        h, w = img.shape
        m = None if mask is None else self._img(mask)
        cap = 2 * max(self.params.nfeatures, 1) + 256
        while True:
            kps = np.zeros(cap, KP_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = ctypes.c_int(0)
            st = lib().orb_bird_extract(self.h, _p(img), w, h, img.strides[0], _p(m), w if m is None else m.strides[0],
                                        _p(kps), cap, ctypes.byref(n), _p(desc))
            if st == -3:
                cap = n.value
                continue
            check(st, "orb_bird_extract")
            return kps[:n.value].copy(), desc[:n.value].copy()

    def extract_device(self, d_img, w, h, d_mask=None, cap=None):
        """Fused extract on a device-resident image (and mask) — device pointers as ints."""
        cap = cap or 2 * max(self.params.nfeatures, 1) + 256
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int(0)
        check(lib().orb_bird_extract_device(self.h, ctypes.c_void_p(d_img), w, h, w,
                                            None if d_mask is None else ctypes.c_void_p(d_mask), w, _p(kps), cap,
                                            ctypes.byref(n), _p(desc)), "orb_bird_extract_device")
        return kps[:n.value], desc[:n.value]

    def debug_candidates(self, level):
        cap = 1 << 16
        while True:
            out = np.zeros(cap, KP_DTYPE)
            n = lib().orb_bird_debug_candidates(self.h, level, _p(out), cap)
            if n >= 0:
                return out[:n]
            if n < -1:
                cap = -n - 1
                continue
            check(n, "orb_bird_debug_candidates")

    def debug_level(self, level):
        w, h = ctypes.c_int(), ctypes.c_int()
        check(lib().orb_bird_debug_level(self.h, level, None, ctypes.byref(w), ctypes.byref(h)), "debug_level")
        out = np.zeros((h.value, w.value), np.uint8)
        check(lib().orb_bird_debug_level(self.h, level, _p(out), ctypes.byref(w), ctypes.byref(h)), "debug_level")
        return out


def cornerSubPix(image, corners, winSize=(5, 5), maxCount=40, epsilon=0.001, device=0):
    """cv::cornerSubPix(image, corners, winSize, Size(-1,-1), TermCriteria(EPS+MAX_ITER, maxCount, epsilon))."""
    b = BirdORB(device=device)
    try:
        return b.cornerSubPix(image, corners, winSize, maxCount, epsilon)
    finally:
        b.close()


def bird_footprint_mask(mask):
    """Frame.cc:320-327: copy of `mask` with the vehicle footprint (+15 px) zeroed (host helper)."""
    m = np.ascontiguousarray(mask, np.uint8).copy()
    h, w = m.shape
    check(lib().orb_bird_footprint_mask(_p(m), w, h, m.strides[0]), "orb_bird_footprint_mask")
    return m

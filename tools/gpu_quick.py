"""Stage-by-stage GPU vs oracle comparison (diagnostic; not part of the test suite)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402
import orbgpu  # noqa: E402
from orbgpu.synth import synth_frame  # noqa: E402


def compare(w, h, nfeat, idx=0, kind="scene"):
    img = synth_frame(w, h, idx, kind)
    o = oracle.OracleExtractor(nfeat)
    ok_k, ok_d = o(img)
    g = orbgpu.ORBextractor(nfeat, 1.2, 8, 20, 7)
    t0 = time.time()
    gk, gd = g(img)
    t1 = time.time()
    print(f"== {w}x{h} nfeat={nfeat} kind={kind} idx={idx}: oracle {len(ok_k)} gpu {len(gk)} ({(t1-t0)*1e3:.1f} ms)")
    pyr = g.mvImagePyramid
    bad = False
    for l in range(8):
        ol = o.level(l)
        if ol.shape != pyr[l].shape or not np.array_equal(ol, pyr[l]):
            diff = np.argwhere(ol != pyr[l]) if ol.shape == pyr[l].shape else "shape"
            print(f"  level {l} pyramid MISMATCH {ol.shape} {pyr[l].shape} {diff[:5] if not isinstance(diff, str) else diff}")
            bad = True
            continue
        oc = o.candidates(l)
        gc = g.debug_candidates(l)
        if oc.shape != gc.shape or not np.array_equal(oc, gc):
            print(f"  level {l} candidates MISMATCH oracle {len(oc)} gpu {len(gc)}")
            n = min(len(oc), len(gc))
            d = np.argwhere((oc[:n] != gc[:n]).any(1))
            if len(d):
                i = d[0][0]
                print("   first diff at", i, oc[max(0, i-2):i+3].tolist(), gc[max(0, i-2):i+3].tolist())
            bad = True
            continue
        ok = o.level_keypoints(l)
        gkl = g.debug_level_keypoints(l)
        okx = np.stack([ok["x"], ok["y"], ok["response"]], 1).astype(np.int32)
        if okx.shape != gkl.shape or not np.array_equal(okx, gkl):
            print(f"  level {l} octree MISMATCH oracle {len(okx)} gpu {len(gkl)}")
            n = min(len(okx), len(gkl))
            d = np.argwhere((okx[:n] != gkl[:n]).any(1))
            if len(d):
                i = d[0][0]
                print("   first diff at", i, okx[max(0, i-2):i+3].tolist(), gkl[max(0, i-2):i+3].tolist())
            bad = True
    if len(ok_k) == len(gk):
        kb = ok_k.tobytes() == gk.tobytes()
        db = np.array_equal(ok_d, gd)
        if not kb:
            for f in ok_k.dtype.names:
                m = ok_k[f] != gk[f]
                if m.any():
                    i = np.argwhere(m)[0][0]
                    print(f"  keypoint field {f} mismatches: {m.sum()} first {i}: {ok_k[i]} vs {gk[i]}")
        if not db:
            m = (ok_d != gd).any(1)
            i = np.argwhere(m)[0][0]
            print(f"  descriptors mismatch rows {m.sum()} first {i}")
        print("  keypoints bit-exact:", kb, " descriptors bit-exact:", db)
        bad |= not (kb and db)
    else:
        bad = True
    return not bad


if __name__ == "__main__":
    print("devices:", orbgpu.device_count())
    allok = True
    for (w, h, n, i, kind) in [(320, 240, 500, 0, "scene"), (640, 480, 1000, 0, "scene"), (640, 480, 1000, 1, "scene"),
                               (1280, 720, 2000, 0, "scene"), (641, 479, 1000, 2, "scene"),
                               (640, 480, 1000, 0, "flat"), (640, 480, 1000, 3, "noise"),
                               (1280, 720, 4000, 4, "scene")]:
        allok &= compare(w, h, n, i, kind)
    print("ALL OK" if allok else "SOME MISMATCH")

"""Generate tests/golden/*.npz with the oracle restatement (SURVEY §8c "Golden vectors").

The reference ships no fixtures and cannot be built here (OpenCV absent), so these vectors are
produced by the oracle and pin it against drift; inputs are regenerated from the seeded synthetic
generator and checked by sha256.  Run: python tools/gen_golden.py
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from orbgpu.synth import synth_frame  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

CASES = [("extract_320x240_500.npz", 320, 240, 500, 0, "scene"),
         ("extract_640x480_1000.npz", 640, 480, 1000, 0, "scene"),
         ("extract_noise_640x480.npz", 640, 480, 1000, 3, "noise")]


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, w, h, nf, idx, kind in CASES:
        img = synth_frame(w, h, idx, kind)
        k, d = oracle.OracleExtractor(nf)(img)
        np.savez_compressed(os.path.join(OUT, name), cfg=np.array([w, h, nf, idx]), kind=np.array(kind),
                            img_sha256=np.array(hashlib.sha256(img.tobytes()).hexdigest()), kps=k, desc=d)
        print(name, len(k))


def stereo():
    """Frame::ComputeStereoMatches on a seeded synthetic stereo pair (oracle), 640x480 / 1000 features."""
    from orbgpu.synth import synth_stereo_right
    left = synth_frame(640, 480, 3)
    right = synth_stereo_right(left, 3)
    ol, orr = oracle.OracleExtractor(1000), oracle.OracleExtractor(1000)
    kl, dl = ol(left)
    kr, dr = orr(right)
    u, d, n = oracle.stereo_matches(ol, orr, kl, dl, kr, dr, 0.12, 0.12 * 500.0)
    np.savez_compressed(os.path.join(OUT, "stereo_640x480.npz"), cfg=np.array([640, 480, 1000, 3]),
                        mb=np.float32(0.12), mbf=np.float32(0.12 * 500.0),
                        left_sha256=np.array(hashlib.sha256(left.tobytes()).hexdigest()),
                        right_sha256=np.array(hashlib.sha256(right.tobytes()).hexdigest()),
                        uright=u, depth=d, n=np.int32(n))
    print("stereo_640x480.npz", n)


if __name__ == "__main__":
    main()
    stereo()

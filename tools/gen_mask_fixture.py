"""tests/golden/mask_new_front.npz: the reference's only image, Examples/Monocular/mask_new_front.png
(1920x1208, read by mono_fisheye.cc:56 and applied by applyMask :102-108 / :202-212), reduced to the
bool array of camera pixels that stay (G channel <= 250) and bit-packed, plus the oracle's outputs on the
driver's 950x400 frame built from it (orbgpu.synth.fisheye_driver_frame, seed 0 and 5):
  * ORBextractor with fisheye.yaml's parameters (2000, 1.2, 8, 15, 5; fisheye.yaml:29-42);
  * BirdORB (cv::ORB(2000) + cornerSubPix + compute, Frame.cc:320-342) with the frame's keep mask;
and the PNG itself converted to gray (SURVEY 8(d)'s low-texture edge frame) with the oracle's extraction.
Run here (the PNG is read from /root/reference, which the GPU box does not have): python tools/gen_mask_fixture.py
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

import oracle  # noqa: E402
from orbgpu.synth import fisheye_driver_frame  # noqa: E402

PNG = "/root/reference/Examples/Monocular/mask_new_front.png"
OUT = os.path.join(ROOT, "tests", "golden", "mask_new_front.npz")
SEEDS = (0, 5)


def main():
    rgb = np.asarray(Image.open(PNG).convert("RGB"))
    keep = rgb[:, :, 1] <= 250            # applyMask: pixel[1] (G in BGR and RGB alike) > 250 -> 0
    res = {"keep_bits": np.packbits(keep, axis=1), "shape": np.array(keep.shape),
           "png_sha256": np.array(hashlib.sha256(open(PNG, "rb").read()).hexdigest())}
    for s in SEEDS:
        img, km = fisheye_driver_frame(keep, s)
        k, d = oracle.OracleExtractor(2000, 1.2, 8, 15, 5)(img)
        bk, bd = oracle.OracleCvORB(2000).extract(img, km)
        res.update({f"img_sha256_{s}": np.array(hashlib.sha256(img.tobytes()).hexdigest()),
                    f"kps_{s}": k, f"desc_{s}": d, f"bird_kps_{s}": bk, f"bird_desc_{s}": bd})
        print(s, img.shape, int((km == 0).sum()), "masked px;", len(k), "keypoints;", len(bk), "birdview keypoints")
    # SURVEY 8(d)'s low-texture edge frame: the PNG itself converted to gray as cv::cvtColor(BGR2GRAY) does
    # for 8U (fixed point: (4899 R + 9617 G + 1868 B + 2^13) >> 14), extracted at 1920x1208 with KITTI's
    # parameters (2000, 1.2, 8, 20, 7): flat regions leave most cells empty at iniThFAST (the minThFAST
    # fallback, ORBextractor.cc:812-816)
    r, g, b = (rgb[:, :, i].astype(np.int64) for i in range(3))
    gray = ((4899 * r + 9617 * g + 1868 * b + 8192) >> 14).astype(np.uint8)
    k, d = oracle.OracleExtractor(2000, 1.2, 8, 20, 7)(gray)
    res.update({"gray": gray, "kps_gray": k, "desc_gray": d})
    print("gray", gray.shape, len(k), "keypoints")
    np.savez_compressed(OUT, **res)
    print(OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()

"""Debug helper: one synthetic frame through orbgpu.ORBextractor vs the oracle, and where keypoints /
descriptors differ (field, level, position) -- for bisecting a k_describe change on the GPU box."""
import sys
import numpy as np
sys.path.insert(0, "orb-slam-birdview_amd")
sys.path.insert(0, "oracle")
import oracle
import orbgpu
from orbgpu.synth import synth_frame

w, h, nf = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (320, 240, 500)))
img = synth_frame(w, h, 0, "scene")
ok, od = oracle.OracleExtractor(nf)(img)
gk, gd = orbgpu.ORBextractor(nf, 1.2, 8, 20, 7)(img)
print("counts", len(gk), len(ok))
n = min(len(gk), len(ok))
for f in ok.dtype.names:
    bad = np.nonzero(gk[f][:n] != ok[f][:n])[0]
    print(f, "mismatches", len(bad), bad[:10])
dbad = np.nonzero((gd[:n] != od[:n]).any(1))[0]
print("descriptor rows differing", len(dbad), "of", n)
for i in dbad[:12]:
    nbits = int(np.unpackbits(gd[i] ^ od[i]).sum())
    print(" kp", i, "oct", ok["octave"][i], "x %.1f y %.1f" % (ok["x"][i], ok["y"][i]), "angle", ok["angle"][i], gk["angle"][i], "bits", nbits,
          "bytes", np.nonzero(gd[i] != od[i])[0][:16])

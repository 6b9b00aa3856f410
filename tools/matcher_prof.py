"""Kernel trace of the per-call matcher leg (tools/matcher_latency) at one frame size: writes the leg's inputs the
way bench.py's matcher_leg does (numpy only: nothing here touches the GPU), then runs rocprofv3 --kernel-trace --stats
on the C++ driver as a child process.  usage: python3 tools/matcher_prof.py <w> <h> <nfeatures> <outdir>"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
from orbgpu.synth import bench_frames, synth_stereo_right, write_synth_vocab_large  # noqa: E402

w, h, nf, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
os.makedirs(out, exist_ok=True)
a = np.ascontiguousarray(bench_frames(w, h, 1, first=0)[0])
b = np.ascontiguousarray(np.roll(a, (2, 3), axis=(0, 1)))
sr = np.ascontiguousarray(synth_stereo_right(a, 0))
raw, voc = os.path.join(out, "frames.raw"), os.path.join(out, "voc.bin")
with open(raw, "wb") as f:
    f.write(a.tobytes() + b.tobytes() + a.tobytes() + sr.tobytes())
write_synth_vocab_large(voc, 10, 6)
r = subprocess.run(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", os.path.join(out, "prof"),
                    "-o", "run", "--", os.path.join(ROOT, "tools", "matcher_latency"), raw, str(w), str(h), str(nf), voc,
                    "50", "10"], capture_output=True, text=True, timeout=300)
print(r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "", r.stderr[-500:] if r.returncode else "")
os.unlink(voc)
os.unlink(raw)
sys.exit(r.returncode)

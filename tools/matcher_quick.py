"""Run bench.py's matcher leg alone (GPU box): python3 tools/matcher_quick.py [c3|c2]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orb-slam-birdview_amd"))
import bench  # noqa: E402
from orbgpu.synth import synth_frame  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
w, h, nf = (1280, 720, 2000) if cfg == "c3" else (640, 480, 1000)
print(json.dumps(bench.matcher_leg(synth_frame(w, h, 0), w, h, nf, 0)), flush=True)

set -o pipefail
O=gpurun_out/c22; mkdir -p $O /tmp/tl; export TMPDIR=/tmp
ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_tripoll.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py -k "triangulation" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
echo "pytest (tripoll): $(tail -1 $O/pytest.log)"
python3 - <<'PY'
import sys; sys.path.insert(0, 'orb-slam-birdview_amd')
import numpy as np
from orbgpu.synth import bench_frames, synth_stereo_right, write_synth_vocab_large
a = np.ascontiguousarray(bench_frames(1280, 720, 1)[0]); b = np.ascontiguousarray(np.roll(a, (2, 3), axis=(0, 1)))
sr = np.ascontiguousarray(synth_stereo_right(a, 0))
open('/tmp/tl/frames.raw', 'wb').write(a.tobytes() + b.tobytes() + a.tobytes() + sr.tobytes())
write_synth_vocab_large('/tmp/tl/voc.bin', 10, 6)
PY
cp ab/liborbgpu_tripoll.so /tmp/tl/liborbgpu.so
for r in 1 2 3; do
  timeout -k 10 120 ./tools/matcher_latency /tmp/tl/frames.raw 1280 720 2000 /tmp/tl/voc.bin 200 20 > $O/tree$r.log 2>&1 || { echo "tree run failed"; tail $O/tree$r.log; exit 1; }
  echo "tree    $(grep -o '"SearchForTriangulation[^}]*}' $O/tree$r.log)"
  LD_LIBRARY_PATH=/tmp/tl timeout -k 10 120 ./tools/matcher_latency /tmp/tl/frames.raw 1280 720 2000 /tmp/tl/voc.bin 200 20 > $O/poll$r.log 2>&1 || { echo "poll run failed"; tail $O/poll$r.log; exit 1; }
  echo "tripoll $(grep -o '"SearchForTriangulation[^}]*}' $O/poll$r.log)"
done

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c10; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -k stripe > $O/pytest_stripe.log 2>&1; rc=$?; tail -3 $O/pytest_stripe.log; [ $rc -eq 0 ] || exit 1
$T 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_variants.py tests/test_host_mirror.py tests/test_gpu_stereo.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for K in 64 32 128; do
$T 180 env ORBGPU_STRIPES=$K python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5b1p4_$K.txt 2>&1 && echo -n "K $K p4 " && python3 -c "
import json; d=json.loads(open('$O/c5b1p4_$K.txt').read().strip().splitlines()[-1]); print(round(d['value']/1e6,1), d['ms_per_step'], d['kernels_ms_per_step'])" || exit 1
$T 180 env ORBGPU_STRIPES=$K python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/c5b1p1_$K.txt 2>&1 && echo -n "K $K p1 " && python3 -c "
import json; d=json.loads(open('$O/c5b1p1_$K.txt').read().strip().splitlines()[-1]); print(round(d['value']/1e6,1), d['ms_per_step'], d['kernels_ms_per_step'])" || exit 1
done
python3 -c "
import sys; sys.path.insert(0,'orb-slam-birdview_amd')
import numpy as np
from orbgpu.synth import bench_frames
open('/tmp/frames.raw','wb').write(np.ascontiguousarray(bench_frames(1280,720,16)).tobytes())
"
for K in 0 64; do $T 120 env ORBGPU_STRIPES=$K ./tools/host_latency /tmp/frames.raw 1280 720 16 2000 300 0 > $O/host_$K.txt 2>&1 && echo -n "host K $K " && tail -1 $O/host_$K.txt || exit 1; done

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c32; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_flow.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for v in 0 1; do
ORBGPU_FLOW=1 ORBGPU_FLOW_CHAIN=$v timeout -k 10 180 python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/c5_$v.txt 2>&1 || exit 1
python3 -c "
import json
d=json.loads(open('$O/c5_$v.txt').read().strip().splitlines()[-1]); print('chain=$v', round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done
# C5 8 frames per step: small-batch octree at 512 (tree) vs 1024 threads (ab/liborbgpu_oct1024.so)
for rep in 1 2; do for lib in tree oct1024; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  timeout -k 10 180 python bench.py --config c5 --only-extract --steps 400 > $O/c5b8_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/c5b8_$lib.txt').read().strip().splitlines()[-1]); print('$lib c5b8', round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done; done

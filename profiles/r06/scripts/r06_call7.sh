set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c15; mkdir -p $O
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_variants.py tests/test_tie_order.py tests/test_gpu_flow.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
$T 120 env ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_stamps.so python tools/octree_stamps.py 1 4000 > $O/oct_c5b1.txt 2>&1 && cat $O/oct_c5b1.txt || exit 1
$T 180 python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5b1p4.txt 2>&1 && tail -1 $O/c5b1p4.txt | cut -c100-200 &&
$T 180 python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/c5b1p1.txt 2>&1 && tail -1 $O/c5b1p1.txt | cut -c100-200 &&
$T 300 python bench.py --only-extract --steps 200 > $O/c3.txt 2>&1 && python3 -c "
import json; d=json.loads(open('$O/c3.txt').read().strip().splitlines()[-1]); print('C3', d['value']/1e6, d['kernels_ms_per_step'])"


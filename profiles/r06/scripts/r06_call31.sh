# k_resize_tiled with 64-row tiles for batches (ab/liborbgpu_rstall.so) vs 32-row (tree): parity, C3 time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c31; mkdir -p $O
ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_rstall.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_flow.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do for lib in rstall tree; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  timeout -k 10 180 python bench.py --only-extract --steps 200 > $O/c3_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/c3_$lib.txt').read().strip().splitlines()[-1]); print('$lib', round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done; done

# sincos single evaluation with VGPR quadrant selects (ab/liborbgpu_trigonce.so): determinism, parity, time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c25; mkdir -p $O
export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_trigonce.so
for rep in 1 2; do timeout -k 10 300 python -u tools/r06_desc_diag.py > $O/diag_$rep.txt 2>&1 || exit 1; grep "kps equal" $O/diag_$rep.txt; done
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_flow.py tests/test_gpu_bird.py tests/test_host_mirror.py tests/test_tie_order.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for lib in trigonce tree; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  timeout -k 10 180 python bench.py --only-extract --steps 200 > $O/c3_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/c3_$lib.txt').read().strip().splitlines()[-1]); print('$lib', round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done; done

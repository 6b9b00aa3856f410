# glibc_sincosf with each polynomial evaluated once (tree) vs twice (ab/liborbgpu_r6old.so, HEAD): parity over
# every path that rotates BRIEF (extraction, dataflow, birdview, host mirror), then C3 / C5 time.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c21; mkdir -p $O
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_flow.py tests/test_gpu_bird.py tests/test_host_mirror.py tests/test_tie_order.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for lib in tree r6old; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  $T 180 python bench.py --only-extract --steps 200 > $O/c3_$lib.txt 2>&1 || exit 1
  $T 180 python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
for f in ['$O/c3_$lib.txt','$O/c5_$lib.txt']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print('$lib', f.split('/')[-1], round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done; done

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c16; mkdir -p $O
T="timeout -k 10"
for lib in oct512 oct256; do
  $T 300 env ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -k "small_batch or c5_bench or tie or maximum" tests/test_tie_order.py > $O/pytest_$lib.log 2>&1; rc=$?; echo -n "$lib: "; tail -1 $O/pytest_$lib.log; [ $rc -eq 0 ] || exit 1
done
for rep in 1 2; do for lib in tree oct512 oct256; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  $T 180 python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/p1_$lib.txt 2>&1 || exit 1
  $T 180 python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/p4_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
for f in ['$O/p1_$lib.txt','$O/p4_$lib.txt']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print('$lib', f[-10:], round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done; done

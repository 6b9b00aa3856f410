# batched SearchForTriangulation: parity, then the matcher legs with the pinned-mirror reads (zero copy) for every
# size vs a DMA above 32 KiB / 128 KiB of staged records (ORBGPU_TRI_ZC_MAX, an A/B switch removed afterwards)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c27; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_matcher.py tests/test_matcher_adapter.py tests/test_host_mirror.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
ORBGPU_TRI_ZC_MAX=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_matcher.py -k triangulation > $O/pytest_dma.log 2>&1; rc=$?; tail -1 $O/pytest_dma.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for zc in inf 131072 32768; do
  if [ $zc = inf ]; then unset ORBGPU_TRI_ZC_MAX; else export ORBGPU_TRI_ZC_MAX=$zc; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-hamming --no-stereo --no-host-path --no-bird --no-c4 > $O/bench_$zc.txt 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/bench_$zc.txt').read().strip().splitlines()[-1])
for k in ('matcher','matcher_c2'):
    m=d.get(k) or {}
    print('$zc', k, {n:(v['gpu_us'],v['cpu_us'],v['speedup'],v['equal']) for n,v in m.items() if isinstance(v,dict) and 'gpu_us' in v and 'Triang' in n})"
done; done

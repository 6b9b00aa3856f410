# triangulation host staging into cached memory then one copy into the pinned mirror (ab/trilocal) vs writing the
# pinned mirror record by record (tree): matcher legs, C2 and C3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c30; mkdir -p $O
LD_LIBRARY_PATH=$PWD/ab/trilocal timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_matcher_adapter.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do for v in tree trilocal; do
  if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=$PWD/ab/trilocal; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-hamming --no-stereo --no-host-path --no-bird --no-c4 > $O/bench_$v.txt 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/bench_$v.txt').read().strip().splitlines()[-1])
for k in ('matcher','matcher_c2'):
    m=d.get(k) or {}
    print('$v', k, {n:(v['gpu_us'],v['speedup']) for n,v in m.items() if isinstance(v,dict) and 'gpu_us' in v and 'Tri' in n})"
done; done

# batched BoW searches: parity (matcher, adapter, host mirror), then the matcher legs with the _x10 entries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c28; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_matcher.py tests/test_matcher_adapter.py tests/test_host_mirror.py tests/test_gpu_vocab.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-hamming --no-stereo --no-host-path --no-bird --no-c4 > $O/bench_$rep.txt 2>&1 || exit 1
python3 -c "
import json
d=json.loads(open('$O/bench_$rep.txt').read().strip().splitlines()[-1])
for k in ('matcher','matcher_c2'):
    m=d.get(k) or {}
    print(k, {n:(v['gpu_us'],v['cpu_us'],v['speedup'],v['equal']) for n,v in m.items() if isinstance(v,dict) and 'gpu_us' in v})"
done

# SearchForTriangulation with ctx-owned host lists: matcher / adapter / bow-chain tests, the per-call matcher leg x2
set -o pipefail
mkdir -p gpurun_out/ab24; export TMPDIR=/tmp
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread"
$T tests/test_gpu_matcher.py tests/test_matcher_adapter.py tests/test_gpu_bow_chain.py > gpurun_out/ab24/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/ab24/pytest.log; [ $rc -eq 0 ] || exit 1
MA="--steps 5 --warmup 2 --no-cpu --no-hamming --no-stereo --no-host-path --no-bird --no-c4 --no-profile-pass"
for i in 1 2; do
  timeout -k 10 200 python3 bench.py $MA > gpurun_out/ab24/bench_matcher_$i.log 2>&1 || { tail -5 gpurun_out/ab24/bench_matcher_$i.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab24/bench_matcher_$i.log') if l.startswith('{')][-1])['matcher']; print(json.dumps({k: (v.get('gpu_us'), v.get('cpu_us'), v.get('speedup'), v.get('equal')) for k, v in d.items() if isinstance(v, dict) and 'gpu_us' in v}))"
done

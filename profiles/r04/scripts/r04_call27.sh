# SearchForTriangulation completion signal: matcher / adapter / bow-chain tests, the per-call matcher leg x2 with the
# signal (default) and x2 with ORBGPU_DONE_SIGNAL=0 (stream synchronisation), alternating
set -o pipefail
mkdir -p gpurun_out/ab27; export TMPDIR=/tmp
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread"
$T tests/test_gpu_matcher.py tests/test_matcher_adapter.py tests/test_gpu_bow_chain.py > gpurun_out/ab27/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/ab27/pytest.log; [ $rc -eq 0 ] || exit 1
MA="--steps 5 --warmup 2 --no-cpu --no-hamming --no-stereo --no-host-path --no-bird --no-c4 --no-profile-pass"
for i in 1 2; do
  for sig in 2 1 0; do
    L=gpurun_out/ab27/bench_matcher_${sig}_$i.log
    ORBGPU_DONE_SIGNAL=$sig timeout -k 10 200 python3 bench.py $MA > $L 2>&1 || { tail -5 $L; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$L') if l.startswith('{')][-1])['matcher']; print('signal=$sig', json.dumps({k: (v.get('gpu_us'), v.get('cpu_us'), v.get('speedup'), v.get('equal')) for k, v in d.items() if isinstance(v, dict) and 'gpu_us' in v}))"
  done
done

# fp4 top-2 with the trains expanded while staged (no expansion kernel, ORBGPU_TOP2=8fx) vs the default
set -o pipefail
mkdir -p gpurun_out/ab17; export TMPDIR=/tmp
T="timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread"
for v in 8fx 8f; do
  ORBGPU_TOP2=$v $T tests/test_gpu_matcher.py > gpurun_out/ab17/pytest_$v.log 2>&1; echo "$v: $(tail -1 gpurun_out/ab17/pytest_$v.log)"
  grep -E "n_bad" gpurun_out/ab17/pytest_$v.log | head -3 | cut -c1-300
done
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 8f 8fx 8f 8fx; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab17/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab17/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab17/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
ORBGPU_TOP2=8fx timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab17/pytest_gpu_x.log 2>&1; echo "all gpu tests, 8fx: $(tail -1 gpurun_out/ab17/pytest_gpu_x.log)"
exit 0

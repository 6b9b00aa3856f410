# fp4 fragments kept live until the chain's result is read: matcher tests under the three fp4 forms, bench A/B,
# then (if the resident form passes) the full GPU suite under it
set -o pipefail
mkdir -p gpurun_out/ab12; export TMPDIR=/tmp
T="timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread"
ok=1
for v in 8fu R 8fp; do
  ORBGPU_TOP2=$v $T tests/test_gpu_matcher.py > gpurun_out/ab12/pytest_$v.log 2>&1 || ok=0; echo "$v: $(tail -1 gpurun_out/ab12/pytest_$v.log)"
  grep -E "n_bad" gpurun_out/ab12/pytest_$v.log | head -4 | cut -c1-300
done
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 8fp R 81p 8fp R; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab12/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab12/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab12/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
[ $ok -eq 1 ] || exit 0
ORBGPU_TOP2=R timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab12/pytest_gpu_R.log 2>&1; echo "all gpu tests, R: $(tail -1 gpurun_out/ab12/pytest_gpu_R.log)"

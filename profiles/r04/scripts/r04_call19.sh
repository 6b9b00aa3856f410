# fp4 in-staging form with 4-wave workgroups (ORBGPU_TOP2=4fx) vs the default 8-wave one
set -o pipefail
mkdir -p gpurun_out/ab19; export TMPDIR=/tmp
T="timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread"
ORBGPU_TOP2=4fx $T tests/test_gpu_matcher.py > gpurun_out/ab19/pytest_4fx.log 2>&1; echo "4fx: $(tail -1 gpurun_out/ab19/pytest_4fx.log)"
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 8fx 4fx 8fx 4fx; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab19/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab19/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab19/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
exit 0

# f16 key bits masked explicitly (no pad, no fragment keep): matcher tests under every top-2 form, bench A/B,
# then the full GPU suite under the default
set -o pipefail
mkdir -p gpurun_out/ab14; export TMPDIR=/tmp
T="timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread"
for v in 8fu R 8fp 81p; do
  ORBGPU_TOP2=$v $T tests/test_gpu_matcher.py > gpurun_out/ab14/pytest_$v.log 2>&1; echo "$v: $(tail -1 gpurun_out/ab14/pytest_$v.log)"
  grep -E "n_bad" gpurun_out/ab14/pytest_$v.log | head -3 | cut -c1-300
done
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 8fp R 8fu 81p 8fp R; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab14/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab14/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab14/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab14/pytest_gpu.log 2>&1; echo "all gpu tests, default: $(tail -1 gpurun_out/ab14/pytest_gpu.log)"
exit 0

# fp4 in-staging top-2 with two 32-train subtiles per stage (queries block-scaled 2^1, keys dist << 6 | row):
# the probe's scaled-MFMA check, matcher tests under 82fx, bench A/B against 8fx
set -o pipefail
mkdir -p gpurun_out/ab20; export TMPDIR=/tmp
timeout -k 10 60 ./tools/mfma_fp4_probe > gpurun_out/ab20/probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/ab20/probe.log
T="timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread"
ORBGPU_TOP2=82fx $T tests/test_gpu_matcher.py > gpurun_out/ab20/pytest_82fx.log 2>&1; echo "82fx: $(tail -1 gpurun_out/ab20/pytest_82fx.log)"
grep -E "n_bad" gpurun_out/ab20/pytest_82fx.log | head -3 | cut -c1-300
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 8fx 82fx 8fx 82fx; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab20/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab20/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab20/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
exit 0

# Hamming A/B: matcher GPU tests on the default build, then the bench's Hamming leg under each
# ORBGPU_TOP2=<waves><subtiles> variant, then the profiling passes of the default
set -o pipefail
mkdir -p gpurun_out/ab; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py > gpurun_out/pytest_matcher.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_matcher.log; [ $rc -eq 0 ] || exit 1
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
ORBGPU_TOP2=81pPol timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py > gpurun_out/pytest_matcher_l.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_matcher_l.log; [ $rc -eq 0 ] || exit 1
for v in 81pPo 81pPol 81pPoL 81pP 81p 81P 81pPol 81pPo; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab/top2_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab/top2_$v.log') if l.startswith('{')][-1])['hamming']; print('$v', d['kernel_avg_us'], d['mfma_i8']['frac'], d['matches_per_s'])"
done
bash tools/ham_prof.sh > gpurun_out/ab/ham_prof.log 2>&1 || { tail -20 gpurun_out/ab/ham_prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ham/report.json')); print(d.get('trace_mean_us_per_dispatch'), d.get('trace_leg_us'), d.get('frac_from_trace'), d.get('top2_mfma'), d.get('hbm_bytes_per_dispatch'))"

# the resident-chunk fp4 top-2 (ORBGPU_TOP2=R): matcher tests, bench A/B against the default, then (if it is kept)
# the full GPU suite and the Hamming profile under it
set -o pipefail
mkdir -p gpurun_out/ab10; export TMPDIR=/tmp
T="timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
ORBGPU_TOP2=8fu $T tests/test_gpu_matcher.py > gpurun_out/ab10/pytest_8fu.log 2>&1; rc=$?; echo "8fu (unpipelined fp4, padded): $(tail -1 gpurun_out/ab10/pytest_8fu.log)"
ORBGPU_TOP2=R $T tests/test_gpu_matcher.py > gpurun_out/ab10/pytest_R.log 2>&1; rc=$?; echo "R: $(tail -1 gpurun_out/ab10/pytest_R.log)"; [ $rc -eq 0 ] || { tail -40 gpurun_out/ab10/pytest_R.log; exit 1; }
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 8fp R 8fp R; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab10/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab10/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab10/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
ORBGPU_TOP2=R timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab10/pytest_gpu_R.log 2>&1; rc=$?; echo "all gpu tests, R: $(tail -1 gpurun_out/ab10/pytest_gpu_R.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ab10/pytest_gpu_R.log; exit 1; }
ORBGPU_TOP2=R HAM_OUT=gpurun_out/ham_R bash tools/ham_prof.sh > gpurun_out/ab10/ham_prof_R.log 2>&1 || { tail -20 gpurun_out/ab10/ham_prof_R.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ham_R/report.json')); print('R', d.get('trace_mean_us_per_dispatch'), d.get('trace_leg_us'), d.get('frac_from_trace'), d.get('top2_mfma'), d.get('hbm_bytes_per_dispatch'))"

# fp4 form of the Hamming top-2: the operand-map probe, the matcher GPU tests under the fp4 and lookahead forms,
# the bench Hamming leg per ORBGPU_TOP2 variant, then the profiling passes of the int8 default and of the fp4 form
set -o pipefail
mkdir -p gpurun_out/ab8; export TMPDIR=/tmp
timeout -k 10 60 ./tools/mfma_fp4_probe > gpurun_out/ab8/probe.log 2>&1; rc=$?; cat gpurun_out/ab8/probe.log; [ $rc -eq 0 ] || exit 1
T="timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for v in 8fp 8fpl 81pl; do
  ORBGPU_TOP2=$v $T tests/test_gpu_matcher.py > gpurun_out/ab8/pytest_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/ab8/pytest_$v.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ab8/pytest_$v.log; exit 1; }
done
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 81p 8fp 81pl 8fpl 81pL 81pPl 8fpP 81p 8fp; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab8/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab8/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab8/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
ORBGPU_TOP2=8fp timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab8/pytest_gpu_fp4.log 2>&1; rc=$?; echo "all gpu tests, fp4: $(tail -1 gpurun_out/ab8/pytest_gpu_fp4.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ab8/pytest_gpu_fp4.log; exit 1; }
HAM_OUT=gpurun_out/ham_i8 bash tools/ham_prof.sh > gpurun_out/ab8/ham_prof_i8.log 2>&1 || { tail -20 gpurun_out/ab8/ham_prof_i8.log; exit 1; }
ORBGPU_TOP2=8fp HAM_OUT=gpurun_out/ham_fp4 bash tools/ham_prof.sh > gpurun_out/ab8/ham_prof_fp4.log 2>&1 || { tail -20 gpurun_out/ab8/ham_prof_fp4.log; exit 1; }
for f in i8 fp4; do python3 -c "import json; d=json.load(open('gpurun_out/ham_$f/report.json')); print('$f', d.get('trace_mean_us_per_dispatch'), d.get('trace_leg_us'), d.get('frac_from_trace'), d.get('top2_mfma'), d.get('hbm_bytes_per_dispatch'))"; done

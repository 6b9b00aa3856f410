# fp4 in-staging top-2 with the staged rows loaded two stages ahead: GPU suite, bench Hamming leg x3, profile
set -o pipefail
mkdir -p gpurun_out/ab23; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab23/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/ab23/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|n_bad" gpurun_out/ab23/pytest_gpu.log | head; exit 1; }
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab23/top2_$i.log 2>&1 || { tail -5 gpurun_out/ab23/top2_$i.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab23/top2_$i.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('8fx+prefetch2', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
HAM_OUT=gpurun_out/ham23 bash tools/ham_prof.sh > gpurun_out/ab23/ham_prof.log 2>&1 || { tail -20 gpurun_out/ab23/ham_prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ham23/report.json')); print(d.get('trace_mean_us_per_dispatch'), d.get('trace_leg_us'), d.get('frac_from_trace'), d.get('top2_mfma'), d.get('hbm_bytes_per_dispatch'))"

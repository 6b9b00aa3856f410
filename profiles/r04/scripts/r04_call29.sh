# fp4 top-2 accumulator seed rebuilt per stage at 8 waves per SIMD vs held at 6 (build_ab/liborbgpu_s0.so, ORBGPU_TOP2_SEED_PER_STAGE=0):
# GPU suite on the new form, bench Hamming leg alternating x3, rocprof trace + PMC of the new form
set -o pipefail
mkdir -p gpurun_out/ab29; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab29/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/ab29/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|n_bad" gpurun_out/ab29/pytest_gpu.log | head; exit 1; }
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for i in 1 2 3; do
  for v in seed8 s0; do
    L=gpurun_out/ab29/top2_${v}_$i.log
    if [ $v = s0 ]; then export ORBGPU_LIB_PATH=$PWD/orb-slam-birdview_amd/build_ab/liborbgpu_s0.so; else unset ORBGPU_LIB_PATH; fi
    timeout -k 10 120 python3 bench.py $ARGS > $L 2>&1 || { tail -5 $L; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$L') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
  done
done
unset ORBGPU_LIB_PATH
HAM_OUT=gpurun_out/ham29 bash tools/ham_prof.sh > gpurun_out/ab29/ham_prof.log 2>&1 || { tail -20 gpurun_out/ab29/ham_prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ham29/report.json')); print(d.get('trace_mean_us_per_dispatch'), d.get('trace_leg_us'), d.get('frac_from_trace'), d.get('top2_mfma'), d.get('hbm_bytes_per_dispatch'))"

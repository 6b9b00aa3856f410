# round-4 evidence on the final defaults: GPU tests + smoke + PMC + bench lines + rocprof traces (tools/gpu_round.sh),
# then the Hamming leg's two-chunk expansion overlap A/B and the host path under HSA_ENABLE_SDMA=0
set -o pipefail
export TMPDIR=/tmp
PMC=1 bash tools/gpu_round.sh || exit 1
mkdir -p gpurun_out/ab9
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 8fp 8fpo 8fp 8fpo; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab9/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab9/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab9/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
ORBGPU_TOP2=8fpo timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py > gpurun_out/ab9/pytest_o.log 2>&1; rc=$?; echo "8fpo: $(tail -1 gpurun_out/ab9/pytest_o.log)"; [ $rc -eq 0 ] || exit 1
bash tools/host_quick.sh HSA_ENABLE_SDMA=0 > gpurun_out/ab9/host_sdma.log 2>&1 || { tail -5 gpurun_out/ab9/host_sdma.log; exit 1; }
cut -c1-120 gpurun_out/ab9/host_sdma.log

# pipelined fp4 in-staging top-2 (ORBGPU_TOP2=8fxp: stage j's MFMAs beside stage j-1's top-2; 96 VGPRs) vs the default
set -o pipefail
mkdir -p gpurun_out/ab31; export TMPDIR=/tmp
T="timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread"
ORBGPU_TOP2=8fxp $T tests/test_gpu_matcher.py > gpurun_out/ab31/pytest_8fxp.log 2>&1; rc=$?; echo "8fxp: $(tail -1 gpurun_out/ab31/pytest_8fxp.log)"; [ $rc -eq 0 ] || { grep -E "n_bad|^FAILED" gpurun_out/ab31/pytest_8fxp.log | head -3 | cut -c1-300; exit 1; }
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for i in 1 2 3; do
  for v in default 8fxp; do
    L=gpurun_out/ab31/top2_${v}_$i.log
    if [ $v = default ]; then unset ORBGPU_TOP2; else export ORBGPU_TOP2=$v; fi
    timeout -k 10 120 python3 bench.py $ARGS > $L 2>&1 || { tail -5 $L; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$L') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
  done
done

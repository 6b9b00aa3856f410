# diagnose the fp4 top-2 forms that read a chain's result right after its last MFMA (unpipelined 'u', resident 'R')
set -o pipefail
mkdir -p gpurun_out/ab11; export TMPDIR=/tmp
T="timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread"
for v in 8fu R; do
  ORBGPU_TOP2=$v $T tests/test_gpu_matcher.py -k "top2" > gpurun_out/ab11/pytest_$v.log 2>&1; echo "$v: $(tail -1 gpurun_out/ab11/pytest_$v.log)"
  grep -E "^E  .*n_bad|AssertionError: \(|assert False|n_bad" gpurun_out/ab11/pytest_$v.log | head -12 | cut -c1-400
done
exit 0

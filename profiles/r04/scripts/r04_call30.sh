# HEAD check: GPU tests, smoke, the default bench line
set -o pipefail
export TMPDIR=/tmp
SKIP_TESTS= bash -c 'true'
mkdir -p gpurun_out/final30
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/final30/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/final30/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final30/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/final30/smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final30/bench.log 2>&1 || { tail -5 gpurun_out/final30/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/final30/bench.log') if l.startswith('{')][-1]); h=d['hamming']; print(d['value'], d['ms_per_step'], h['kernel_avg_us'], h['matches_per_s'], (h.get('mfma_fp4') or {}).get('frac'), d['roofline']['frac'])"

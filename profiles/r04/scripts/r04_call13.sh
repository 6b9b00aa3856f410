# fp4 chain probe (result read right after a dependent chain, with 0 / 32 / 128 extra wait states); the
# unpipelined fp4 form with a 128-state pad; the full GPU suite under the resident form
set -o pipefail
mkdir -p gpurun_out/ab13; export TMPDIR=/tmp
timeout -k 10 60 ./tools/mfma_fp4_chain_probe > gpurun_out/ab13/chain_probe.log 2>&1; echo "probe rc=$?"; cat gpurun_out/ab13/chain_probe.log
T="timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread"
ORBGPU_TOP2=8fu $T tests/test_gpu_matcher.py > gpurun_out/ab13/pytest_8fu.log 2>&1; echo "8fu pad128: $(tail -1 gpurun_out/ab13/pytest_8fu.log)"
grep -E "n_bad" gpurun_out/ab13/pytest_8fu.log | head -3 | cut -c1-300
ORBGPU_TOP2=R timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab13/pytest_gpu_R.log 2>&1; echo "all gpu tests, R: $(tail -1 gpurun_out/ab13/pytest_gpu_R.log)"
exit 0

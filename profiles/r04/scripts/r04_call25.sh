# completion-signal diagnosis: the new triangulation test under both settings (no -x), then the existing ones
set -o pipefail
mkdir -p gpurun_out/ab25; export TMPDIR=/tmp
T="timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread"
$T tests/test_gpu_matcher.py -k "triangulation" > gpurun_out/ab25/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab25/pytest.log; grep -n "AssertionError: " gpurun_out/ab25/pytest.log; exit $rc

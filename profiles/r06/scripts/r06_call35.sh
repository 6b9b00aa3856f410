set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c35; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py -x -v --timeout 120 --timeout-method thread > $O/pytest_fuzz.log 2>&1; rc=$?; tail -5 $O/pytest_fuzz.log; exit $rc

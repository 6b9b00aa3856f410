# Hamming iteration: the matcher GPU tests (incl. the bench-shape top-2), then the profiling passes
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py > gpurun_out/pytest_matcher.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_matcher.log; [ $rc -eq 0 ] || exit 1
bash tools/ham_prof.sh

set -o pipefail
O=gpurun_out/c21; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
echo "pytest: $(tail -1 $O/pytest.log)"

# first run of the dataflow launch: its own tests (each step time-limited), then the small-batch extraction tests,
# then the C5 one-frame bench (4 and 1 in flight)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c2; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_flow.py > $O/pytest_flow.log 2>&1; rc=$?; tail -15 $O/pytest_flow.log; [ $rc -eq 0 ] || exit 1
$T 180 python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5b1.txt 2>&1 && tail -1 $O/c5b1.txt | cut -c1-600 &&
$T 180 python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/c5b1p1.txt 2>&1 && tail -1 $O/c5b1p1.txt | cut -c1-600 &&
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_variants.py > $O/pytest_extract.log 2>&1; rc=$?; tail -3 $O/pytest_extract.log; exit $rc

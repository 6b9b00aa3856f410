set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c36; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/pytest_fuzz.log 2>&1 && \
timeout -k 10 600 python -u tools/fuzz_parity.py 400 0 > $O/fuzz_extract.log 2>&1 && \
timeout -k 10 600 python -u tools/fuzz_matcher.py 150 0 > $O/fuzz_matcher.log 2>&1; rc=$?
tail -2 $O/pytest_fuzz.log; tail -1 $O/fuzz_extract.log; tail -1 $O/fuzz_matcher.log; exit $rc

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c34; mkdir -p $O
timeout -k 10 900 python -u tools/fuzz_matcher.py 150 0 > $O/fuzz_matcher.log 2>&1; rc=$?; tail -3 $O/fuzz_matcher.log; exit $rc

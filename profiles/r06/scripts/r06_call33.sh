set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c33; mkdir -p $O
timeout -k 10 900 python -u tools/fuzz_parity.py 400 0 > $O/fuzz.log 2>&1; rc=$?; tail -3 $O/fuzz.log; grep -c refused $O/fuzz.log; exit $rc

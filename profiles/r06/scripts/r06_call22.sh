# the glibc_sincosf rewrite: which part differs on the device (the sincos sweep vs the extraction tests)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c22; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -k "sincosf or extract_bit_exact" > $O/pytest.log 2>&1; tail -5 $O/pytest.log
grep -E "^E  " $O/pytest.log | head -20
exit 0

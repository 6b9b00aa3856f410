# quick check of an extraction-kernel change: extraction / fuzz / mirror tests, then the C3 bench (extraction only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_fuzz.py tests/test_host_mirror.py -m gpu > $O/pytest.log 2>&1 && \
timeout -k 10 200 python bench.py --only-extract > $O/bench1.log 2>&1 && \
timeout -k 10 200 python bench.py --only-extract > $O/bench2.log 2>&1; rc=$?
tail -2 $O/pytest.log; grep -h '^{' $O/bench1.log $O/bench2.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(round(d['value']/1e6,1), d['kernels_ms_per_step'])"
exit $rc

#!/bin/bash
# host path: extraction parity tests, then a kernel trace of the host loop and its timeline
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_variants.py -m gpu > $OUT/ext.log 2>&1; tail -2 $OUT/ext.log
grep -q " passed" $OUT/ext.log && ! grep -q "failed" $OUT/ext.log || exit 1
bash tools/host_path_prof.sh || exit 1
python3 tools/timeline.py $OUT/hp 2
bash tools/host_quick.sh

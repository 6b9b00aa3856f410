#!/bin/bash
# Quick GPU iteration: GPU tests then a short bench. Stops at the first failure.
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests -q -m gpu -x > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log

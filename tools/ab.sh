#!/bin/bash
# A/B: GPU tests once, then the bench under each env setting in $VARIANTS (';'-separated), interleaved
# twice in one call (cdna guide rule 24).  Prints kernels_ms_per_step and value per run.
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 420 python -m pytest tests -q -m gpu -x > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
IFS=';' read -ra VS <<< "$VARIANTS"
for rep in 1 2; do
  for v in "${VS[@]}"; do
    env $v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-hamming ${BENCH_ARGS} > $OUT/ab.log 2>&1 || { echo "bench failed ($v)"; tail -20 $OUT/ab.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/ab.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'Mfeat/s', d['kernels_ms_per_step'])"
  done
done

#!/bin/bash
# A/B of library builds (GPU box): the C3 extraction bench (--only-extract) under each liborbgpu.so given
# (paths; "tree" = the in-tree build), interleaved twice.  Prints value and per-kernel ms per run.
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --steps 50 --warmup 10 --only-extract ${BENCH_ARGS} > $OUT/ab.log 2>&1 || { echo "bench failed ($lib)"; tail -20 $OUT/ab.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/ab.log') if l.startswith('{')][-1]); print('$lib', round(d['value']/1e6,2), 'Mfeat/s', d['kernels_ms_per_step'])"
  done
done
unset ORBGPU_LIB_PATH

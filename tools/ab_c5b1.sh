#!/bin/bash
# A/B of library builds on C5 at one frame per step, four in flight (what one GPU does at N = 8)
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --config c5 --batch 1 --pipelines 4 --steps 400 --warmup 40 --only-extract > $OUT/abc5.log 2>&1 || { echo "bench failed ($lib)"; tail -20 $OUT/abc5.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$OUT/abc5.log') if l.startswith('{')][-1]); print('$lib', round(d['value']/1e6,2), 'Mfeat/s', d['kernels_ms_per_step'])"
  done
done
unset ORBGPU_LIB_PATH

#!/bin/bash
# C5 at one frame per step: frames in flight (pipelines) against the runtime's hardware queues per process
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for cfg in "4 4" "8 8" "8 4" "16 16"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python bench.py --config c5 --batch 1 --pipelines $1 --steps 400 --warmup 40 --only-extract > $OUT/hwq.log 2>&1 || { echo "bench failed ($cfg)"; tail -5 $OUT/hwq.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$OUT/hwq.log') if l.startswith('{')][-1]); print('P=$1 HWQ=$2', round(d['value']/1e6,2), 'Mfeat/s')"
done

#!/bin/bash
# Host-path latency (diagnostic): GPU tests, then the C++ mirror's operator() per host frame, then a
# kernel trace of the same loop (launch order / overlap of the latency order).
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest -x -q tests -m gpu > $OUT/pt_host.log 2>&1 || { tail -30 $OUT/pt_host.log; exit 1; }
tail -1 $OUT/pt_host.log
python3 -c "
import sys; sys.path.insert(0,'orb-slam-birdview_amd')
import numpy as np
from orbgpu.synth import synth_batch
open('/tmp/frames.raw','wb').write(np.ascontiguousarray(synth_batch(1280,720,16)).tobytes())
"
for rep in 1 2; do
  timeout -k 10 60 ./tools/host_latency /tmp/frames.raw 1280 720 16 2000 300 || exit 1
done


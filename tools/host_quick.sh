#!/bin/bash
# Host-path latency A/B (GPU box): the C++ mirror's operator() per host C3 frame (tools/host_latency),
# default settings vs the env assignments given as arguments (e.g. ORBGPU_GRAPH=0), two runs each.
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
python3 -c "
import sys; sys.path.insert(0,'orb-slam-birdview_amd')
import numpy as np
from orbgpu.synth import synth_batch
open('/tmp/frames.raw','wb').write(np.ascontiguousarray(synth_batch(1280,720,16)).tobytes())
"
for rep in 1 2; do
  echo -n "default: "; timeout -k 10 60 ./tools/host_latency /tmp/frames.raw 1280 720 16 2000 300 || exit 1
  for kv in "$@"; do
    echo -n "$kv: "; env $kv timeout -k 10 60 ./tools/host_latency /tmp/frames.raw 1280 720 16 2000 300 || exit 1
  done
done

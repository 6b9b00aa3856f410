#!/bin/bash
# k_fast_wave's VALU by phase (GPU box): SQ counters of the ab/cutN builds (-DORBGPU_FAST_CUT=N: 1 stops after
# the ROI load + widening, 2 after the pass-0 prefilter + compaction, 3 after the pass-0 arc strengths) and
# of the in-tree build.  Build the cut libraries first (DESIGN.md §4.5 has the recipe and the numbers).
for n in 1 2 3 tree; do
  if [ $n = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/cut$n/liborbgpu.so; fi
  COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" bash tools/sq_quick.sh 2>&1 | grep fast | sed "s/^/cut$n /"
done

#!/bin/bash
# SQ / MFMA counters of the Hamming leg's kernels (k_expand_pm1, k_top2_mfma, k_top2b_merge)
COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-profile-pass" \
bash "$(dirname "$0")/sq_quick.sh"

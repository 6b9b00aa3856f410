#!/bin/bash
# One SQ counter pass over a short bench run: per-kernel counters per launch for quick A/B of kernel
# edits (tools/sq_quick.py prints them).  Defaults: the extraction batch launches only.
#   COUNTERS="..."  override the counter list (at most 8 SQ_, 2 GRBM_ per pass)
#   BENCH_ARGS="..." override the bench arguments (e.g. the Hamming leg: see tools/sq_hamming.sh)
OUT=gpurun_out/sq; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
CTRS=${COUNTERS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --only-extract --no-profile-pass"}
timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py $ARGS > $OUT/bench.log 2>&1 || { echo "SQ pass failed"; tail -20 $OUT/bench.log; exit 1; }
python3 tools/sq_quick.py $OUT

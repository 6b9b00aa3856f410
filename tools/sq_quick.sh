#!/bin/bash
# One SQ counter pass over the bench's batch launches only (--only-extract): per-kernel VALU / LDS /
# SALU instruction counts per launch for quick A/B of kernel edits (tools/sq_quick.py prints them).
OUT=gpurun_out/sq; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 3 --warmup 1 --only-extract --no-profile-pass ${BENCH_ARGS} > $OUT/bench.log 2>&1 || { echo "SQ pass failed"; tail -20 $OUT/bench.log; exit 1; }
python3 tools/sq_quick.py $OUT

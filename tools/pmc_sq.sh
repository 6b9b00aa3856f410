#!/bin/bash
# SQ counter passes (issue/stall breakdown per kernel) over a short bench run; --kernel-trace only.
# Results under gpurun_out/pmc_sq/; summarised by tools/pmc_sq_report.py.
OUT=gpurun_out/pmc_sq; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu --no-hamming --no-host-path --no-stereo ${BENCH_ARGS}"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_sq_report.py $OUT

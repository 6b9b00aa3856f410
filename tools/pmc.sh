#!/bin/bash
# rocprofv3 PMC passes (one TCC counter per pass, --kernel-trace only; no sys/runtime traces):
#   calibration binary (known byte counts per access width) and a short bench run, FETCH_SIZE then
#   WRITE_SIZE.  Results under gpurun_out/pmc/<pass>/; tools/pmc_report.py turns them into
#   profiles/pmc_traffic.json.  Every GPU step has its own time limit; the script stops at the first failure.
OUT=gpurun_out/pmc; mkdir -p $OUT; export TMPDIR=/tmp
# only the batch launches: the host-path, stereo and C4 legs would mix 1- and 2-frame dispatches
# into the per-launch means
ARGS="--steps 3 --warmup 1 --only-extract --no-profile-pass ${BENCH_ARGS}"
timeout -k 10 120 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/pmc_calib tools/pmc_calib.hip || { echo "calib build failed"; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/calib_$ctr -o run -- /tmp/pmc_calib > $OUT/calib_$ctr.log 2>&1 || { echo "calib $ctr failed"; tail -20 $OUT/calib_$ctr.log; exit 1; }
  echo "calib $ctr ok"
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/bench_$ctr -o run -- python3 bench.py $ARGS > $OUT/bench_$ctr.log 2>&1 || { echo "bench $ctr failed"; tail -20 $OUT/bench_$ctr.log; exit 1; }
  echo "bench $ctr ok"
done
# issue counters of the same kernels (VALU roofline): one SQ pass
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $OUT/bench_SQ -o run -- python3 bench.py $ARGS > $OUT/bench_SQ.log 2>&1 || { echo "bench SQ failed"; tail -20 $OUT/bench_SQ.log; exit 1; }
echo "bench SQ ok"
python3 tools/pmc_report.py $OUT > $OUT/report.json && cat $OUT/report.json

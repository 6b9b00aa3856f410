#!/bin/bash
# Evidence for the Hamming half of the headline metric (bench.py's `hamming` leg: 255 consecutive C3 frame
# pairs per orb_hamming_top2_frames_device launch): a rocprofv3 kernel trace + stats of the leg, then PMC
# passes over the same run (SQ issue / MFMA counters; FETCH_SIZE; WRITE_SIZE), each its own run with
# --kernel-trace only.  tools/ham_report.py turns gpurun_out/ham/ into profiles/<round>/<tag>_hamming.json.
# Every GPU step has its own limit; the script stops at the first failure.
OUT=${HAM_OUT:-gpurun_out/ham}; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
ARGS="--steps 20 --warmup 3 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $OUT/$name.log; echo "$name rc=$rc"; [ $rc -eq 0 ] || tail -20 $OUT/$name.log; return $rc; }
step bench 240 python3 bench.py $ARGS || exit 1
step trace 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS || exit 1
step sq 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS || exit 1
step sq2 240 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS || exit 1
step fetch 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS || exit 1
step write 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS || exit 1
python3 tools/ham_report.py $OUT > $OUT/report.json && cat $OUT/report.json

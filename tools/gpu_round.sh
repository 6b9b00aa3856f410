#!/bin/bash
# One GPU-box session: GPU tests, smoke, the bench (default C3 line + C2 / C5 lines), a rocprofv3
# kernel-trace of ONLY the timed extraction loop (so profiles/ reproduces roofline.frac), then PMC passes.
# Each GPU step has its own limit; the script stops at the first failure.
# Afterwards, locally: python3 tools/collect_profiles.py rNN_vM  (copies the summaries into profiles/).
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $OUT/$name.log; echo "$name rc=$rc"; return $rc; }
if [ -z "$SKIP_TESTS" ]; then
  step pytest_gpu 480 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu || exit 1
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
# PMC passes first, so the bench line's roofline.traffic / roofline.valu come from this same build
if [ -n "$PMC" ]; then
  bash tools/pmc.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
  echo "pmc ok"
  export ORBGPU_PMC_JSON=$OUT/pmc/report.json
fi
step bench 600 python bench.py || exit 1
# the driver's own command (BENCH_rNN.json)
step bench_driver_form 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
step bench_c2 300 python bench.py --config c2 --no-cpu --no-c4 --no-bird || exit 1
step bench_c5 300 python bench.py --config c5 --steps 50 --warmup 5 --no-cpu --no-c4 --no-bird --no-stereo || exit 1
# what one GPU does at N = 8 in C5 (one frame per step, four in flight)
step bench_c5b1 300 python bench.py --config c5 --batch 1 --pipelines 4 --steps 400 --warmup 40 --only-extract || exit 1
# the timed loop as the bench runs it (two batches in flight: kernel durations of the two streams overlap)
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --only-extract --no-profile-pass --steps 20 --warmup 3 || exit 1
# the same loop one batch at a time: per-launch durations comparable with the bench's HIP-event roofline pass
step rocprof_serial 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_serial -o run -- python3 bench.py --only-extract --no-profile-pass --pipelines 1 --steps 100 --warmup 20 || exit 1
exit 0

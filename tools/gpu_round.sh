#!/bin/bash
# One GPU-box session: GPU tests, smoke, rocprof kernel-trace stats, PMC passes (traffic + issue
# counters), then the bench, whose roofline.traffic / roofline.valu read the PMC report of this same
# session (ORBGPU_PMC_JSON).  Each GPU step has its own limit; the script stops at the first failure.
# Afterwards, locally: python3 tools/collect_profiles.py rNN_vM  (copies the summaries into profiles/).
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $OUT/$name.log; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 480 python -m pytest tests -q -m gpu -x || exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu || exit 1
bash tools/pmc.sh > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $OUT/pmc.log; exit 1; }
echo "pmc ok"
export ORBGPU_PMC_JSON=$OUT/pmc/report.json
step bench 300 python bench.py --steps 20 --warmup 3 || exit 1
exit 0

#!/bin/bash
# One GPU-box session: tests, smoke, bench, rocprof kernel trace. Each GPU step has its own limit;
# the script stops at the first failure.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $OUT/$name.log; echo "$name rc=$rc"; return $rc; }
step pytest_gpu 420 python -m pytest tests -q -m gpu -x || exit 1
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 300 python bench.py --steps 10 --warmup 2 || exit 1
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 5 --warmup 1 --no-cpu || exit 1
exit 0

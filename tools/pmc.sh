#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, --kernel-trace only,
# no sys/runtime traces).  Results under gpurun_out/pmc/<pass>/.
OUT=gpurun_out/pmc; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp; cd - >/dev/null
ARGS="--steps 5 --warmup 1 --no-cpu --no-hamming"
[ -n "$LIST" ] && { rocprofv3 -L > $OUT/counters.txt 2>&1; grep -oE "^[[:space:]]*(SQ|TCC|TCP|TA|GRBM)[A-Za-z0-9_]*" $OUT/counters.txt | sort -u > $OUT/counter_names.txt; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc ${grp//,/ } --kernel-trace --output-format csv -d $OUT/p$i -o run -- python bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -20 $OUT/p$i.log; exit 1; }
  echo "pass $i ($grp) ok"
done

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c29; mkdir -p $O
timeout -k 10 300 python3 tools/matcher_prof.py 640 480 1000 $O/c2 > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
cat $O/c2/prof/run_kernel_stats.csv | cut -d, -f1-8 | head -20

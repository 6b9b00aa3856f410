# round-4 evidence on the final Hamming default (fp4, unpipelined, masked keys): GPU tests + smoke + PMC + bench
# lines + rocprof traces (tools/gpu_round.sh), then the Hamming leg's trace + PMC (tools/ham_prof.sh)
set -o pipefail
export TMPDIR=/tmp
PMC=1 bash tools/gpu_round.sh || exit 1
HAM_OUT=gpurun_out/ham_final bash tools/ham_prof.sh > gpurun_out/ham_final.log 2>&1 || { tail -20 gpurun_out/ham_final.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ham_final/report.json')); print(d.get('trace_mean_us_per_dispatch'), d.get('trace_leg_us'), d.get('frac_from_trace'), d.get('top2_mfma'), d.get('hbm_bytes_per_dispatch'))"

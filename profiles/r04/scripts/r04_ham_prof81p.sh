set -o pipefail
export ORBGPU_TOP2=81p
bash tools/ham_prof.sh > gpurun_out/ham_prof.log 2>&1 || { tail -20 gpurun_out/ham_prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ham/report.json')); print(d['trace_mean_us'], d['frac_from_trace'], d['top2_mfma']); print(d['sq_per_launch']['k_top2_mfma'])"

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c11; mkdir -p $O
T="timeout -k 10"
$T 300 env ORBGPU_STRIPES=64 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 200 --no-profile-pass > $O/run.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r06c11/prof/**/*kernel_stats.csv', recursive=True)[0]
for row in csv.DictReader(open(f)):
    print(row['Name'][:60], row['Calls'], row['AverageNs'], row['MinNs'], row['MaxNs'])
PY

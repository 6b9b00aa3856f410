set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c13; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -k stripe > $O/pytest_stripe.log 2>&1; rc=$?; tail -2 $O/pytest_stripe.log; [ $rc -eq 0 ] || exit 1
for K in 64 128 256; do
$T 300 env ORBGPU_STRIPES=$K rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$K -o run -- python3 bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 200 --no-profile-pass > $O/run$K.log 2>&1 || exit 1
python3 - $K <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/r06c13/prof{sys.argv[1]}/**/*kernel_stats.csv', recursive=True)[0]
for row in csv.DictReader(open(f)):
    if 'stripes' in row['Name'] or 'resize' in row['Name'] or 'chain' in row['Name']: print(sys.argv[1], row['Name'][:40], row['Calls'], row['AverageNs'], row['MinNs'])
PY
done

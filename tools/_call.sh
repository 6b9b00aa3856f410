set -o pipefail
O=gpurun_out/c19; mkdir -p $O; export TMPDIR=/tmp
ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_patch.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_variants.py tests/test_mask_fixture.py > $O/pytest_patch.log 2>&1 || { echo "pytest patch failed"; tail -30 $O/pytest_patch.log; exit 1; }
echo "pytest (patch lib): $(tail -1 $O/pytest_patch.log)"
for v in tree patch; do
  if [ $v = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$v.so; fi
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/pmc_$v -o run -- python3 bench.py --steps 3 --warmup 1 --only-extract --no-profile-pass > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -20 $O/pmc_$v.log; exit 1; }
  python3 - $O/pmc_$v <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    k = 'describe' if 'k_describe' in n else None
    if k: acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k in acc: print(sys.argv[1], k, {c: round(sum(v)/len(v)/1e6, 2) for c, v in acc[k].items()}, "M per launch")
PY
done
unset ORBGPU_LIB_PATH
bash tools/gpu_run.sh c19 "ab=tree,ab/liborbgpu_patch.so@--steps 100 --warmup 20 --only-extract"

# Overflow slots slot-major per level (tree) vs cell-contiguous (ab/liborbgpu_r6old.so): parity, octree/fast
# traffic (FETCH_SIZE / WRITE_SIZE, separate passes, --kernel-trace only), time (C3 batch, C5 one frame).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c17; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py tests/test_gpu_flow.py tests/test_tie_order.py tests/test_host_mirror.py > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for lib in tree r6old; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    $T 240 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/pmc_${lib}_$ctr -o run -- python3 bench.py --steps 3 --warmup 1 --only-extract --no-profile-pass > $O/pmc_${lib}_$ctr.log 2>&1 || { echo "pmc $lib $ctr failed"; tail -5 $O/pmc_${lib}_$ctr.log; exit 1; }
  done
  python3 - $O $lib <<'PY'
import sys
sys.path.insert(0, "tools")
from pmc_report import load
o, lib = sys.argv[1], sys.argv[2]
for ctr, fac in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
    d, _ = load(f"{o}/pmc_{lib}_{ctr}", ctr)
    print(lib, ctr, {k: round(sum(v) / len(v) * 1024 * fac / 1e6, 2) for k, v in sorted(d.items()) if k in ("fast", "octree", "resize", "describe")}, "MB per launch (FETCH x2 calibration)")
PY
done
unset ORBGPU_LIB_PATH
for rep in 1 2; do for lib in tree r6old; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  $T 180 python bench.py --only-extract --steps 200 > $O/c3_$lib.txt 2>&1 || exit 1
  $T 180 python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
for f in ['$O/c3_$lib.txt','$O/c5_$lib.txt']:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print('$lib', f.split('/')[-1], round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done; done

# k_resize_tiled: runs of 2 / 4 / 8 horizontally adjacent tiles per XCD (rsrun2 / tree / rsrun8) vs plain
# round-robin (r6old): parity, FETCH_SIZE of the resize launches, C3 time.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c19; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -k "pyramid or bench or c2 or c5 or variant" > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for lib in tree rsrun2 rsrun8 r6old; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  $T 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_${lib} -o run -- python3 bench.py --steps 3 --warmup 1 --only-extract --no-profile-pass > $O/pmc_${lib}.log 2>&1 || { echo "pmc $lib failed"; tail -5 $O/pmc_${lib}.log; exit 1; }
  python3 - $O $lib <<'PY'
import sys
sys.path.insert(0, "tools")
from pmc_report import load
o, lib = sys.argv[1], sys.argv[2]
d, _ = load(f"{o}/pmc_{lib}", "FETCH_SIZE")
print(lib, "FETCH", {k: round(sum(v) / len(v) * 2048 / 1e6, 2) for k, v in sorted(d.items()) if k in ("resize",)}, "MB per launch")
PY
done
unset ORBGPU_LIB_PATH
for rep in 1 2; do for lib in tree rsrun2 rsrun8 r6old; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  $T 180 python bench.py --only-extract --steps 200 > $O/c3_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/c3_$lib.txt').read().strip().splitlines()[-1]); print('$lib', round(d['value']/1e6,1), d['kernels_ms_per_step'])"
done; done

# Hamming top-2 occupancy A/B: tree (4 waves x 2 chains, 124 VGPRs, 4 waves/SIMD), t2one (8 waves x 1 chain, 86
# VGPRs, 5 waves/SIMD), t2one6 (the same forced to 6 waves/SIMD, 80 VGPRs), t2two5 (4 x 2 forced to 5 waves/SIMD).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c20; mkdir -p $O
T="timeout -k 10"
for lib in t2one t2one6 t2two5; do
  $T 300 env ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py -k "top2 or hamming" > $O/pytest_$lib.log 2>&1; rc=$?; echo -n "$lib: "; tail -1 $O/pytest_$lib.log; [ $rc -eq 0 ] || exit 1
done
B="--no-cpu --no-stereo --no-host-path --no-bird --no-c4 --no-matcher --steps 30 --warmup 5"
for rep in 1 2; do for lib in tree t2one t2one6 t2two5; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  $T 180 python bench.py $B > $O/b_$lib.txt 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/b_$lib.txt').read().strip().splitlines()[-1]); h=d['hamming']; print('$lib', round(h['matches_per_s']/1e12,3), 'T', h['us_per_launch_wall'], 'us wall', h['kernel_avg_us'], 'us kernel', round(h['mfma_fp4']['frac'],4))"
done; done

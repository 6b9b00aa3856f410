set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c4; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_bench_ranks.py > $O/pytest_ranks.log 2>&1; tail -5 $O/pytest_ranks.log
$T 120 env ORBGPU_FLOW=0 ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_stamps.so python tools/octree_stamps.py 1 4000 > $O/oct_c5b1.txt 2>&1 && cat $O/oct_c5b1.txt

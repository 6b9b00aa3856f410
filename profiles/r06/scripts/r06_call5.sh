set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c5; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flow.py > $O/pytest_flow.log 2>&1; rc=$?; tail -2 $O/pytest_flow.log; [ $rc -eq 0 ] || exit 1
$T 120 env ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_stamps.so python tools/octree_stamps.py 1 4000 > $O/oct_c5b1.txt 2>&1 && cat $O/oct_c5b1.txt

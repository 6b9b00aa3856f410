set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c6; mkdir -p $O
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flow.py > $O/pytest_flow.log 2>&1; rc=$?; tail -2 $O/pytest_flow.log; [ $rc -eq 0 ] || exit 1
$T 120 python tools/flow_stamps.py 1 4000 256 > $O/stamps256.txt 2>&1 && cat $O/stamps256.txt || exit 1
for nb in 64 128 256; do
  $T 180 env ORBGPU_FLOW=1 ORBGPU_FLOW_BLOCKS=$nb python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/c5b1p1_$nb.txt 2>&1 && echo -n "p1 blocks $nb " && tail -1 $O/c5b1p1_$nb.txt | cut -c100-200 || exit 1
  $T 180 env ORBGPU_FLOW=1 ORBGPU_FLOW_BLOCKS=$nb python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5b1p4_$nb.txt 2>&1 && echo -n "p4 blocks $nb " && tail -1 $O/c5b1p4_$nb.txt | cut -c100-200 || exit 1
done

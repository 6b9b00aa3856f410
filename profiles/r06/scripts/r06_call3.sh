set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c3; mkdir -p $O
T="timeout -k 10"
$T 120 python tools/flow_stamps.py 1 4000 64 > $O/stamps64.txt 2>&1 && cat $O/stamps64.txt &&
$T 120 python tools/flow_stamps.py 1 4000 256 > $O/stamps256.txt 2>&1 && cat $O/stamps256.txt &&
for nb in 128 256; do
  $T 180 env ORBGPU_FLOW_BLOCKS=$nb python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/c5b1p1_$nb.txt 2>&1 && echo "p1 blocks $nb" && tail -1 $O/c5b1p1_$nb.txt | cut -c150-300 || exit 1
  $T 180 env ORBGPU_FLOW_BLOCKS=$nb python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5b1p4_$nb.txt 2>&1 && echo "p4 blocks $nb" && tail -1 $O/c5b1p4_$nb.txt | cut -c150-300 || exit 1
done

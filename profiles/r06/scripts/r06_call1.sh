set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c1; mkdir -p $O
timeout -k 10 120 env ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_stamps.so python tools/octree_stamps.py 1 4000 > $O/oct_c5b1.txt 2>&1 && cat $O/oct_c5b1.txt &&
timeout -k 10 120 env ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_stamps.so python tools/octree_stamps.py 64 2000 > $O/oct_c3b64.txt 2>&1 &&
timeout -k 10 180 env ORBGPU_BENCH_ONE_DEVICE=1 python bench.py --gpus 2 --only-extract --steps 5 --config c3 > $O/n2_c3.txt 2>&1 && tail -1 $O/n2_c3.txt | cut -c1-400 &&
timeout -k 10 180 env ORBGPU_BENCH_ONE_DEVICE=1 python bench.py --gpus 2 --only-extract --steps 5 --config c5 > $O/n2_c5.txt 2>&1 && tail -1 $O/n2_c5.txt | cut -c1-400 &&
timeout -k 10 180 python bench.py --config c5 --batch 1 --pipelines 4 --only-extract --steps 400 > $O/c5b1.txt 2>&1 && tail -1 $O/c5b1.txt | cut -c1-300 &&
timeout -k 10 180 python bench.py --config c5 --batch 1 --pipelines 1 --only-extract --steps 400 > $O/c5b1p1.txt 2>&1 && tail -1 $O/c5b1p1.txt | cut -c1-300

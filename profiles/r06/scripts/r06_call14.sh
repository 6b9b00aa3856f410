set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c14; mkdir -p $O
T="timeout -k 10"
for K in 64 256; do $T 120 env ORBGPU_STRIPES=$K ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_stamps.so python tools/stripe_stamps.py > $O/st$K.txt 2>&1; echo "K $K"; tail -2 $O/st$K.txt; done

# octree phase split (kernel stamps build in a scratch copy): one C5 frame, one C3 frame, a 64-frame C3 batch
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/oct; rm -rf /tmp/sb; mkdir -p /tmp/sb
cp -r include orb-slam-birdview_amd /tmp/sb/ && rm -rf /tmp/sb/orb-slam-birdview_amd/build
make -s -C /tmp/sb/orb-slam-birdview_amd -j16 STAMPS=1 liborbgpu.so > gpurun_out/oct/build.log 2>&1 || { tail -20 gpurun_out/oct/build.log; exit 1; }
for a in "1 4000" "1 2000" "64 2000"; do
  echo "== B, nfeatures = $a"
  ORBGPU_LIB_PATH=/tmp/sb/orb-slam-birdview_amd/liborbgpu.so timeout -k 10 120 python3 tools/octree_stamps.py $a || exit 1
done 2>&1 | tee gpurun_out/oct/stamps.txt

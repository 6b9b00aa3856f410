# octree phase-2 ranking on 32-bit keys: the whole GPU suite, C5 one-frame-per-step and host-path timings, stamps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/oct22
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/oct22/pytest_gpu.log 2>&1; rc=$?; tail -1 gpurun_out/oct22/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^FAILED|Error" gpurun_out/oct22/pytest_gpu.log | head; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --config c5 --batch 1 --pipelines 4 --steps 400 --warmup 40 --only-extract > gpurun_out/oct22/c5b1_$i.log 2>&1 || { tail -5 gpurun_out/oct22/c5b1_$i.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/oct22/c5b1_$i.log') if l.startswith('{')][-1]); print('c5b1', d['value'], d['kernels_ms_per_step'])"
done
bash tools/host_quick.sh > gpurun_out/oct22/host.log 2>&1 || { tail -5 gpurun_out/oct22/host.log; exit 1; }
cut -c1-100 gpurun_out/oct22/host.log
rm -rf /tmp/sb; mkdir -p /tmp/sb && cp -r include orb-slam-birdview_amd /tmp/sb/ && rm -rf /tmp/sb/orb-slam-birdview_amd/build
make -s -C /tmp/sb/orb-slam-birdview_amd -j16 STAMPS=1 liborbgpu.so > gpurun_out/oct22/build.log 2>&1 || { tail -20 gpurun_out/oct22/build.log; exit 1; }
ORBGPU_LIB_PATH=/tmp/sb/orb-slam-birdview_amd/liborbgpu.so timeout -k 10 120 python3 tools/octree_stamps.py 1 4000 2>&1 | grep -A3 "level 0" | tee gpurun_out/oct22/stamps.txt

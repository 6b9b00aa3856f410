set -o pipefail
mkdir -p gpurun_out/c11
for v in stag6 stag8 stag10; do
  ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py -k top2 > gpurun_out/c11/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -20 gpurun_out/c11/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c11/pytest_$v.log)"
done
bash tools/gpu_run.sh c11 "ab=tree,ab/liborbgpu_stag6.so,ab/liborbgpu_stag8.so,ab/liborbgpu_stag10.so@--steps 20 --warmup 3 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher"

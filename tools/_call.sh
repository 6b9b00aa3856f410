set -o pipefail
mkdir -p gpurun_out/c7
for v in pipe6 pipe8 pipe10; do
  ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py -k top2 > gpurun_out/c7/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -20 gpurun_out/c7/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c7/pytest_$v.log)"
done
bash tools/gpu_run.sh c7 "ab=tree,ab/liborbgpu_pipe6.so,ab/liborbgpu_pipe8.so,ab/liborbgpu_pipe10.so@--steps 20 --warmup 3 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher"

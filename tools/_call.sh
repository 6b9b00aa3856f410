set -o pipefail
mkdir -p gpurun_out/c4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py -k top2 > gpurun_out/c4/pytest_tree.log 2>&1 || { echo "pytest tree failed"; tail -20 gpurun_out/c4/pytest_tree.log; exit 1; }
echo "tree: $(tail -1 gpurun_out/c4/pytest_tree.log)"
for v in pf2 tps4pf2; do
  ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_matcher.py -k top2 > gpurun_out/c4/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -20 gpurun_out/c4/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c4/pytest_$v.log)"
done
bash tools/gpu_run.sh c4 "ab=tree,ab/liborbgpu_pf2.so,ab/liborbgpu_tps4.so,ab/liborbgpu_tps4pf2.so,ab/liborbgpu_tps1pf2.so@--steps 20 --warmup 3 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher" ham

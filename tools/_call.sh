set -o pipefail
mkdir -p gpurun_out/c9
for v in sc1 sc2 sc3 sc4; do
  ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extract.py -k "small_batch" tests/test_gpu_variants.py > gpurun_out/c9/pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -20 gpurun_out/c9/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/c9/pytest_$v.log)"
done
bash tools/gpu_run.sh c9 "ab=tree,ab/liborbgpu_sc1.so,ab/liborbgpu_sc2.so,ab/liborbgpu_sc3.so,ab/liborbgpu_sc4.so@--config c5 --batch 1 --pipelines 4 --steps 400 --warmup 40 --only-extract"

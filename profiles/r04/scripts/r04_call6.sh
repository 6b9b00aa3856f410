# new GPU tests (mask fixture, vocab -> BoW chain), the matcher tests under each zero-copy mode, then the
# per-call matcher leg under each mode
set -o pipefail
mkdir -p gpurun_out/zc; export TMPDIR=/tmp
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread"
$T tests/test_mask_fixture.py tests/test_gpu_bow_chain.py tests/test_gpu_stereo.py > gpurun_out/zc/pytest_new.log 2>&1; rc=$?; tail -3 gpurun_out/zc/pytest_new.log; [ $rc -eq 0 ] || exit 1
for zc in 1 2; do
  ORBGPU_MATCH_ZC=$zc $T tests/test_gpu_matcher.py tests/test_gpu_bow_chain.py tests/test_matcher_adapter.py tests/test_gpu_vocab.py tests/test_gpu_stereo.py > gpurun_out/zc/pytest_zc$zc.log 2>&1; rc=$?; echo "zc=$zc"; tail -2 gpurun_out/zc/pytest_zc$zc.log; [ $rc -eq 0 ] || exit 1
done
ARGS="--steps 5 --warmup 2 --no-cpu --no-hamming --no-stereo --no-host-path --no-bird --no-c4 --no-profile-pass"
for zc in 0 1 2 0 1 2; do
  ORBGPU_MATCH_ZC=$zc timeout -k 10 200 python3 bench.py $ARGS > gpurun_out/zc/bench_zc$zc.log 2>&1 || { echo "bench zc $zc failed"; tail -5 gpurun_out/zc/bench_zc$zc.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/zc/bench_zc$zc.log') if l.startswith('{')][-1])['matcher']; print('zc=$zc', json.dumps({k: v for k, v in d.items() if k != 'note'}))"
done
# the forked host path: extraction / mirror tests (forked by default), then its latency A/B
$T tests/test_gpu_extract.py tests/test_host_mirror.py tests/test_gpu_variants.py > gpurun_out/zc/pytest_fork.log 2>&1; rc=$?; tail -2 gpurun_out/zc/pytest_fork.log; [ $rc -eq 0 ] || exit 1
ORBGPU_UPLOAD=1 $T tests/test_gpu_extract.py tests/test_host_mirror.py > gpurun_out/zc/pytest_upload.log 2>&1; rc=$?; tail -2 gpurun_out/zc/pytest_upload.log; [ $rc -eq 0 ] || exit 1
bash tools/host_quick.sh ORBGPU_FORK=0 ORBGPU_UPLOAD=1 "ORBGPU_UPLOAD=1 ORBGPU_FORK=0" > gpurun_out/zc/host_fork.log 2>&1 || { tail -5 gpurun_out/zc/host_fork.log; exit 1; }
cat gpurun_out/zc/host_fork.log | cut -c1-200

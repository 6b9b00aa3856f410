# Hamming A/B + profile, then the C5 one-frame-per-step fork A/B
# (archived round-4 record: the tools/r04_*.sh scripts it calls were moved out of tools/ in round 5; not runnable as is)
set -o pipefail
mkdir -p gpurun_out/c7; export TMPDIR=/tmp
bash tools/r04_ham_ab2.sh || exit 1
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread"
ORBGPU_FORK_BATCH=1 $T tests/test_gpu_extract.py tests/test_gpu_variants.py > gpurun_out/c7/pytest_forkbatch.log 2>&1; rc=$?; tail -2 gpurun_out/c7/pytest_forkbatch.log; [ $rc -eq 0 ] || exit 1
for fb in 0 1 0 1; do
  ORBGPU_FORK_BATCH=$fb timeout -k 10 120 python3 bench.py --config c5 --batch 1 --pipelines 4 --steps 400 --warmup 40 --only-extract > gpurun_out/c7/c5b1_fb$fb.log 2>&1 || { echo "c5b1 $fb failed"; tail -5 gpurun_out/c7/c5b1_fb$fb.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c7/c5b1_fb$fb.log') if l.startswith('{')][-1]); print('fork_batch=$fb', d['value'], d['ms_per_step'])"
done

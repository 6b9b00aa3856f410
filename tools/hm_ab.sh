OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 420 python -m pytest tests -q -m gpu -x > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for v in 0 1 0 1; do
  ORBGPU_TOP2_MFMA=$v timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-stereo --no-host-path > $OUT/hm.log 2>&1 || { echo "bench failed"; tail -20 $OUT/hm.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/hm.log').read().strip().splitlines()[-1]); h=d['hamming']; print('mfma=$v', round(h['matches_per_s']/1e12,3), 'T/s', h['kernel_avg_us'], 'us')"
done

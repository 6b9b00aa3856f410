OUT=gpurun_out; mkdir -p $OUT
for b in ${BS:-256 512 1024}; do for p in ${PS:-2 3}; do
  echo -n "B=$b P=$p: "
  timeout -k 10 150 python bench.py --batch $b --pipelines $p --steps 60 --warmup 6 --only-extract > $OUT/bs_${b}_$p.log 2>&1 || { tail -5 $OUT/bs_${b}_$p.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(round(d['value']/1e6,1), d['ms_per_step'], d['kernels_ms_per_step'])" $OUT/bs_${b}_$p.log
done; done

mkdir -p gpurun_out
for P in 2 3 4 2; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --only-extract --no-profile-pass --pipelines $P > gpurun_out/pp$P.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pp$P.log') if l.startswith('{')][-1]); print('P=$P', round(d['value']/1e6,2), d['ms_per_step'])"
done

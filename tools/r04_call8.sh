# fp4 form of the Hamming top-2: the operand-map probe, the matcher GPU tests under the fp4 and lookahead forms,
# the bench Hamming leg per ORBGPU_TOP2 variant, then the profiling passes of the int8 default and of the fp4 form
set -o pipefail
mkdir -p gpurun_out/ab8; export TMPDIR=/tmp
timeout -k 10 60 ./tools/mfma_fp4_probe > gpurun_out/ab8/probe.log 2>&1; rc=$?; cat gpurun_out/ab8/probe.log; [ $rc -eq 0 ] || exit 1
T="timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread"
# host path: the fork / streamed-upload switches (parity), their latency, the matcher leg with per-call input modes
$T tests/test_gpu_extract.py -k "host_path" > gpurun_out/ab8/pytest_host.log 2>&1; rc=$?; echo "host: $(tail -1 gpurun_out/ab8/pytest_host.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ab8/pytest_host.log; exit 1; }
$T tests/test_gpu_matcher.py tests/test_gpu_bow_chain.py tests/test_gpu_vocab.py tests/test_matcher_adapter.py > gpurun_out/ab8/pytest_zcdef.log 2>&1; rc=$?; echo "zc default: $(tail -1 gpurun_out/ab8/pytest_zcdef.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ab8/pytest_zcdef.log; exit 1; }
bash tools/host_quick.sh ORBGPU_UPLOAD=1 ORBGPU_FORK=1 > gpurun_out/ab8/host.log 2>&1 || { tail -5 gpurun_out/ab8/host.log; exit 1; }
cut -c1-160 gpurun_out/ab8/host.log
MA="--steps 5 --warmup 2 --no-cpu --no-hamming --no-stereo --no-host-path --no-bird --no-c4 --no-profile-pass"
timeout -k 10 200 python3 bench.py $MA > gpurun_out/ab8/bench_matcher.log 2>&1 || { tail -5 gpurun_out/ab8/bench_matcher.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab8/bench_matcher.log') if l.startswith('{')][-1])['matcher']; print(json.dumps({k: (v.get('gpu_us'), v.get('cpu_us'), v.get('speedup'), v.get('equal')) for k, v in d.items() if isinstance(v, dict) and 'gpu_us' in v}))"
for v in 8fp 8fpl 8f 81pl; do
  ORBGPU_TOP2=$v $T tests/test_gpu_matcher.py > gpurun_out/ab8/pytest_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/ab8/pytest_$v.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/ab8/pytest_$v.log; exit 1; }
done
ARGS="--steps 50 --warmup 5 --no-cpu --no-host-path --no-stereo --no-bird --no-c4 --no-matcher --no-profile-pass"
for v in 81p 8fp 81pl 8fpl 81pL 8f 81pPl 8fpP 81p 8fp; do
  ORBGPU_TOP2=$v timeout -k 10 120 python3 bench.py $ARGS > gpurun_out/ab8/top2_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/ab8/top2_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab8/top2_$v.log') if l.startswith('{')][-1])['hamming']; m=d.get('mfma_fp4') or d.get('mfma_i8'); print('$v', d['kernel_avg_us'], m['frac'], d['matches_per_s'])"
done
HAM_OUT=gpurun_out/ham_i8 bash tools/ham_prof.sh > gpurun_out/ab8/ham_prof_i8.log 2>&1 || { tail -20 gpurun_out/ab8/ham_prof_i8.log; exit 1; }
ORBGPU_TOP2=8fp HAM_OUT=gpurun_out/ham_fp4 bash tools/ham_prof.sh > gpurun_out/ab8/ham_prof_fp4.log 2>&1 || { tail -20 gpurun_out/ab8/ham_prof_fp4.log; exit 1; }
for f in i8 fp4; do python3 -c "import json; d=json.load(open('gpurun_out/ham_$f/report.json')); print('$f', d.get('trace_mean_us_per_dispatch'), d.get('trace_leg_us'), d.get('frac_from_trace'), d.get('top2_mfma'), d.get('hbm_bytes_per_dispatch'))"; done

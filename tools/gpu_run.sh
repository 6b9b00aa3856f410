#!/bin/bash
# One GPU-box call as a list of steps (the one runner of round 5; round-4's one-off call scripts are kept as
# records under profiles/r04/scripts/).  Usage, from the repo root on the box:
#   bash tools/gpu_run.sh <tag> <step> [<step> ...]
# Output goes to gpurun_out/<tag>/<n>_<step name>.log.  Every step runs under its own time limit and the call
# stops at the first failing step (no retries).  Steps:
#   pytest[=<pytest args>]        the GPU suite (default: all of tests/ -m gpu)
#   smoke                         __graft_entry__.smoke()
#   bench[=<bench.py args>]       one bench line, its JSON summarised
#   ab=<lib>[,<lib>...][@<args>]  bench.py under each liborbgpu build (paths, "tree" = the in-tree one), run twice,
#                                 interleaved (ORBGPU_LIB_PATH)
#   ham                           tools/ham_prof.sh (Hamming leg: trace + PMC passes)
#   pmc                           tools/pmc.sh (extraction kernels: PMC passes)
#   rocprof[=<bench.py args>]     rocprofv3 --kernel-trace --stats of bench.py (default: the timed extraction loop)
#   host                          tools/host_latency on 16 C3 frames (the C++ mirror's per-frame latency)
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
n=0
summ() {   # one bench JSON line -> the numbers worth reading in the gpurun tail
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
h = d.get('hamming') or {}
r = d.get('roofline') or {}
k = d.get('kernels_ms_per_step') or {}
print(f"value {d['value']/1e6:.2f} M/s  ms/step {d['ms_per_step']}  kernels {k}  fast frac {r.get('frac')}",
      f" ham {h.get('kernel_avg_us')} us {(h.get('matches_per_s') or 0)/1e12:.3f} T/s frac {(h.get('mfma_fp4') or {}).get('frac')}"
      if h else "")
m = d.get('matcher') or {}
if m:
    print("matcher", {c: (v.get('gpu_us'), v.get('cpu_us'), v.get('equal')) for c, v in m.items()
                      if isinstance(v, dict) and 'gpu_us' in v})
hp = d.get('host_path') or {}
if hp:
    print("host_path ms", hp.get('ms_per_frame'))
EOF
}
run() {   # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2; n=$((n + 1))
  local log=$OUT/${n}_$name.log
  echo "== $n $name: $*"
  timeout -k 10 $lim "$@" > $log 2>&1; local rc=$?
  echo "rc=$rc" >> $log
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; tail -25 $log; exit 1; fi
  return 0
}
for s in "$@"; do
  case "$s" in
    pytest|pytest=*)
      a=${s#pytest}; a=${a#=}; [ -z "$a" ] && a="tests -m gpu"
      run pytest 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $a
      tail -2 $OUT/${n}_pytest.log | head -1 ;;
    smoke)
      run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"; tail -2 $OUT/${n}_smoke.log | head -1 ;;
    bench|bench=*)
      a=${s#bench}; a=${a#=}
      run bench 600 python bench.py $a; summ $OUT/${n}_bench.log ;;
    ab=*)
      spec=${s#ab=}; libs=${spec%%@*}; a=""; [[ "$spec" == *@* ]] && a=${spec#*@}
      IFS=',' read -ra LS <<< "$libs"
      for rep in 1 2; do
        for lib in "${LS[@]}"; do
          if [ "$lib" = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/$lib; fi
          run ab 300 python bench.py $a; echo -n "  [$lib] "; summ $OUT/${n}_ab.log
        done
      done
      unset ORBGPU_LIB_PATH ;;
    ham)
      run ham 1200 env HAM_OUT=$OUT/ham bash tools/ham_prof.sh; tail -30 $OUT/${n}_ham.log ;;
    pmc)
      run pmc 1200 bash tools/pmc.sh; tail -5 $OUT/${n}_pmc.log ;;
    rocprof|rocprof=*)
      a=${s#rocprof}; a=${a#=}; [ -z "$a" ] && a="--only-extract --no-profile-pass --pipelines 1 --steps 100 --warmup 20"
      run rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$n -o run -- python3 bench.py $a ;;
    host)
      python3 -c "
import sys; sys.path.insert(0,'orb-slam-birdview_amd')
import numpy as np
from orbgpu.synth import bench_frames
open('/tmp/frames.raw','wb').write(np.ascontiguousarray(bench_frames(1280,720,16)).tobytes())
"
      run host 120 ./tools/host_latency /tmp/frames.raw 1280 720 16 2000 300 0; tail -2 $OUT/${n}_host.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0

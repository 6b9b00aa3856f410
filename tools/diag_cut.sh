#!/bin/bash
# Builds liborbgpu variants whose k_fast_wave stops after a phase (ORBGPU_FAST_CUT=1: ROI store, 2: pass-0
# prefilter, 3: pass-0 arc strength; the cell count is written as 0, so the later kernels see no
# candidates) into diag_build/cutN/, and k_describe variants stopping after the window load (d1), IC
# angle (d2) and row pass (d3) into diag_build/cutdN/ — instruction-count diagnostics only, never the product.
set -e
cd "$(dirname "$0")/../orb-slam-birdview_amd"
for n in 1 2 3 d1 d2 d3; do
  case $n in d*) DEF="-DORBGPU_DESC_CUT=${n#d}";; *) DEF="-DORBGPU_FAST_CUT=$n";; esac
  mkdir -p ../diag_build/cut$n
  for f in csrc/*.hip; do
    b=$(basename $f .hip)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
      -mcode-object-version=5 $DEF -c $f -o ../diag_build/cut$n/$b.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -shared -fPIC -o ../diag_build/cut$n/liborbgpu.so ../diag_build/cut$n/*.o
done

#!/bin/bash
# host-path kernel timeline under each liborbgpu.so given (paths; "tree" = in-tree build)
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
for lib in "$@"; do
  if [ "$lib" = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/$lib; fi
  rm -rf $OUT/hp
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/hp -o run -- python3 tools/host_path_trace.py > $OUT/hp.log 2>&1 || exit 1
  echo "== $lib"; python3 tools/timeline.py $OUT/hp 2
done

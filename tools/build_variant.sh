#!/bin/bash
# A/B build of liborbgpu with compile-time switches in ONE translation unit (run here, on the CPU):
#   tools/build_variant.sh <name> <csrc file stem> [-DNAME=VALUE ...]
# compiles csrc/<stem>.hip with the Makefile's flags plus the given defines, links it with the in-tree build's
# other objects and writes ab/liborbgpu_<name>.so (ab/ is git-ignored; it travels to the GPU box, where
# tools/gpu_run.sh "ab=ab/liborbgpu_<name>.so,tree" runs the bench under each).  Nothing in the product reads
# these defines at run time: a variant that wins is made the code, the others are deleted.
set -e
NAME=${1:?name}; STEM=${2:?csrc stem}; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/orb-slam-birdview_amd
make -s -C $PKG liborbgpu.so
mkdir -p $ROOT/ab/obj_$NAME
IFS=',' read -ra STEMS <<< "$STEM"
for st in "${STEMS[@]}"; do
  # the Makefile's own flags for this object (HIPFLAGS + EXTRA_<stem>): variants compile as the library does
  FLAGS=$(make -s -C $PKG --no-print-directory print-flags-$st)
  /opt/rocm/bin/hipcc $FLAGS "$@" -c $PKG/csrc/$st.hip -o $ROOT/ab/obj_$NAME/$st.o
done
# the library's object list from the Makefile (not a glob: a stale object of a deleted source stays out)
OBJS=""
for o in $(make -s -C $PKG --no-print-directory print-objs); do
  b=$(basename $o)
  if [ -f $ROOT/ab/obj_$NAME/$b ]; then OBJS="$OBJS $ROOT/ab/obj_$NAME/$b"; else OBJS="$OBJS $PKG/$o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -shared -fPIC -o $ROOT/ab/liborbgpu_$NAME.so $OBJS
rm -rf $ROOT/ab/obj_$NAME
echo "ab/liborbgpu_$NAME.so"

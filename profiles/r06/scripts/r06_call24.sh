# describe nondeterminism after the sincos rewrite: which change removes it (diagnostic)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c24; mkdir -p $O
for lib in tree biasplain sgprnop r6old; do
  if [ $lib = tree ]; then unset ORBGPU_LIB_PATH; else export ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_$lib.so; fi
  echo "== $lib"; timeout -k 10 300 python -u tools/r06_desc_diag.py > $O/$lib.txt 2>&1 || { tail -5 $O/$lib.txt; exit 1; }
  grep "kps equal" $O/$lib.txt
done

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c23; mkdir -p $O
echo "== tree"; timeout -k 10 300 python -u tools/r06_desc_diag.py 2>&1 | tee $O/tree.txt || exit 1
echo "== r6old"; ORBGPU_LIB_PATH=$PWD/ab/liborbgpu_r6old.so timeout -k 10 300 python -u tools/r06_desc_diag.py 2>&1 | tee $O/r6old.txt

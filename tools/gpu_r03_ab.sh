# A/B of library variants on one box: J.v / smoother / slab-sum launch times (tools/jv_bench.py at 128^3)
# and the configs[2] bench step. Usage: tools/gpu_r03_ab.sh lib1 lib2 ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab.log; rm -f $O
for L in "$@"; do
  echo "== $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O 2>&1 || exit 1
done
for L in "$@"; do
  echo "== bench $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 150 python bench.py --steps 8 --warmup 2 --no-cpu >> $O 2>&1 || exit 1
done

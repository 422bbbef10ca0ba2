# bench-only A/B of library variants (configs[2] step), base first and last (box noise)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/ab_bench.log; rm -f $O
for L in softx_2020_200_amd/libgls_native.so "$@" softx_2020_200_amd/libgls_native.so; do
  echo "== bench $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu >> $O 2>&1 || exit 1
done

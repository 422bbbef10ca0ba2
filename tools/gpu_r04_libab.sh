# A/B of library variants on one box (GLS_NATIVE_LIB): J.v / FP32 smoother / slab-sum / residual launch
# times at 128^3 (tools/jv_bench.py), then the configs[2] bench step. Usage: tools/gpu_r04_libab.sh lib1 ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/libab.log; rm -f $O
for L in "$@"; do
  echo "== $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
for L in "$@"; do
  echo "== bench $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu 2>&1 | grep -v amdgpu.ids | cut -c1-1500 >> $O || exit 1
done
cat $O

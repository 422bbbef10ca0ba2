# A/B of library variants on one box (GLS_NATIVE_LIB): J.v / FP32 smoother / slab-sum / residual launch
# times at 128^3 (tools/jv_bench.py), then the configs[2] bench step (full lines in gpurun_out/libab_*.json).
# Usage: tools/gpu_r04_libab.sh lib1 ...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/libab.log; rm -f $O
for L in "$@"; do
  echo "== $L" >> $O
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 2>&1 | grep -v amdgpu.ids >> $O || exit 1
done
for L in "$@"; do
  B=$(basename $L .so)
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/libab_$B.json 2> gpurun_out/libab_$B.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel_ms']
print('== bench', sys.argv[2], 'ms/step %.2f' % d['ms_per_step'], 'gmres %.1f' % d['linear_iterations_per_step'],
      ' '.join('%s=%.3f' % (n, k[n]) for n in ('jacobian_apply','smoother_jv_f32','slab_sum','residual','diagonal')))" gpurun_out/libab_$B.json $B >> $O || exit 1
done
cat $O

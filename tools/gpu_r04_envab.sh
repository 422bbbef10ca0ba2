# A/B of runtime switches on one box: the configs[2] bench line with each env setting (ms/step, GMRES
# its, kernel times), then cylinder3d with GMRES restart / ILU fill variants. Output gpurun_out/envab.log
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/envab.log; rm -f $O
run() {  # run TAG ENV... -- bench args
  local tag=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 bench.py "$@" > gpurun_out/envab_$tag.json 2> gpurun_out/envab_$tag.err || { echo "FAIL $tag" >> $O; return 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernel_ms',{})
print('%-14s ms/step %7.2f  its %5.1f  %s' % (sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'],
      ' '.join('%s=%.3f' % (n, k[n]) for n in ('jacobian_apply','smoother_jv_f32','slab_sum','residual','diagonal') if n in k)))" gpurun_out/envab_$tag.json $tag >> $O
}
B="--steps 8 --warmup 2 --no-cpu"
VARIANTS=("base X=1" "lupiv GLS_MG_COARSE_SOLVER=lu" "base2 X=1" "lupiv2 GLS_MG_COARSE_SOLVER=lu")
for v in "${VARIANTS[@]}"; do
  set -- $v
  run $1 $2 -- $B || exit 1
done
cat $O

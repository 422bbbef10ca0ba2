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
run base X=1 -- $B || exit 1
run nofirst GLS_MG_NO_FIRST_FUSE=1 -- $B || exit 1
run noreslin GLS_NO_RESLIN=1 -- $B || exit 1
run base2 X=1 -- $B || exit 1
run gj GLS_MG_COARSE_SOLVER=gj -- $B || exit 1
run lunpvt GLS_MG_COARSE_SOLVER=lu_npvt -- $B || exit 1
C="--workload cylinder3d --steps 6 --warmup 2"
run cyl30 X=1 -- $C || exit 1
run cyl60 X=1 -- $C --restart 60 || exit 1
run cyl100 X=1 -- $C --restart 100 || exit 1
cat $O

# octree workload: GMG on the refinement hierarchy vs the multicolor ILU, one box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/octbench.log; rm -f $O
run() {  # TAG -- bench args
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py --workload octree "$@" > gpurun_out/oct_$tag.json 2> gpurun_out/oct_$tag.err || { echo "FAIL $tag" >> $O; tail -20 gpurun_out/oct_$tag.err; return 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-12s ms/step %8.2f  its %6.1f  it/s %6.2f  Mdof/s %6.2f  n_dofs %d  J.v %.3f ms  %s' % (sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'], d['value'], d['mdof_per_s'], d['config']['n_dofs'], d['roofline']['launch_ms'], d['config']['linear_solver']))" gpurun_out/oct_$tag.json $tag >> $O
}
B="--cells 4 --octree-steps ${OCT_STEPS:-3} --steps 5 --warmup 1"
run mg22w6 $B --mg-smooth 2 2 --mg-omega 0.6 || exit 1
run mg11w6 $B --mg-smooth 1 1 --mg-omega 0.6 || exit 1
run mg22w8 $B --mg-smooth 2 2 --mg-omega 0.8 || exit 1
run ilu $B --precond ilu || exit 1
cat $O

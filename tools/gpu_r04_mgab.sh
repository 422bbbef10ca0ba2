# A/B of the V-cycle parameters on the configs[2] bench line (one box): damping, sweeps per level
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/mgab.log; rm -f $O
run() {  # TAG -- bench args
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu "$@" > gpurun_out/mgab_$tag.json 2> gpurun_out/mgab_$tag.err || { echo "FAIL $tag" >> $O; return 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-10s ms/step %7.2f  its %5.1f' % (sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step']))" gpurun_out/mgab_$tag.json $tag >> $O
}
run base || exit 1
run om08 --mg-omega 0.8 || exit 1
run om10 --mg-omega 1.0 || exit 1
run cls1 --mg-coarse-level-sweeps 1 || exit 1
run cls3 --mg-coarse-level-sweeps 3 || exit 1
run fine12 --mg-fine-sweeps 1 2 || exit 1
run fine21 --mg-fine-sweeps 2 1 || exit 1
run sm22 --mg-smooth 2 2 || exit 1
run crs4 --mg-coarsest 4 || exit 1
run base2 || exit 1
cat $O

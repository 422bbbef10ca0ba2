# octree workload, hierarchy down to 2^3: sizes 300k / 1.28M / 2.2M DoFs (GMG), ILU at 1.28M, and a
# rocprofv3 kernel-stats run of the 300k GMG line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/octbench2.log; rm -f $O
run() {  # TAG -- bench args
  local tag=$1; shift
  timeout -k 10 400 python3 bench.py --workload octree "$@" > gpurun_out/oct2_$tag.json 2> gpurun_out/oct2_$tag.err || { echo "FAIL $tag" >> $O; tail -20 gpurun_out/oct2_$tag.err; return 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-12s ms/step %8.2f  its %6.1f  it/s %6.2f  Mdof/s %6.2f  n_dofs %d  J.v %.3f ms  %s' % (sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'], d['value'], d['mdof_per_s'], d['config']['n_dofs'], d['roofline']['launch_ms'], d['config']['linear_solver']))" gpurun_out/oct2_$tag.json $tag >> $O
}
M="--mg-smooth 2 2 --mg-omega 0.6"
run mg4s3 --cells 4 --octree-steps 3 --steps 5 --warmup 1 $M || exit 1
run mg4s4 --cells 4 --octree-steps 4 --steps 5 --warmup 1 $M || exit 1
run mg8s3 --cells 8 --octree-steps 3 --steps 5 --warmup 1 $M || exit 1
run mg4s4v11 --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 1 1 --mg-omega 0.6 || exit 1
run ilu4s4 --cells 4 --octree-steps 4 --steps 2 --warmup 1 --precond ilu || exit 1
cat $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_oct -o oct -- python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 $M > gpurun_out/oct2_prof.json 2> gpurun_out/oct2_prof.err || exit 1
find gpurun_out/prof_oct -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/oct_kernel_stats.csv
python3 -c "
import csv
r=list(csv.DictReader(open('gpurun_out/oct_kernel_stats.csv')))
for x in r[:25]: print(x['Name'][:90], x['Calls'], x['AverageNs'], x['Percentage'])"

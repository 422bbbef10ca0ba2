# round-5 box N: per-cell linearization cache A/B (octree, cylinder3d) without the condensation fold; the
# refined configs[4] problem with Jacobi level smoothing; kernel stats of one refined hierarchy-MG step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
: > gpurun_out/r05n_ab.txt
run() {
  local tag="$1" cfg="$2"; shift 2
  env $cfg timeout -k 10 400 python3 bench.py "$@" --no-pmc --no-cpu > gpurun_out/r05n_tmp.json 2> gpurun_out/r05n_tmp.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$tag $cfg rc $rc" >> gpurun_out/r05n_ab.txt; tail -4 gpurun_out/r05n_tmp.err >> gpurun_out/r05n_ab.txt; return $rc; fi
  cp gpurun_out/r05n_tmp.json "gpurun_out/r05n_$tag.json"
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r05n_tmp.json').read().strip().splitlines()[-1]);print('%-14s %-20s %9.3f ms  its %5.1f  %7.2f it/s  %6.2f Mdof/s  %s DoFs' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'], d['value'], d.get('mdof_per_s', 0), d['config'].get('n_dofs')))" "$tag" "$cfg" >> gpurun_out/r05n_ab.txt
}
OCT="--workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6"
run oct_c0 "GLS_CELL_CACHE=0" $OCT && run oct_c1 "GLS_CELL_CACHE=1" $OCT && run oct_c0b "GLS_CELL_CACHE=0" $OCT && run oct_c1b "GLS_CELL_CACHE=1" $OCT \
  && run cyl_c0 "GLS_CELL_CACHE=0" --workload cylinder3d && run cyl_c1 "GLS_CELL_CACHE=1" --workload cylinder3d \
  && run cyl_r2_hmgj "GLS_CELL_CACHE=1" --workload cylinder3d --cyl-refine 2 --cyl-precond hmg --cyl-smoother jacobi --steps 2 --warmup 1
rc=$?; cat gpurun_out/r05n_ab.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05n_prof_r2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload cylinder3d --cyl-refine 2 --cyl-precond hmg --steps 1 --warmup 0 --no-pmc --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r05n_prof_r2.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05n_prof_r2.err
rc=$?; echo "prof rc $rc"; exit $rc

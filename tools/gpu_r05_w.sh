# round-5 box W: configs[3]'s problem at real size (cylinder_shell refined globally, Q2-Q1 MappingQ2 on every cell)
# with the multigrid on the refinement hierarchy (multicolor ILU(0) smoothing, exact LU on the base mesh); ILU(0)
# for comparison at 1.7 M DoFs
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT

run() {
  local tag="$1"; shift
  timeout -k 10 500 python3 bench.py --workload taylorcouette3d "$@" --no-pmc --no-cpu > gpurun_out/r05w_$tag.json 2> gpurun_out/r05w_$tag.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$tag rc $rc" >> gpurun_out/r05w_tc.txt; tail -4 gpurun_out/r05w_$tag.err >> gpurun_out/r05w_tc.txt; return $rc; fi
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r05w_$tag.json').read().strip().splitlines()[-1]);print('%-10s %10.2f ms  its %5.1f  %6.2f it/s  %6.2f Mdof/s  %s DoFs  setup %.0f s  %s' % (sys.argv[1], d['ms_per_step'], d['linear_iterations_per_step'], d['value'], d['mdof_per_s'], d['config']['n_dofs'], d.get('setup_s', 0), d['config']['linear_solver']))" $tag >> gpurun_out/r05w_tc.txt
}
run r4_hmgc --cyl-refine 3 --cyl-precond hmg --cyl-smoother ilu-coarse --steps 3 --warmup 1 \
  && run r5_hmgc --cyl-refine 4 --cyl-precond hmg --cyl-smoother ilu-coarse --steps 2 --warmup 1
rc=$?; cat gpurun_out/r05w_tc.txt; exit $rc

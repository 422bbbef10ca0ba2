# round-5 box M: A/B of the per-cell linearization cache and the folded hanging-row condensation on the
# octree and cylinder3d lines; the configs[4] problem globally refined (1.0 M / 7.8 M DoFs) with ILU(0) and
# with the multigrid on its refinement hierarchy
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
: > gpurun_out/r05m_ab.txt
run() {  # tag env-settings bench-args...
  local tag="$1" cfg="$2"; shift 2
  env $cfg timeout -k 10 400 python3 bench.py "$@" --no-pmc --no-cpu > gpurun_out/r05m_tmp.json 2> gpurun_out/r05m_tmp.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$tag $cfg rc $rc" >> gpurun_out/r05m_ab.txt; tail -4 gpurun_out/r05m_tmp.err >> gpurun_out/r05m_ab.txt; return $rc; fi
  cp gpurun_out/r05m_tmp.json "gpurun_out/r05m_$tag.json"
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r05m_tmp.json').read().strip().splitlines()[-1]);print('%-14s %-40s %9.3f ms  its %5.1f  %7.2f it/s  %6.2f Mdof/s  %s DoFs' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'], d['value'], d.get('mdof_per_s', 0), d['config'].get('n_dofs')))" "$tag" "$cfg" >> gpurun_out/r05m_ab.txt
}
OCT="--workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6"
run oct_base "GLS_CELL_CACHE=0 GLS_NO_COND_FOLD=1" $OCT && run oct_fold "GLS_CELL_CACHE=0" $OCT && run oct_new "GLS_CELL_CACHE=1" $OCT \
  && run oct_base2 "GLS_CELL_CACHE=0 GLS_NO_COND_FOLD=1" $OCT && run oct_new2 "GLS_CELL_CACHE=1" $OCT \
  && run cyl_base "GLS_CELL_CACHE=0" --workload cylinder3d && run cyl_new "GLS_CELL_CACHE=1" --workload cylinder3d \
  && run cyl_r1_ilu "GLS_CELL_CACHE=1" --workload cylinder3d --cyl-refine 1 --steps 3 --warmup 1 \
  && run cyl_r1_hmg "GLS_CELL_CACHE=1" --workload cylinder3d --cyl-refine 1 --cyl-precond hmg --steps 3 --warmup 1 \
  && run cyl_r2_hmg "GLS_CELL_CACHE=1" --workload cylinder3d --cyl-refine 2 --cyl-precond hmg --steps 2 --warmup 1
rc=$?; cat gpurun_out/r05m_ab.txt; exit $rc

# round-5 box X2: octree line at HEAD (one-pass C v): three bench runs and the kernel stats of one
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r05x2_oct.txt
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05x2_tmp.json 2> gpurun_out/r05x2_tmp.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/r05x2_tmp.err; exit $rc; }
  echo "run $i: $(python3 -c "import json;d=json.loads(open('gpurun_out/r05x2_tmp.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3), 'ms', d['linear_iterations_per_step'], 'its', round(d['value'],2), 'it/s', round(d['mdof_per_s'],1), 'Mdof/s')")" >> gpurun_out/r05x2_oct.txt
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05x2_prof -o oct -- python3 $GRAFT_REPO_ROOT/bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/r05x2_prof.err
rc=$?; echo "prof rc $rc"; cat $GRAFT_REPO_ROOT/gpurun_out/r05x2_oct.txt; exit $rc

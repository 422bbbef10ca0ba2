# round-5 box TCP: kernel stats of configs[3]'s problem at 1.7 M DoFs (taylorcouette3d, --cyl-refine 3, hierarchy multigrid)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05tc_prof -o tc -- python3 $GRAFT_REPO_ROOT/bench.py --workload taylorcouette3d --cyl-refine 3 --cyl-precond hmg --steps 3 --warmup 1 --no-pmc --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r05tc.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05tc.err
rc=$?; echo "prof rc $rc"; exit $rc

# round-5 box X: kernel stats of the octree line (1.28 M DoFs, damped Jacobi + FP32 bricks) at HEAD
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05x_prof -o oct -- python3 $GRAFT_REPO_ROOT/bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r05x_oct.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05x_oct.err
rc=$?; echo "prof rc $rc"; tail -c 600 $GRAFT_REPO_ROOT/gpurun_out/r05x_oct.json; exit $rc

# round-5 box O: hanging / octree / forest / mapped GPU tests after the one-pass C v, then the octree line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_octree_mg.py tests/test_gpu_forest_bricks.py tests/test_gpu_uforest.py tests/test_hanging.py tests/test_gpu_umesh_mg.py tests/test_gpu_dist_general.py tests/test_gpu_dist_mg.py tests/test_kelly.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05o_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05o_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05o_oct$i.json 2> gpurun_out/r05o_oct$i.err
rc=$?; echo "oct rc $rc $(python3 -c "import json;d=json.loads(open('gpurun_out/r05o_oct$i.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['linear_iterations_per_step'])")"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05o_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu --steps 5 --warmup 1 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/r05o_prof.err
echo "prof rc $?"

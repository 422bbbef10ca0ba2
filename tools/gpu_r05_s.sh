# round-5 box S: multigrid / app / distributed tests with multicolor ILU smoothing on every level; octree line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_umesh_mg.py tests/test_gpu_octree_mg.py tests/test_gpu_dist_mg.py tests/test_gpu_app_configs.py tests/test_gpu_app.py tests/test_gpu_solver.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r05s_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05s_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05s_oct.json 2> gpurun_out/r05s_oct.err
rc=$?; echo "oct rc $rc $(python3 -c "import json;d=json.loads(open('gpurun_out/r05s_oct.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['linear_iterations_per_step'])")"
exit $rc

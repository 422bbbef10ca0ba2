# round-5 box P: hanging / octree / forest / mapped GPU tests with the flattened condensation fold, then the
# octree line with the fold off / on
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_octree_mg.py tests/test_gpu_forest_bricks.py tests/test_gpu_uforest.py tests/test_hanging.py tests/test_gpu_umesh_mg.py tests/test_gpu_dist_general.py tests/test_gpu_dist_mg.py tests/test_kelly.py tests/test_gpu_app_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05p_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05p_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
GLS_COND_FOLD=$v timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --mg-smooth 2 2 --mg-omega 0.6 --no-pmc --no-cpu > gpurun_out/r05p_oct$v.json 2> gpurun_out/r05p_oct$v.err
rc=$?; echo "oct fold=$v rc $rc $(python3 -c "import json;d=json.loads(open('gpurun_out/r05p_oct$v.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['linear_iterations_per_step'])")"; [ $rc -ne 0 ] && exit $rc
done
exit 0

# octree multigrid on the GPU: the new tests, then the multigrid / hanging regressions
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  tests/test_gpu_octree_mg.py > gpurun_out/octmg_tests.log 2>&1 || { tail -40 gpurun_out/octmg_tests.log; exit 1; }
grep -E "PASSED|FAILED|octree GMG" gpurun_out/octmg_tests.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_solver.py tests/test_hanging.py > gpurun_out/octmg_regress.log 2>&1 || { tail -40 gpurun_out/octmg_regress.log; exit 1; }
tail -3 gpurun_out/octmg_regress.log

# coarse LU default (unpivoted + pivoted retry): the solver tests, then the bench A/B against the pivoted LU
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_dist.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lu_tests.log 2>&1
rc=$?; echo "tests rc $rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/lu_tests.log | tail -40; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r04_envab.sh

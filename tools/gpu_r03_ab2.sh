# A/B of library variants + GPU parity / full-size tests on the candidate (first argument)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C=$1
GLS_NATIVE_LIB=$PWD/$C timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_solver.py -m gpu > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r03_ab.sh "$@"

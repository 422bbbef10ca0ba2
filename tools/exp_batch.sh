# GPU tests of the smoother path, then bench variants: gpurun_out/exp_<name>.json
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_solver.py -m gpu > gpurun_out/t.log 2>&1 || { echo TESTS_FAIL; exit 1; }
run() { local name=$1; shift; env "$@" timeout -k 10 200 python3 bench.py --steps 3 --no-cpu $BARGS > gpurun_out/exp_$name.json 2> gpurun_out/exp_$name.err || { echo "FAIL $name"; exit 1; }; }
BARGS="" run paired X=1
BARGS="" run unpaired GLS_F32_UNPAIRED=1
BARGS="--mg-smooth 1 0" run v10 X=1
BARGS="--mg-smooth -1 1" run v01 X=1
BARGS="--mg-smooth -1 2" run v02 X=1
echo OK

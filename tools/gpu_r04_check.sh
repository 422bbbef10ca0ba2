# round-4 candidate check on one MI355X: the named tests first (fast feedback), then the full -m gpu
# suite, then the configs[2] bench line. Usage: bash tools/gpu_r04_check.sh [pytest node ids...]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_first.log 2>&1
  rc=$?; echo "first tests rc $rc"; tail -3 gpurun_out/gpu_tests_first.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc $rc"; cat gpurun_out/bench.json | cut -c1-600; exit $rc

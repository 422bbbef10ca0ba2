# round-4 evidence, part 1: the full -m gpu suite and smoke on one MI355X. Usage: bash tools/gpu_r04_final_tests.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-r04g}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/smoke_$T.log; exit 1; }
echo ALL_OK

# round-5 box E: the full -m gpu suite at HEAD (Oseen smoothing default, partial FP32 linearization copy), then
# the default bench line as the driver runs it
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r05e_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/r05e_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r05e_bench.json 2> gpurun_out/r05e_bench.err
rc=$?; echo "bench rc $rc"; exit $rc

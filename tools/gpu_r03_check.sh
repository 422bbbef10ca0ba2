# round-3 candidate check: full -m gpu suite, configs[2] bench line, cylinder3d (configs[4] problem) line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python3 bench.py --workload cylinder3d --steps 5 --warmup 1 > gpurun_out/bench_cyl3d.json 2> gpurun_out/bench_cyl3d.err
rc=$?; echo "cyl3d rc $rc"; exit $rc

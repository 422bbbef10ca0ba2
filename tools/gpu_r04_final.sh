# round-4 evidence run on one MI355X: the full -m gpu suite, smoke, the configs[2] bench line under
# rocprofv3 kernel-trace stats and plain, PMC traffic of the pencil J.v, cylinder3d lines.
# Usage: bash tools/gpu_r04_final.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-r04f}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/smoke_$T.log; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_bench_$T.json 2> gpurun_out/prof_bench_$T.err || { echo PROF_FAIL; exit 1; }
bash tools/pmc_traffic.sh 128 gpurun_out/pmc_traffic_$T > gpurun_out/pmc_traffic_$T.txt 2>&1 || { echo TRAFFIC_FAIL; exit 1; }
timeout -k 10 300 python3 bench.py --workload cylinder3d --steps 10 --warmup 2 > gpurun_out/bench_cyl_$T.json 2> gpurun_out/bench_cyl_$T.err || { echo CYL_FAIL; exit 1; }
cut -c1-400 gpurun_out/bench_$T.json; cut -c1-400 gpurun_out/bench_cyl_$T.json
echo ALL_OK

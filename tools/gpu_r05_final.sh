# round-5 final box: the full -m gpu suite and smoke at HEAD, the default bench line as the driver runs it
# (live PMC traffic passes included), and rocprofv3 kernel stats of the same command (CSV)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r05g_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -2 gpurun_out/r05g_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05g_smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; tail -1 gpurun_out/r05g_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r05g_bench.json 2> gpurun_out/r05g_bench.err
rc=$?; echo "bench rc $rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r05g_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-pmc --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r05g_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05g_prof.err
rc=$?; echo "prof rc $rc"; [ $rc -ne 0 ] && exit $rc
cd $GRAFT_REPO_ROOT && timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --cells 64 --steps 3 --warmup 1 --no-pmc --no-cpu > gpurun_out/r05g_np2.json 2> gpurun_out/r05g_np2.err
rc=$?; echo "np2 rc $rc $(tail -c 400 gpurun_out/r05g_np2.json)"; exit $rc

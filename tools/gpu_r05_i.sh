# round-5 box I: solver / parity tests after the GMRES and line-search copy removal, then bench A/B
# (default vs the fused first pre-sweep with the Oseen smoother) and a kernel trace of the default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_linear_methods.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r05i_tests.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1 0 1; do
  GLS_MG_FIRST_FUSE=$v timeout -k 10 300 python3 bench.py --no-pmc > gpurun_out/r05i_bench_ff$v.json 2> gpurun_out/r05i_bench_ff$v.err
  rc=$?; echo "bench ff=$v rc $rc $(python3 -c "import json;d=json.loads(open('gpurun_out/r05i_bench_ff$v.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['linear_iterations_per_step'])")"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05i_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-pmc --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r05i_trace.json 2> $GRAFT_REPO_ROOT/gpurun_out/r05i_trace.err
rc=$?; echo "trace rc $rc"; exit $rc

# round-5 box B: the new / changed GPU tests, the step budget with the default kernels (trace + PMC), W-cycle A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_app_reference.py \
  "tests/test_gpu_app.py::test_app_periodic_kelly_adaptation_general_mesh" "tests/test_gpu_app.py::test_app_kelly_forest_multigrid" \
  "tests/test_gpu_app.py::test_app_periodic_kelly_adaptation" > gpurun_out/r05b_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r05b_tests.log; [ $rc -ne 0 ] && exit $rc
for G in 1 2; do
  GLS_MG_GAMMA=$G timeout -k 10 200 python3 bench.py --no-cpu --steps 6 --warmup 2 > gpurun_out/r05b_bench_gamma$G.json 2> gpurun_out/r05b_bench_gamma$G.err
  rc=$?; echo "bench gamma=$G rc $rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05b_trace -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --jv-reps 2 > gpurun_out/r05b_trace.json 2> gpurun_out/r05b_trace.err
rc=$?; echo "trace rc $rc"; [ $rc -ne 0 ] && exit $rc
i=0
for CTR in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $CTR -d gpurun_out/r05b_pmc$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --jv-reps 2 > gpurun_out/r05b_pmc$i.json 2> gpurun_out/r05b_pmc$i.err
  rc=$?; echo "pmc $CTR rc $rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

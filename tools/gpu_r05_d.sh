# round-5 box D: Oseen (Picard) smoother operator A/B at configs[2] (GLS_MG_OSEEN), alternating runs, plus the
# solver / multigrid GPU tests with it forced on
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for V in 0 1 0 1; do
  GLS_MG_OSEEN=$V timeout -k 10 200 python3 bench.py --no-cpu --no-pmc --steps 6 --warmup 2 >> gpurun_out/r05d_bench_oseen_$V.json 2>> gpurun_out/r05d_bench_oseen_$V.err
  rc=$?; echo "bench oseen=$V rc $rc"; [ $rc -ne 0 ] && exit $rc
done
GLS_MG_OSEEN=1 timeout -k 10 200 python3 bench.py --no-cpu --no-pmc --cells 64 --k 1 --kp 1 --nu 1 --scheme steady --steps 6 --warmup 2 > gpurun_out/r05d_bench_q1_oseen1.json 2> gpurun_out/r05d_bench_q1_oseen1.err
rc=$?; echo "q1 oseen rc $rc"; [ $rc -ne 0 ] && exit $rc
GLS_MG_OSEEN=0 timeout -k 10 200 python3 bench.py --no-cpu --no-pmc --cells 64 --k 1 --kp 1 --nu 1 --scheme steady --steps 6 --warmup 2 > gpurun_out/r05d_bench_q1_oseen0.json 2> gpurun_out/r05d_bench_q1_oseen0.err
rc=$?; echo "q1 newton rc $rc"; [ $rc -ne 0 ] && exit $rc
GLS_MG_OSEEN=1 timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_solver.py tests/test_gpu_dist.py > gpurun_out/r05d_tests_oseen.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/r05d_tests_oseen.log; exit $rc

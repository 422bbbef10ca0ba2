# round-5 first box: pair-kernel A/B (jv_bench + bench), launcher-less N=2 (gloo, one GPU), kernel trace +
# PMC FETCH/WRITE passes of the bench step (tools/step_budget.py), then the full -m gpu suite
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for P in 1 0; do
  GLS_PENCIL_PAIR=$P timeout -k 10 120 python3 tools/jv_bench.py 128 20 > gpurun_out/r05a_jv_pair$P.txt 2>&1
  rc=$?; echo "jv pair=$P rc $rc"; [ $rc -ne 0 ] && exit $rc
  GLS_PENCIL_PAIR=$P timeout -k 10 200 python3 bench.py --no-cpu --steps 6 --warmup 2 > gpurun_out/r05a_bench_pair$P.json 2> gpurun_out/r05a_bench_pair$P.err
  rc=$?; echo "bench pair=$P rc $rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --cells 64 --steps 2 --warmup 1 --no-cpu > gpurun_out/r05a_np2.json 2> gpurun_out/r05a_np2.err
rc=$?; echo "np2 rc $rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05a_trace -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --jv-reps 2 > gpurun_out/r05a_trace.json 2> gpurun_out/r05a_trace.err
rc=$?; echo "trace rc $rc"; [ $rc -ne 0 ] && exit $rc
i=0
for CTR in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $CTR -d gpurun_out/r05a_pmc$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --jv-reps 2 > gpurun_out/r05a_pmc$i.json 2> gpurun_out/r05a_pmc$i.err
  rc=$?; echo "pmc $CTR rc $rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r05a_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/r05a_gpu_tests.log; exit $rc

# round-5 box C: the default bench line as the driver runs it (live PMC traffic passes, CPU baseline), and the
# 16-byte Gram-Schmidt kernels A/B (GLS_VEC16)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
SECONDS=0
timeout -k 10 600 python3 bench.py > gpurun_out/r05c_bench_default.json 2> gpurun_out/r05c_bench_default.err
rc=$?; echo "bench default rc $rc in ${SECONDS}s"; [ $rc -ne 0 ] && exit $rc
for V in 0 1 0 1; do
  GLS_VEC16=$V timeout -k 10 200 python3 bench.py --no-cpu --no-pmc --steps 6 --warmup 2 >> gpurun_out/r05c_bench_vec16_$V.json 2>> gpurun_out/r05c_bench_vec16_$V.err
  rc=$?; echo "bench vec16=$V rc $rc"; [ $rc -ne 0 ] && exit $rc
done
GLS_VEC16=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05c_trace16 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-pmc --jv-reps 2 > gpurun_out/r05c_trace16.json 2> gpurun_out/r05c_trace16.err
rc=$?; echo "trace16 rc $rc"; exit $rc

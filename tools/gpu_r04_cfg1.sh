# configs[1] (Q1-Q1 64^3 steady) bench line with the measured CPU Newton on the job's 16 threads and on
# 1 thread (--cpu-full --cpu-full-1core); heartbeat so the long host legs are not taken for a hang
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1100 python3 bench.py --cells 64 --k 1 --kp 1 --nu 1 --scheme steady --steps 10 --warmup 3 --cpu-full --cpu-full-1core \
    > gpurun_out/bench_q1_64_cpufull1.json 2> gpurun_out/bench_q1_64_cpufull1.err || { echo FAIL; tail -5 gpurun_out/bench_q1_64_cpufull1.err; exit 1; }
cut -c1-600 gpurun_out/bench_q1_64_cpufull1.json

# round-3 counters + traffic at HEAD, and the configs[1] line with its measured CPU Newton
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
bash tools/pmc_r03.sh > gpurun_out/pmc_r03.txt 2>&1 || { echo PMC_FAIL; exit 1; }
bash tools/pmc_traffic.sh 128 gpurun_out/pmc_traffic > gpurun_out/pmc_traffic.txt 2>&1 || { echo TRAFFIC_FAIL; exit 1; }
timeout -k 10 600 python3 bench.py --cells 64 --k 1 --kp 1 --nu 1 --scheme steady --steps 10 --warmup 3 --cpu-full > gpurun_out/bench_q1_64.json 2> gpurun_out/bench_q1_64.err || { echo Q1_FAIL; exit 1; }
echo ALL_OK

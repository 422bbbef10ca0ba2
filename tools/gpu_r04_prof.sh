# round-4 evidence on one MI355X: kernel-trace stats of the configs[2] bench, the pencil / brick kernel
# counters (tools/pmc_r04.sh) and their HBM traffic (tools/pmc_traffic.sh). Usage: bash tools/gpu_r04_prof.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-r04}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_bench_$T.json 2> gpurun_out/prof_bench_$T.err || { echo PROF_FAIL; exit 1; }
bash tools/pmc_r04.sh gpurun_out/pmc_$T > gpurun_out/pmc_$T.txt 2>&1 || { echo PMC_FAIL; exit 1; }
bash tools/pmc_traffic.sh 128 gpurun_out/pmc_traffic_$T > gpurun_out/pmc_traffic_$T.txt 2>&1 || { echo TRAFFIC_FAIL; exit 1; }
cat gpurun_out/pmc_$T.txt gpurun_out/pmc_traffic_$T.txt
echo ALL_OK

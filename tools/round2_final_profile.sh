#!/bin/bash
# Round-2 HEAD measurement on one MI355X: PMC HBM traffic of the J.v kernels (separate passes),
# rocprofv3 kernel stats of the bench, then the default bench line (with the CPU baseline)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_traffic.sh 128 gpurun_out/pmc_traffic_r02 > gpurun_out/pmc_r02.txt 2>&1 || { echo PMC_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_prof_r02.json 2> gpurun_out/bench_prof_r02.err || { echo PROF_FAIL; exit 1; }
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK

set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
bash tools/pmc_traffic.sh 128 gpurun_out/pmc_traffic > gpurun_out/pmc.txt 2>&1 || { echo PMC_FAIL; exit 1; }
cp gpurun_out/pmc.txt profiles/r01_pmc_traffic_jvq_128.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo PROF_FAIL; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK

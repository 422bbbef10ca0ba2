# counters + HBM traffic of the brick kernels at HEAD (after the two-test-field J.v integration)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/pmc_r03.sh > gpurun_out/pmc_r03.txt 2>&1 || { echo PMC_FAIL; exit 1; }
bash tools/pmc_traffic.sh 128 gpurun_out/pmc_traffic > gpurun_out/pmc_traffic.txt 2>&1 || { echo TRAFFIC_FAIL; exit 1; }
echo ALL_OK

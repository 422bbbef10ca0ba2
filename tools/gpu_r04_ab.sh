# round-4 A/B on one box: J.v / FP32 smoother / slab-sum launch times at 128^3 for the lane-per-point
# vs pencil brick kernels and the CSR vs structured slab sums, then the bench step with each default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
for cfg in "GLS_PENCIL=0 GLS_SLAB_CSR=1" "GLS_PENCIL=1 GLS_SLAB_CSR=1" "GLS_PENCIL=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python3 tools/jv_bench.py 128 20 || exit 1
done 2>&1 | tee gpurun_out/ab_jv.txt
for cfg in "GLS_PENCIL=0 GLS_SLAB_CSR=1" "GLS_PENCIL=1"; do
  echo "== bench $cfg"
  env $cfg timeout -k 10 240 python3 bench.py --no-cpu --steps 10 --warmup 3 | cut -c1-900 || exit 1
done 2>&1 | tee gpurun_out/ab_bench.txt

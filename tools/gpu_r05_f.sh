# round-5 box F: the replica-hierarchy multigrid across ranks (2 / 3 gloo ranks on the one GPU)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu_dist_mg.py -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/r05f_dist_mg.log 2>&1
rc=$?; echo "dist mg rc $rc"; tail -5 gpurun_out/r05f_dist_mg.log; exit $rc

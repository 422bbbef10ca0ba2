# round-5 box G: replica-hierarchy multigrid across ranks (library tests + the app at --np 4 --precond hmg)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_app_configs.py -m gpu -k "hierarchy or pipeline" -v -s --timeout 600 --timeout-method thread > gpurun_out/r05g_dist_mg.log 2>&1
rc=$?; echo "dist mg rc $rc"; tail -5 gpurun_out/r05g_dist_mg.log; exit $rc

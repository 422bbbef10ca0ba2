# Gram-corrected single-pass Gram-Schmidt (default) vs CGS2 + DGKS (GLS_GMRES_CGS2=1): full -m gpu suite on
# the default, then configs[2] and cylinder3d lines for both on the same box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_gs.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/gpu_tests_gs.log; [ $rc -ne 0 ] && exit $rc
O=gpurun_out/gs_ab.log; rm -f $O
for V in 0 1 0; do
  echo "== GLS_GMRES_CGS2=$V" >> $O
  GLS_GMRES_CGS2=$V timeout -k 10 200 python3 bench.py --no-cpu --steps 6 --warmup 2 >> $O 2>&1 || exit 1
  GLS_GMRES_CGS2=$V timeout -k 10 150 python3 bench.py --workload cylinder3d --steps 5 --warmup 1 >> $O 2>&1 || exit 1
done
echo ALL_OK

# batched ILU probing + multicolor factorization kernel: ILU / app / adaptive GPU tests, then the
# cylinder3d line and the configs[4]-problem app log
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 800 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_ilu.py tests/test_gpu_dist_general.py tests/test_gpu_app_configs.py tests/test_gpu_app.py tests/test_gpu_uforest.py -m gpu > gpurun_out/ilu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ilu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --workload cylinder3d --steps 3 --warmup 1 > gpurun_out/bench_cyl3d.json 2> gpurun_out/bench_cyl3d.err
rc=$?; echo "cyl3d rc $rc"; [ $rc -ne 0 ] && exit $rc
cd apps/cases && GLS_ILU_VERBOSE=1 timeout -k 10 300 ../gls_navier_stokes_3d cylinder3d_q2q1_re200.prm > ../../gpurun_out/app_cyl3d.log 2>&1
rc=$?; echo "app rc $rc"; exit $rc

# ILU factorization kernel iteration: ILU GPU tests, configs[4]-problem app log, cylinder3d line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ilu.py -m gpu > gpurun_out/ilu_tests3.log 2>&1
rc=$?; tail -2 gpurun_out/ilu_tests3.log; [ $rc -ne 0 ] && exit $rc
cd apps/cases && GLS_ILU_VERBOSE=1 timeout -k 10 300 ../gls_navier_stokes_3d cylinder3d_q2q1_re200.prm > ../../gpurun_out/app_cyl3d3.log 2>&1
rc=$?; echo "app rc $rc"; [ $rc -ne 0 ] && exit $rc
cd ../.. && timeout -k 10 200 python3 bench.py --workload cylinder3d --steps 3 --warmup 1 > gpurun_out/bench_cyl3d3.json 2> gpurun_out/bench_cyl3d3.err
rc=$?; echo "cyl3d rc $rc"; exit $rc

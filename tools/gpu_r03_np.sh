# round-3: enclosed-flow distributed Newton test, then the app's --np pipelines (configs[3] np 4,
# configs[4] np 2) with progress logs
set -o pipefail
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 500 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_gpu_dist_general.py -k enclosed > gpurun_out/tests_encl.log 2>&1
rc=$?; echo "enclosed rc $rc"; [ $rc -gt 1 ] && exit $rc
export GLS_APP_TIMEOUT=400 GLS_NP_WATCHDOG=45
timeout -k 10 1000 python -u -m pytest -v --timeout 900 --timeout-method thread "tests/test_gpu_app_configs.py::test_configs3_taylor_couette3d_kelly_pipeline[4]" "tests/test_gpu_app_configs.py::test_configs4_cylinder3d_re200_bdf2_kelly_pipeline[2]" --basetemp=gpurun_out/np_tmp > gpurun_out/tests_np.log 2>&1
rc=$?; echo "np rc $rc"; rm -rf gpurun_out/np_tmp/*/dump gpurun_out/np_tmp/*/*.vtu; exit $rc

# round-3: the app's --np pipelines (configs[4] np 2, configs[3] np 4) with progress logs
set -o pipefail
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
export GLS_APP_TIMEOUT=300 GLS_NP_WATCHDOG=45
timeout -k 10 700 python -u -m pytest -v --timeout 650 --timeout-method thread "tests/test_gpu_app_configs.py::test_configs4_cylinder3d_re200_bdf2_kelly_pipeline[2]" "tests/test_gpu_app_configs.py::test_configs4_cylinder3d_re200_bdf2_kelly_pipeline[1]" --basetemp=gpurun_out/np_tmp > gpurun_out/tests_np.log 2>&1
rc=$?; echo "np rc $rc"; rm -rf gpurun_out/np_tmp/*/dump gpurun_out/np_tmp/*/*.vtu; exit $rc

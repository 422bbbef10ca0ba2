# round-3 batch 3: ILU tests, e2 distributed general-mesh test, app reference cases, configs pipelines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ilu.py tests/test_gpu_dist_general.py > gpurun_out/tests_b3a.log 2>&1
rc=$?; echo "ilu+dist rc $rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_app_reference.py tests/test_gpu_app_configs.py > gpurun_out/tests_b3b.log 2>&1
rc=$?; echo "app rc $rc"; [ $rc -gt 1 ] && exit $rc
bash tools/gpu_r03_ilublk.sh multicolor:0 || exit 1

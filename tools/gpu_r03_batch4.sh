# round-3 batch 4: e2 (general meshes across ranks): operator test + the app's --np pipelines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_dist_general.py > gpurun_out/tests_b4a.log 2>&1
rc=$?; echo "dist general rc $rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_app_configs.py > gpurun_out/tests_b4b.log 2>&1
rc=$?; echo "configs rc $rc"; exit $rc

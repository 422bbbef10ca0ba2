set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ilu.py tests/test_native_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ilu_tests.log 2>&1 || exit 1
bash tools/gpu_r02_apps.sh

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ilu.py > gpurun_out/ilu.log 2>&1
echo "ilu rc $?"
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_app_reference.py > gpurun_out/appref.log 2>&1
echo "appref rc $?"

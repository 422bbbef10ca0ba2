# round-3 batch 2: ILU tests (multicolor / blocks), adaptive configs pipeline tests, cylinder ILU orderings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_ilu.py > gpurun_out/tests_ilu.log 2>&1
rc=$?; echo "ilu tests rc $rc"; [ $rc -gt 1 ] && exit $rc
bash tools/gpu_r03_ilublk.sh multicolor:0 cm:0 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_app_configs.py > gpurun_out/tests_configs.log 2>&1
rc=$?; echo "configs tests rc $rc"; exit $rc

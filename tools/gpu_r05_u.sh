# round-5 box U: app tests after method = amg -> hierarchy multigrid for every order and configs[3]'s prm on amg
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_app_configs.py tests/test_gpu_app.py tests/test_gpu_app_reference.py tests/test_configs0_cavity.py -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r05u_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05u_tests.log; grep -a "GMRES totals" gpurun_out/r05u_tests.log; exit $rc

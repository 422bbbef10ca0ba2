#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests/test_hanging.py tests/test_gpu_rccl.py tests/test_gpu_app.py tests/test_gpu_app_reference.py tests/test_gpu_ilu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/apptests.log 2>&1 || exit $?
bash tools/gpu_r02_apps.sh

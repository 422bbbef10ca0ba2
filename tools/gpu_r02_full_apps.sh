#!/bin/bash
# Full GPU suite, then the BASELINE configs / reference examples through the application.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?
echo "pytest rc=$rc" > gpurun_out/full.log
[ $rc -gt 1 ] && exit $rc
bash tools/gpu_r02_apps.sh

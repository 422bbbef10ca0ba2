#!/bin/bash
# multi-level Kelly: face-piece kernel vs oracle, app pipeline (refine + coarsen + smoothing) vs oracle
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests/test_kelly.py tests/test_gpu_app.py -m gpu -x -v -k "kelly" --timeout 300 --timeout-method thread > gpurun_out/kelly_tests.log 2>&1

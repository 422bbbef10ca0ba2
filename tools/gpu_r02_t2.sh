#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02t2; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_solver.py tests/test_gpu_dist.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python3 bench.py --steps 3 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json

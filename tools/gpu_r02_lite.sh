#!/bin/bash
# Lite J.v linearization (tau, R_s cached; u, grad u re-derived): parity tests, J.v A/B against the
# padded-line LDS layout (default) vs the round-2 baseline (tools/ab/libgls_r0.so) and padded + lite (tools/ab/libgls_r1.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
stop() { echo "step '$1' ended with $2" >> $O/lite.log; exit $2; }
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "parity or fullsize or golden or solver or mapped" > $O/lite_tests.log 2>&1 || stop pytest $?
for L in softx_2020_200_amd/libgls_native.so tools/ab/libgls_r0.so tools/ab/libgls_r1.so; do
  echo "== $L" >> $O/lite_jv.log
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O/lite_jv.log 2>&1 || stop jv_bench $?
done
for L in softx_2020_200_amd/libgls_native.so tools/ab/libgls_r0.so tools/ab/libgls_r1.so; do
  echo "== $L" >> $O/lite_bench.log
  GLS_NATIVE_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu >> $O/lite_bench.log 2>&1 || stop bench $?
done
echo done >> $O/lite.log

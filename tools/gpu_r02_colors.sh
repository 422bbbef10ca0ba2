#!/bin/bash
# Colored brick launches (GLS_BRICK_COLORS=1; build the library with EXTRA=-DGLS_BRICK_COLORS_BUILD, the
# path is compiled out by default) vs the default slab + k_slab_sum path: full GPU suite,
# J.v microbench and bench for both.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out
mkdir -p $O
cd $R
stop() { echo "step '$1' ended with $2" >> $O/colors.log; exit $2; }
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/colors_tests.log 2>&1 || stop pytest $?
for V in GLS_BRICK_COLORS=1 X=1; do
  echo "== $V" >> $O/colors_jv.log
  env $V timeout -k 10 120 python tools/jv_bench.py 128 20 >> $O/colors_jv.log 2>&1 || stop jv_bench $?
done
for V in GLS_BRICK_COLORS=1 X=1; do
  echo "== $V" >> $O/colors_bench.log
  env $V timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu >> $O/colors_bench.log 2>&1 || stop bench $?
done
echo done >> $O/colors.log

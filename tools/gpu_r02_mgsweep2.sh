#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02m2; mkdir -p $OUT
run() {
  local name=$1; shift
  echo "== $name $*" >> $OUT/summary.txt
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu --steps 3 $BARGS > $OUT/$name.log 2>&1 || return 1
  grep -o '"ms_per_step": [0-9.]*\|"linear_iterations_per_step": [0-9.]*' $OUT/$name.log | tr '\n' ' ' >> $OUT/summary.txt
  grep "getri done\|direct solve" $OUT/$name.log | tail -1 >> $OUT/summary.txt
  echo >> $OUT/summary.txt
}
BARGS="--mg-coarsest 2" run gj GLS_MG_LSWEEPS=5:4:4 GLS_MG_VERBOSE=1 || exit 1
BARGS="--mg-coarsest 2" run lu GLS_MG_LSWEEPS=5:4:4 GLS_MG_VERBOSE=1 GLS_MG_COARSE_SOLVER=lu || exit 1
BARGS="--mg-coarsest 2" run lunp GLS_MG_LSWEEPS=5:4:4 GLS_MG_VERBOSE=1 GLS_MG_COARSE_SOLVER=lu_npvt || exit 1
BARGS="--mg-coarsest 2" run lunp_l5_2 GLS_MG_LSWEEPS=5:2:2 GLS_MG_VERBOSE=1 GLS_MG_COARSE_SOLVER=lu_npvt || exit 1
BARGS="--mg-coarsest 2" run lunp_l5_8 GLS_MG_LSWEEPS=5:8:8 GLS_MG_VERBOSE=1 GLS_MG_COARSE_SOLVER=lu_npvt || exit 1
cat $OUT/summary.txt

#!/bin/bash
# V-cycle coarse-level experiments at Q2 128^3: exact 2^3-cell coarsest solve + per-level sweeps.
set -o pipefail
OUT=gpurun_out/r02m; mkdir -p $OUT
run() { # name env... -- args
  local name=$1; shift
  echo "== $name $*" >> $OUT/summary.txt
  env "$@" timeout -k 10 200 python3 bench.py --no-cpu --steps 3 $BARGS > $OUT/$name.log 2>&1 || return 1
  grep -o '"ms_per_step": [0-9.]*\|"linear_iterations_per_step": [0-9.]*' $OUT/$name.log | tr '\n' ' ' >> $OUT/summary.txt
  echo >> $OUT/summary.txt
}
BARGS="" run base GLS_X=0 || exit 1
BARGS="--mg-coarsest 2" run c2_plain GLS_X=0 || exit 1
BARGS="--mg-coarsest 2" run c2_l5_4 GLS_MG_LSWEEPS=5:4:4 || exit 1
BARGS="--mg-coarsest 2" run c2_l5_8_l4_2 GLS_MG_LSWEEPS=5:8:8,4:2:2 || exit 1
BARGS="--mg-coarsest 2" run c2_l5_16_l4_4 GLS_MG_LSWEEPS=5:16:16,4:4:4 || exit 1
BARGS="--mg-coarsest 2" run c2_l5_30 GLS_MG_LSWEEPS=5:30:30 || exit 1
BARGS="--mg-coarsest 2" run c2_l5_30_l4_4_l3_2 GLS_MG_LSWEEPS=5:30:30,4:4:4,3:2:2 || exit 1
cat $OUT/summary.txt

#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02m3; mkdir -p $OUT; rm -f $OUT/summary.txt
run() {
  local name=$1; shift
  echo "== $name $*" >> $OUT/summary.txt
  timeout -k 10 200 python3 bench.py --no-cpu --steps 3 "$@" > $OUT/$name.log 2>&1 || return 1
  grep -o '"ms_per_step": [0-9.]*\|"linear_iterations_per_step": [0-9.]*' $OUT/$name.log | tr '\n' ' ' >> $OUT/summary.txt
  echo >> $OUT/summary.txt
}
run f01 --mg-fine-sweeps 0 1 || exit 1
run f02 --mg-fine-sweeps 0 2 || exit 1
run f01_w10 --mg-fine-sweeps 0 1 --mg-omega 1.0 || exit 1
run f10 --mg-fine-sweeps 1 0 || exit 1
run c1 --mg-coarse-level-sweeps 1 || exit 1
run c4 --mg-coarse-level-sweeps 4 || exit 1
run w08 --mg-omega 0.8 || exit 1
run w10 --mg-omega 1.0 || exit 1
cat $OUT/summary.txt

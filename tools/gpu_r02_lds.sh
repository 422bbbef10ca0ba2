#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02lds; mkdir -p $OUT; rm -f $OUT/summary.txt
for v in A B C D; do
  GLS_NATIVE_LIB=tools/exp_libgls_$v.so timeout -k 10 200 python3 tools/jv_bench.py 128 20 > $OUT/$v.log 2>&1 || exit 1
  echo "$v $(grep 'n=128' $OUT/$v.log)" >> $OUT/summary.txt
done
cat $OUT/summary.txt

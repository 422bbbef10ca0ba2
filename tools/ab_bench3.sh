#!/bin/bash
# A/B/C of library builds on one box (GLS_NATIVE_LIB overrides; "-" = the in-tree library), twice each
set -e
out=$1; shift
mkdir -p $out
for r in 1 2; do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    if [ "$lib" = "-" ]; then
      timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $out/v${i}_$r.json 2> $out/v${i}_$r.err
    else
      GLS_NATIVE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $out/v${i}_$r.json 2> $out/v${i}_$r.err
    fi
  done
done

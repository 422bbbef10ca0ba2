#!/bin/bash
# A/B of two library builds on one box: bench lines (kernel ms) alternating A, B, A, B
set -e
A=$1; B=$2; out=${3:-gpurun_out/ab}
mkdir -p $out
for r in 1 2; do
  GLS_NATIVE_LIB=$A timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $out/A$r.json 2> $out/A$r.err
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $out/B$r.json 2> $out/B$r.err
done

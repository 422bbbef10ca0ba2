#!/bin/bash
# A/B of an old tree (tools/ab_C: git archive of an earlier commit with its own built library) against
# the current tree on one box: bench lines alternating old, new
set -e
old=$1; out=${2:-gpurun_out/abt}
mkdir -p $out
for r in 1 2; do
  (cd $old && timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu) > $out/C$r.json 2> $out/C$r.err
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $out/H$r.json 2> $out/H$r.err
done

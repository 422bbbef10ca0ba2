#!/bin/bash
# Coarsest-level experiments at Q2 128^3 (bench.py) + residual/linearization PMC passes.
set -o pipefail
OUT=gpurun_out/r02c; mkdir -p $OUT
export GLS_MG_VERBOSE=1
timeout -k 10 240 python3 bench.py --no-cpu --steps 3 --mg-coarse-direct 1 > $OUT/direct_lu.log 2>&1 || exit 1
GLS_MG_COARSE_SOLVER=lu_npvt timeout -k 10 240 python3 bench.py --no-cpu --steps 3 --mg-coarse-direct 1 > $OUT/direct_lu_npvt.log 2>&1 || exit 1
unset GLS_MG_VERBOSE
bash tools/pmc_jv.sh 128 $OUT/pmc > $OUT/pmc.txt 2>&1 || exit 1

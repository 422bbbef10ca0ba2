#!/bin/bash
# Multigrid cycle parameters at the bench workload (Q2 128^3): nonlinear it/s per setting.
# MG_SWEEP="pre post omega coarse_sweeps coarse_omega coarsest|..."
O=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out
mkdir -p $O
IFS="|" read -r -a CFGS <<< "${MG_SWEEP:-1 1 0.9 100 0.7 4}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  echo "pre=$1 post=$2 omega=$3 coarse=$4 comega=$5 coarsest=$6" >> $O/mg_sweep.log
  timeout -k 10 240 python bench.py --steps 2 --warmup 1 --no-cpu --jv-reps 2 --mg-smooth $1 $2 --mg-omega $3 \
      --mg-coarse-sweeps $4 --mg-coarse-omega $5 --mg-coarsest $6 >> $O/mg_sweep.log 2>> $O/mg_sweep.err || exit $?
done

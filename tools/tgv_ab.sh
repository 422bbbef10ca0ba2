#!/bin/bash
# the reference's taylor-green-vortex_gls_sdirk2 case through the app of older trees (tools/ab_T,
# tools/ab_U) and of HEAD: solver statistics
set -e
out=${1:-gpurun_out/tgv_ab}
mkdir -p $out
sed -e "s/set output frequency *= *1 /set output frequency = 1000000 /" -e "s/verbosity *= *quiet/verbosity = verbose/" tests/golden/app_cases/taylor-green-vortex_gls_sdirk2.prm > $out/case.prm
cd $out
for t in T new; do
  app=../../apps/gls_navier_stokes_2d; case $t in T*) app=../../tools/ab_T/apps/gls_navier_stokes_2d;; esac
  GLS_ILU_VERBOSE=1 timeout -k 10 200 stdbuf -oL $app --stats case.prm > $t.log 2>&1 || echo "$t exit $?"
  echo "$t: $(grep newton_iterations $t.log)"
done

#!/bin/bash
# BASELINE configs[3] / configs[4] with local (Kelly) adaptation through the drop-in application
# (line-buffered stdout so progress reaches the log as it happens)
set -e
out=${1:-gpurun_out/amr}
which=${2:-all}
mkdir -p $out
cp apps/cases/*.prm apps/cases/*.msh $out/
cd $out
if [ "$which" != "cylinder" ]; then
  timeout -k 10 400 stdbuf -oL ../../apps/gls_navier_stokes_3d --stats taylor-couette3d_q2q1_kelly.prm > taylor-couette3d-kelly.log 2>&1
fi
if [ "$which" != "couette" ]; then
  timeout -k 10 900 stdbuf -oL ../../apps/gls_navier_stokes_3d --stats cylinder3d_q2q1_re200_kelly.prm > cylinder3d-re200-kelly.log 2>&1
fi

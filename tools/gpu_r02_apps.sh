#!/bin/bash
# BASELINE configs through the drop-in application (apps/gls_navier_stokes_{2d,3d} <prm>):
# configs[2] trajectory (3D cavity Q2 128^3 BDF2, 5 steps), configs[1] (Q1 64^3 steady), the reference's
# examples 01-cavity and 02-taylor-couette (2D) as shipped, and the authored 3D Taylor-Couette (configs[3]).
# Each run has its own time limit; an abort / segfault / timeout ends the script.
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/apps
mkdir -p $O
cd $O
run() {  # name dim prm [extra]
  local name=$1 dim=$2 prm=$3; shift 3
  local t0=$(date +%s.%N)
  timeout -k 10 ${TLIM:-400} $R/apps/gls_navier_stokes_${dim}d "$@" $prm > $O/$name.log 2>&1
  local rc=$?
  rm -f $O/*.vtu $O/*.pvtu $O/*.pvd
  echo "$name rc=$rc wall_s=$(echo "$(date +%s.%N) - $t0" | bc)" >> $O/summary.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
}
cp $R/tests/golden/app_cases/example-0*.prm $R/apps/cases/*.prm $R/apps/cases/*.msh $O/
TLIM=300 run example-01-cavity 2 example-01-cavity.prm
TLIM=300 run example-02-taylor-couette 2 example-02-taylor-couette.prm
TLIM=300 run taylor-couette3d 3 taylor-couette3d_q2q1.prm
TLIM=300 run cavity3d-q1-64 3 cavity3d_q1_64_steady.prm
TLIM=400 run cylinder3d-re200 3 cylinder3d_q2q1_re200.prm
TLIM=600 run cavity3d-q2-128-bdf2 3 cavity3d_q2_128_bdf2.prm
echo done >> $O/summary.txt
# the reference's TGV SDIRK2 / SDIRK3 application tests as shipped (inexact Newton: tol 1e-6, GMRES rel 1e-4)
cp $R/tests/golden/app_cases/taylor-green-vortex_gls_sdirk*.prm $O/
sed -i 's/set output frequency *= *1 /set output frequency = 1000000 /' $O/taylor-green-vortex_gls_sdirk*.prm
TLIM=300 run tgv-sdirk2 2 taylor-green-vortex_gls_sdirk2.prm --precision 9
TLIM=300 run tgv-sdirk3 2 taylor-green-vortex_gls_sdirk3.prm --precision 9
echo done2 >> $O/summary.txt
rm -f $O/*.msh

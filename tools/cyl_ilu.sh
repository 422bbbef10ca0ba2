#!/bin/bash
# cylinder_gls through the 2D app with the default preconditioner (ILU(0) on the hanging-condensed
# operator) and with --precond jacobi: wall time and counts per cycle
set -e
out=${1:-gpurun_out/cyl_ilu}
mkdir -p $out
cp tests/golden/meshes/cylinder_structured.msh $out/
sed 's#\.\./cylinder_structured.msh#cylinder_structured.msh#' tests/golden/app_cases/cylinder_gls.prm | sed 's/set type    = none /set type = iteration /' > $out/case.prm
cd $out
timeout -k 10 200 stdbuf -oL ../../apps/gls_navier_stokes_2d --stats case.prm > ilu.log 2>&1 || echo "ILU run exit $?"
timeout -k 10 200 stdbuf -oL ../../apps/gls_navier_stokes_2d --stats --precond jacobi case.prm > jacobi.log 2>&1 || echo "Jacobi run exit $?"

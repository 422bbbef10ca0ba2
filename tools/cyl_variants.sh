#!/bin/bash
# cylinder_gls (applications_tests/gls_navier_stokes_2d) through the 2D app with the shipped settings
# and with tight solver tolerances: cell / DoF counts and Kelly flag counts per adaptation cycle
set -e
out=${1:-gpurun_out/cyl}
mkdir -p $out
cp tests/golden/meshes/cylinder_structured.msh $out/
sed 's#\.\./cylinder_structured.msh#cylinder_structured.msh#' tests/golden/app_cases/cylinder_gls.prm > $out/shipped.prm
sed -e 's/set tolerance               = 1e-4/set tolerance = 1e-10/' -e 's/set relative residual       = 1e-4/set relative residual = 1e-12/' \
    -e 's/set minimum residual        = 1e-9/set minimum residual = 1e-14/' $out/shipped.prm > $out/tight.prm
cd $out
for v in shipped tight; do
  timeout -k 10 300 ../../apps/gls_navier_stokes_2d --stats $v.prm > $v.log 2>&1
  echo "== $v"; grep -E "Number of active|degrees|kelly:|newton_iter" $v.log
done

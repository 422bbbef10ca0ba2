#!/bin/bash
# slip on a curved wall (hyper_shell rigid rotation) through the 2D app: ILU and Jacobi, verbose Newton
set -e
out=${1:-gpurun_out/slipdbg}; mkdir -p $out; cp tools/shell_rotation.prm $out/case.prm; cd $out
timeout -k 5 60 stdbuf -oL ../../apps/gls_navier_stokes_2d --stats case.prm > ilu.log 2>&1 || echo "ilu exit $?"
timeout -k 5 60 stdbuf -oL ../../apps/gls_navier_stokes_2d --stats --precond jacobi case.prm > jac.log 2>&1 || echo "jacobi exit $?"

# configs[4]-style cylinder (1 step) with block-Jacobi ILU subdomain sizes
set -o pipefail
mkdir -p gpurun_out/apps
W=$(mktemp -d)
cp apps/cases/cylinder3d_extruded.msh $W/
sed -e "s|set time end *= *[0-9.e-]*|set time end = 0.05|" apps/cases/cylinder3d_q2q1_re200.prm > $W/case.prm
for B in "$@"; do
  ( cd $W && GLS_ILU_VERBOSE=1 timeout -k 10 300 $OLDPWD/apps/gls_navier_stokes_3d --stats --ilu-order ${B%%:*} --ilu-block-dofs ${B#*:} case.prm ) > gpurun_out/apps/cyl_${B%%:*}_${B#*:}.log 2>&1 || exit 1
done

# configs[4]-style cylinder (3D Q2-Q1, Re 200, BDF2) for N steps through the app with ILU timing
set -o pipefail
mkdir -p gpurun_out/apps
W=$(mktemp -d)
cp apps/cases/cylinder3d_extruded.msh $W/
sed -e "s|set time end *= *[0-9.e-]*|set time end = $1|" apps/cases/${2:-cylinder3d_q2q1_re200}.prm > $W/case.prm
( cd $W && GLS_ILU_VERBOSE=1 timeout -k 10 ${3:-300} $OLDPWD/apps/gls_navier_stokes_3d --stats case.prm ) > gpurun_out/apps/${2:-cylinder3d_q2q1_re200}_$1.log 2>&1

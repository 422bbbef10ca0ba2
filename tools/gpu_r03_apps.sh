# run the reference's cylinder_gls and TGV sdirk cases through the drop-in app, stdout to gpurun_out/
set -o pipefail
mkdir -p gpurun_out/apps
W=$(mktemp -d)
cp tests/golden/meshes/* $W/
for c in "$@"; do
  sed -e 's|\(set file name *= *\)\.\./|\1|' -e 's|set output frequency *= *1 |set output frequency = 1000000 |' tests/golden/app_cases/$c.prm > $W/$c.prm
  dim=2; case $c in *3d*|cylinder-rigid*) dim=3;; esac
  ( cd $W && timeout -k 10 600 $OLDPWD/apps/gls_navier_stokes_${dim}d --stats $c.prm ) > gpurun_out/apps/$c.log 2>&1 || { echo "$c failed rc $?"; exit 1; }
  echo "$c done"
done

# round-5 box R: configs[3] through the app with --precond hmg: the levels' ILU(0) smoothers in Cuthill-McKee
# order (default below 1e5 DoFs) vs the multicolor order (GLS_MG_ILU_MC_MIN=0); --precond mg (ILU) for scale
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/c3
cp apps/cases/taylor-couette3d_q2q1_kelly.prm /tmp/c3/case.prm
: > gpurun_out/r05r_app.txt
for cfg in "X=1:hmg" "GLS_MG_ILU_MC_MIN=0:hmg" "X=1:mg" "X=1:hmg" "GLS_MG_ILU_MC_MIN=0:hmg"; do
  e="${cfg%%:*}"; pc="${cfg##*:}"
  s=$(date +%s.%N)
  ( cd /tmp/c3 && env $e timeout -k 10 300 $GRAFT_REPO_ROOT/apps/gls_navier_stokes_3d --precond $pc --stats case.prm > out.txt 2> err.txt )
  rc=$?; t=$(date +%s.%N)
  echo "$e --precond $pc rc $rc wall $(python3 -c "print(round($t-$s,2))") s $(grep -a 'linear_iterations' /tmp/c3/out.txt | tail -1) solve_linear_system $(grep -a 'solve_linear_system' /tmp/c3/out.txt | awk -F'|' '{print $4}' | tr -d ' ' | tr '\n' ' ')" >> gpurun_out/r05r_app.txt
  [ $rc -ne 0 ] && { tail -5 /tmp/c3/err.txt; cat gpurun_out/r05r_app.txt; exit $rc; }
  grep -aq "kelly" /tmp/c3/out.txt && cp /tmp/c3/out.txt "gpurun_out/r05r_out_${pc}_$(echo $e | tr '=' '_').txt"
done
cat gpurun_out/r05r_app.txt

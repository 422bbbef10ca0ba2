# round-3 debug: the app's --np residual against a whole-mesh context (GLS_NP_CHECK) on configs[3]
mkdir -p gpurun_out/npc && cp apps/cases/taylor-couette3d_q2q1_kelly.prm gpurun_out/npc/case.prm && cd gpurun_out/npc || exit 1
GLS_NP_CHECK=1 GLS_NP_WATCHDOG=30 timeout -k 5 100 ../../apps/gls_navier_stokes_3d --np 4 case.prm > out.txt 2> err.txt
echo "rc $?"; rm -f *.vtu

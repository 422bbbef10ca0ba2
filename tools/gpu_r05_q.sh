# round-5 box Q: the direct coarse solve's matrix by colored batched probes on per-cell levels -- MG tests, then
# configs[3] through the app with --precond hmg, probe loop (before) vs colored probes (after)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_umesh_mg.py tests/test_gpu_octree_mg.py tests/test_gpu_dist_mg.py tests/test_gpu_app_configs.py tests/test_gpu_solver.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05q_tests.log 2>&1
rc=$?; echo "tests rc $rc"; tail -2 gpurun_out/r05q_tests.log; [ $rc -ne 0 ] && exit $rc
mkdir -p /tmp/c3 && cp apps/cases/taylor-couette3d_q2q1_kelly.prm /tmp/c3/case.prm
for v in 1 0 1 0; do
  s=$(date +%s.%N)
  ( cd /tmp/c3 && env $( [ $v = 1 ] && echo GLS_MG_PROBE_LOOP=1 ) timeout -k 10 300 $GRAFT_REPO_ROOT/apps/gls_navier_stokes_3d --precond hmg --stats case.prm > out_$v.txt 2> err_$v.txt )
  rc=$?; e=$(date +%s.%N)
  echo "probe_loop=$v rc $rc wall $(python3 -c "print(round($e-$s,2))") s $(grep -a 'linear_iterations' /tmp/c3/out_$v.txt | tail -1)"; [ $rc -ne 0 ] && { tail -5 /tmp/c3/err_$v.txt; exit $rc; }
done
cp /tmp/c3/out_0.txt gpurun_out/r05q_app_c3_hmg.txt
exit 0

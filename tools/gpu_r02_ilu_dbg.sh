# ILU tests + diagnostics on the reference's Taylor-Couette example (hyper_shell, Q2-Q1, MappingQ2)
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_ilu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ilu_tests.log 2>&1 || exit 1
O=gpurun_out/ilu_dbg; mkdir -p $O; cp tests/golden/app_cases/example-02-taylor-couette.prm $O/
cd $O && GLS_ILU_VERBOSE=1 timeout -k 10 120 ../../apps/gls_navier_stokes_2d example-02-taylor-couette.prm > tc.log 2>&1; echo "rc=$?" >> tc.log; rm -f *.vtu *.pvtu *.pvd

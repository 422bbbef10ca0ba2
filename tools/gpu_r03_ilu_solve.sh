# ILU multicolor triangular solves: GPU ILU tests, then the configs[4] problem (cylinder3d) app + bench
#  + kernel stats
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ilu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/ilu_tests.log 2>&1 || exit 1
(cd apps/cases && GLS_ILU_VERBOSE=1 timeout -k 10 300 ../gls_navier_stokes_3d cylinder3d_q2q1_re200.prm > ../../gpurun_out/app_cyl3d.log 2>&1) || exit 1
for W in 1; do
  timeout -k 10 200 python3 bench.py --workload cylinder3d --steps 5 --warmup 1 > gpurun_out/bench_cyl3d_w$W.json 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cyl3d -o run --output-format csv -- python3 bench.py --workload cylinder3d --steps 3 --warmup 1 > gpurun_out/bench_cyl3d_prof.json 2> gpurun_out/bench_cyl3d_prof.err || exit 1

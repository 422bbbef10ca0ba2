# A/B of the multicolor ILU coloring order (Cuthill-McKee greedy vs smallest-last) on the configs[4] problem
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in cm sl; do
  (cd apps/cases && GLS_ILU_COLORING=$C GLS_ILU_VERBOSE=1 timeout -k 10 300 ../gls_navier_stokes_3d cylinder3d_q2q1_re200.prm > ../../gpurun_out/app_cyl3d_$C.log 2>&1) || exit 1
  GLS_ILU_COLORING=$C timeout -k 10 200 python3 bench.py --workload cylinder3d --steps 5 --warmup 1 > gpurun_out/bench_cyl3d_$C.json 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cyl3d -o run --output-format csv -- python3 bench.py --workload cylinder3d --steps 3 --warmup 1 > gpurun_out/bench_cyl3d_prof.json 2> gpurun_out/bench_cyl3d_prof.err || exit 1

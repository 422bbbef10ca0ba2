# round-4 evidence, part 2: the configs[2] bench line under rocprofv3 kernel-trace stats and plain, PMC traffic
# of the pencil J.v, cylinder3d and octree lines. Usage: bash tools/gpu_r04_final_bench.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-r04g}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_bench_$T.json 2> gpurun_out/prof_bench_$T.err || { echo PROF_FAIL; exit 1; }
bash tools/pmc_traffic.sh 128 gpurun_out/pmc_traffic_$T > gpurun_out/pmc_traffic_$T.txt 2>&1 || { echo TRAFFIC_FAIL; exit 1; }
timeout -k 10 300 python3 bench.py --workload cylinder3d --steps 10 --warmup 2 > gpurun_out/bench_cyl_$T.json 2> gpurun_out/bench_cyl_$T.err || { echo CYL_FAIL; exit 1; }
timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 > gpurun_out/bench_oct_$T.json 2> gpurun_out/bench_oct_$T.err || { echo OCT_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_oct_$T -o run --output-format csv -- \
    python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 > gpurun_out/prof_oct_$T.json 2> gpurun_out/prof_oct_$T.err || { echo OCTPROF_FAIL; exit 1; }
# configs[3]'s app pipeline (taylor-couette 3D Q2-Q1, 2 Kelly cycles): the reference's ILU vs the hierarchy multigrid
mkdir -p gpurun_out/tc_$T && cp apps/cases/taylor-couette3d_q2q1_kelly.prm gpurun_out/tc_$T/case.prm
for pc in mg hmg; do
  ( cd gpurun_out/tc_$T && s0=$(date +%s%N) && timeout -k 10 300 ../../apps/gls_navier_stokes_3d --stats --precond $pc case.prm > app_$pc.out 2> app_$pc.err \
    && s1=$(date +%s%N) && echo "precond $pc wall $(( (s1 - s0) / 1000000 )) ms; $(grep linear_iterations app_$pc.out)" >> ../tc_$T.txt ) || { echo TC_FAIL; exit 1; }
done
cat gpurun_out/tc_$T.txt
cut -c1-400 gpurun_out/bench_$T.json; cut -c1-300 gpurun_out/bench_cyl_$T.json; cut -c1-300 gpurun_out/bench_oct_$T.json
echo ALL_OK

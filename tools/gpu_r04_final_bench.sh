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
cut -c1-400 gpurun_out/bench_$T.json; cut -c1-300 gpurun_out/bench_cyl_$T.json; cut -c1-300 gpurun_out/bench_oct_$T.json
echo ALL_OK

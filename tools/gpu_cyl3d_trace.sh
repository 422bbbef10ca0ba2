set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cyl -o run --output-format csv -- python3 bench.py --workload cylinder3d --steps 3 --warmup 1 > gpurun_out/bench_cyl_prof.json 2> gpurun_out/bench_cyl_prof.err
rc=$?; echo "rc $rc"; exit $rc

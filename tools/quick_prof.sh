# quick GPU check: selected GPU tests, bench line, kernel trace (gpurun_out/prof2)
set -o pipefail
export TMPDIR=/tmp
T=${1:-tests/test_gpu_solver.py}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $T -m gpu > gpurun_out/t.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 200 python3 bench.py --steps 3 --no-cpu > gpurun_out/b.json 2>gpurun_out/b.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/bp.json 2>gpurun_out/bp.err || { echo PROF_FAIL; exit 1; }
echo OK

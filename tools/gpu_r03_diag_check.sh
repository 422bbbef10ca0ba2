# diagonal-loop restructure: parity / full-size / solver GPU tests, then the bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_diag.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -2 gpurun_out/gpu_tests_diag.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 bench.py --no-cpu --steps 6 --warmup 2 > gpurun_out/bench_diag.json 2> gpurun_out/bench_diag.err
rc=$?; echo "bench rc $rc"; exit $rc

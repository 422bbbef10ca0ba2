# round-4 check on one MI355X: the fused residual + linearization pass, the fused first Jacobi sweep
# (bitwise tests), pencil parity, periodic adaptive meshes (operator vs oracle, app), then the bench line.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_solver.py tests/test_hanging.py tests/test_gpu_app.py -k "fused or pencil or multigrid or gmres or periodic" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fuse_tests.log 2>&1
rc=$?; echo "tests rc $rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/fuse_tests.log | tail -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-cpu > gpurun_out/bench_fuse.json 2> gpurun_out/bench_fuse.err || { echo BENCH_FAIL; tail -5 gpurun_out/bench_fuse.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_fuse.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['linear_iterations_per_step'], d['kernel_ms'])"

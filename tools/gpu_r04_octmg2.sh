# octree multigrid: GPU tests (3D Q1/Q2/Q2-Q1, 2D), the app tests, then the octree bench with the vector SpMV
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  tests/test_gpu_octree_mg.py > gpurun_out/octmg2_tests.log 2>&1 || { tail -40 gpurun_out/octmg2_tests.log; exit 1; }
grep -E "PASSED|FAILED|octree GMG" gpurun_out/octmg2_tests.log
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -s \
  tests/test_gpu_app.py tests/test_gpu_app_reference.py > gpurun_out/octmg2_app.log 2>&1 || { tail -40 gpurun_out/octmg2_app.log; exit 1; }
grep -E "forest GMG|passed|failed" gpurun_out/octmg2_app.log
timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 > gpurun_out/oct3_mg4s4.json 2> gpurun_out/oct3_mg4s4.err || exit 1
timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 3 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 > gpurun_out/oct3_mg4s3.json 2> gpurun_out/oct3_mg4s3.err || exit 1
cut -c1-420 gpurun_out/oct3_mg4s4.json gpurun_out/oct3_mg4s3.json

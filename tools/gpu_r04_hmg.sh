# hierarchy multigrid on adapted general meshes: octree tests (incl. 2D / Q2-Q1), the umesh linear-solve
# tests, the app tests (octree default, configs[3] with --precond hmg), then the octree bench with the vector SpMV
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s \
  ${HMG_TESTS:-tests/test_gpu_octree_mg.py tests/test_gpu_umesh_mg.py} > gpurun_out/hmg_tests.log 2>&1 || { tail -40 gpurun_out/hmg_tests.log; exit 1; }
grep -E "PASSED|FAILED|GMG" gpurun_out/hmg_tests.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -s \
  tests/test_gpu_app_configs.py tests/test_gpu_app.py -k "hierarchy or forest or configs3" > gpurun_out/hmg_app.log 2>&1 || { tail -40 gpurun_out/hmg_app.log; exit 1; }
grep -E "PASSED|FAILED|GMRES totals|forest GMG" gpurun_out/hmg_app.log
timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 > gpurun_out/oct3_mg4s4.json 2> gpurun_out/oct3_mg4s4.err || exit 1
cut -c1-300 gpurun_out/oct3_mg4s4.json

# forest bricks: the parity test, the hanging / octree multigrid regressions, the octree bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu -s tests/test_gpu_forest_bricks.py \
  > gpurun_out/fb_tests.log 2>&1 || { tail -40 gpurun_out/fb_tests.log; exit 1; }
grep -E "PASSED|FAILED|forest bricks" gpurun_out/fb_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hanging.py \
  tests/test_gpu_octree_mg.py tests/test_gpu_parity.py tests/test_gpu_uforest.py tests/test_gpu_mapped.py > gpurun_out/fb_regress.log 2>&1 || { tail -40 gpurun_out/fb_regress.log; exit 1; }
tail -2 gpurun_out/fb_regress.log
timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 > gpurun_out/fb_oct.json 2> gpurun_out/fb_oct.err || { tail -5 gpurun_out/fb_oct.err; exit 1; }
cut -c1-300 gpurun_out/fb_oct.json
python3 -c "
import json; d=json.loads(open('gpurun_out/fb_oct.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['linear_iterations_per_step'], d['roofline']['launch_ms'])"

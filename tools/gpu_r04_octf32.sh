# FP32 forest-brick smoothing: tests, octree lines FP64 vs mixed, the configs[2] line (the FP32 cube kernel unchanged)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -s tests/test_gpu_octree_mg.py \
  tests/test_gpu_forest_bricks.py > gpurun_out/of32_tests.log 2>&1 || { tail -40 gpurun_out/of32_tests.log; exit 1; }
grep -E "FAILED|mixed|passed" gpurun_out/of32_tests.log
O=gpurun_out/of32.log; rm -f $O
for pr in f64 f32 f64 f32; do
  timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 --mg-precision $pr > gpurun_out/of32_$pr.json 2> gpurun_out/of32_$pr.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('octree %s ms/step %7.2f its %4.1f it/s %6.2f' % (sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'], d['value']))" gpurun_out/of32_$pr.json $pr >> $O
done
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --no-cpu > gpurun_out/of32_cube$r.json 2> gpurun_out/of32_cube$r.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('cube ms/step %7.2f its %4.1f' % (d['ms_per_step'], d['linear_iterations_per_step']))" gpurun_out/of32_cube$r.json >> $O
done
cat $O

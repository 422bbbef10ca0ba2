# last evidence call of round 4: full -m gpu suite + smoke, octree FP64 vs mixed-precision smoothing, configs[2] line
set -o pipefail
export TMPDIR=/tmp
T=r04j
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/gpu_tests_$T.log; [ $rc -ne 0 ] && exit $rc
grep -E "octree GMG FP64 / mixed" gpurun_out/gpu_tests_$T.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
O=gpurun_out/last_$T.log; rm -f $O
for pr in f64 f32; do
  timeout -k 10 300 python3 bench.py --workload octree --cells 4 --octree-steps 4 --steps 5 --warmup 1 --mg-smooth 2 2 --mg-omega 0.6 --mg-precision $pr > gpurun_out/oct_${pr}_$T.json 2> gpurun_out/oct_${pr}_$T.err || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('octree %s ms/step %7.2f its %4.1f it/s %6.2f' % (sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'], d['value']))" gpurun_out/oct_${pr}_$T.json $pr >> $O
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_$T.json').read().strip().splitlines()[-1])
print('cube ms/step %7.2f its %4.1f it/s %6.2f' % (d['ms_per_step'], d['linear_iterations_per_step'], d['value']))" >> $O
cat $O
echo ALL_OK

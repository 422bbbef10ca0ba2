# round-5 box L: full -m gpu suite with the per-cell linearization cache and the folded condensation, then
# A/B of both on the octree and cylinder3d lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r05l_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc $rc"; tail -3 gpurun_out/r05l_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/r05l_ab.txt
for w in octree cylinder3d; do
  for cfg in "GLS_CELL_CACHE=0 GLS_NO_COND_FOLD=1" "GLS_CELL_CACHE=0" "GLS_CELL_CACHE=1" "GLS_CELL_CACHE=0 GLS_NO_COND_FOLD=1" "GLS_CELL_CACHE=1"; do
    env $cfg timeout -k 10 300 python3 bench.py --workload $w --no-pmc --no-cpu > gpurun_out/r05l_tmp.json 2> gpurun_out/r05l_tmp.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench $w $cfg rc $rc"; tail -5 gpurun_out/r05l_tmp.err; exit $rc; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/r05l_tmp.json').read().strip().splitlines()[-1]);print('%-12s %-40s %8.3f ms  its %.1f  %.2f it/s' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['linear_iterations_per_step'], d['value']))" $w "$cfg" >> gpurun_out/r05l_ab.txt
  done
done
cat gpurun_out/r05l_ab.txt

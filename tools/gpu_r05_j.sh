# round-5 box J: V-cycle parameter sweep at configs[2] (GMRES iterations vs ms per Newton step)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.log; sleep 30; done ) &
HB=$!
trap "kill $HB" EXIT
: > gpurun_out/r05j_sweep.txt
run() {
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu --steps 6 --warmup 1 "$@" > gpurun_out/r05j_tmp.json 2> gpurun_out/r05j_tmp.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc $rc for $*" >> gpurun_out/r05j_sweep.txt; tail -5 gpurun_out/r05j_tmp.err >> gpurun_out/r05j_sweep.txt; return $rc; fi
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r05j_tmp.json').read().strip().splitlines()[-1]);print('%-60s %8.2f ms  its %.1f' % (' '.join(sys.argv[1:]), d['ms_per_step'], d['linear_iterations_per_step']))" "$@" >> gpurun_out/r05j_sweep.txt
}
run --mg-smooth 2 2 --mg-fine-sweeps 1 1 && run --mg-smooth 3 3 --mg-fine-sweeps 1 1 && run --mg-smooth 2 2 --mg-fine-sweeps 1 2 \
  && run --mg-smooth 2 2 --mg-fine-sweeps 2 1 && run --mg-smooth 3 3 --mg-fine-sweeps 1 2 && run --mg-smooth 2 2 --mg-omega 1.0 \
  && run --mg-fine-sweeps 1 2 --mg-omega 1.0 && run --mg-smooth 2 2 --mg-fine-sweeps 1 1 --mg-omega 1.0 \
  && run --mg-smooth 4 4 --mg-fine-sweeps 1 1 && run --mg-smooth 2 2 --mg-fine-sweeps 1 2 --mg-coarse-level-sweeps 3 && run --mg-smooth 2 2
rc=$?; cat gpurun_out/r05j_sweep.txt; exit $rc
